// PyTorch bindings of the implicit-GEMM convolutions (p2pfl_amd._C.conv_*).
// Every shape / layout / alignment assumption of csrc/conv.hip is checked here
// before the launch, so a bad call is a Python exception, never a GPU fault.
#include <torch/extension.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>

#include "conv.h"

namespace {

void check_nhwc(const torch::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == torch::kBFloat16, name, " must be a bf16 GPU tensor");
  TORCH_CHECK(t.dim() == 4 && t.is_contiguous(), name, " must be a contiguous 4-D (NHWC / OHWC) tensor");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name, " must be 16-byte aligned");
}

int out_size(int in, int k, int stride, int pad, int dil) { return (in + 2 * pad - dil * (k - 1) - 1) / stride + 1; }

p2::ConvShape make_shape(int64_t N, int64_t H, int64_t W, int64_t C, int64_t O, int64_t kh, int64_t kw, int64_t stride,
                         int64_t pad, int64_t dil) {
  TORCH_CHECK(stride >= 1 && stride <= 2 && pad >= 0 && dil >= 1, "conv: stride 1/2, pad >= 0, dilation >= 1");
  TORCH_CHECK(N * H * W < (int64_t(1) << 31) && kh * kw * std::max(C, O) < (int64_t(1) << 31), "conv: size overflow");
  p2::ConvShape s{};
  s.N = int(N);
  s.H = int(H);
  s.W = int(W);
  s.C = int(C);
  s.O = int(O);
  s.kh = int(kh);
  s.kw = int(kw);
  s.stride = int(stride);
  s.pad = int(pad);
  s.dil = int(dil);
  s.OH = out_size(s.H, s.kh, s.stride, s.pad, s.dil);
  s.OW = out_size(s.W, s.kw, s.stride, s.pad, s.dil);
  TORCH_CHECK(s.OH >= 1 && s.OW >= 1, "conv: empty output");
  return s;
}

hipStream_t stream_of(const torch::Tensor& t) { return c10::hip::getCurrentHIPStream(t.device().index()).stream(); }

// fp32 elements of one split-K slice: fragment-native 128 x 128 tiles (gemm_core.h SlabGeom)
int64_t slab_elems(int64_t rows, int64_t cols) { return ((rows + 127) / 128) * ((cols + 127) / 128) * 128 * 128; }

// Split-K configuration: without `counters`, splits > 1 writes fp32 slabs to the output
// tensor itself (reduce with tile_slab_reduce); with `counters` (int32, one per output
// tile of the launch's tile shape, all zero) the slabs go to `ws` (fp32, splits *
// slab_elems) and the launch reduces them itself.
p2::SplitK make_splitk(int64_t splits, const c10::optional<torch::Tensor>& ws, const c10::optional<torch::Tensor>& counters,
                       int64_t rows, int64_t cols, const torch::Tensor& like, const char* who, int64_t variant) {
  TORCH_CHECK(splits >= 1 && splits <= 128, who, ": 1 <= splits <= 128");
  // in-launch counters: one per output tile of the launch's tile shape (64 x 64 with
  // conv.hip kConvT64, else 128 x 128)
  const int64_t ts = (variant & p2::kConvT64) ? 64 : 128;
  p2::SplitK k;
  k.splits = int(splits);
  const bool have_cnt = counters.has_value() && counters->defined();
  if (have_cnt) {
    TORCH_CHECK(splits > 1, who, ": counters only with splits > 1");
    const int64_t tiles = ((rows + ts - 1) / ts) * ((cols + ts - 1) / ts);
    TORCH_CHECK(counters->is_cuda() && counters->scalar_type() == torch::kInt32 && counters->is_contiguous() &&
                    counters->numel() >= tiles && counters->device() == like.device(),
                who, ": counters must be a contiguous int32 GPU tensor with >= ", tiles, " entries");
    TORCH_CHECK(ws.has_value() && ws->defined(), who, ": counters need a workspace");
    TORCH_CHECK(ws->is_cuda() && ws->scalar_type() == torch::kFloat32 && ws->is_contiguous() &&
                    ws->numel() >= splits * slab_elems(rows, cols) && reinterpret_cast<uintptr_t>(ws->data_ptr()) % 16 == 0 &&
                    ws->device() == like.device(),
                who, ": workspace must be contiguous fp32 with splits * slab_elems(rows, cols) elements");
    k.counters = counters->data_ptr<int>();
    k.ws = ws->data_ptr<float>();
  }
  return k;
}

// The output of conv_fwd / conv_dgrad: bf16 NHWC [n, h, w, c], or raw fp32 slabs
// (contiguous, splits * n*h*w*c elements) for a split-K launch without counters.
void check_out(const torch::Tensor& out, const p2::SplitK& k, int n, int h, int w, int c, const char* who) {
  if (k.splits == 1 || k.counters) {
    check_nhwc(out, "out");
    TORCH_CHECK(out.size(0) == n && out.size(1) == h && out.size(2) == w && out.size(3) == c, who, ": out shape");
  } else {
    TORCH_CHECK(out.is_cuda() && out.scalar_type() == torch::kFloat32 && out.is_contiguous() &&
                    out.numel() >= int64_t(k.splits) * slab_elems(int64_t(n) * h * w, c) &&
                    reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0,
                who, ": split-K out must be contiguous fp32 with splits * slab_elems(rows, cols) elements");
  }
}

using OptT = c10::optional<torch::Tensor>;

// x [N, H, W, C], w [O, kh, kw, C]  ->  y [N, OH, OW, O]
void conv_fwd(torch::Tensor x, torch::Tensor w, int64_t stride, int64_t pad, int64_t dil, torch::Tensor y,
              int64_t splits, int64_t variant, OptT ws, OptT counters) {
  check_nhwc(x, "x");
  check_nhwc(w, "w");
  TORCH_CHECK(w.size(3) == x.size(3), "conv_fwd: channel mismatch");
  const auto s = make_shape(x.size(0), x.size(1), x.size(2), x.size(3), w.size(0), w.size(1), w.size(2), stride, pad, dil);
  TORCH_CHECK(s.C % 64 == 0 && s.O % 8 == 0, "conv_fwd: needs C % 64 == 0 and O % 8 == 0 (C=", s.C, " O=", s.O, ")");
  const auto k = make_splitk(splits, ws, counters, int64_t(s.N) * s.OH * s.OW, s.O, x, "conv_fwd", variant);
  check_out(y, k, s.N, s.OH, s.OW, s.O, "conv_fwd");
  TORCH_CHECK(x.device() == w.device() && y.device() == x.device(), "conv_fwd: device mismatch");
  const c10::DeviceGuard g(x.device());
  p2::conv_fwd(s, reinterpret_cast<const uint16_t*>(x.data_ptr()), reinterpret_cast<const uint16_t*>(w.data_ptr()),
               y.data_ptr(), k, int(variant), stream_of(x));
}

int bn_groups(int64_t tiles_m) { return int((tiles_m + 15) / 16); }

// conv_fwd + BatchNorm training statistics in the launch (gemm.h BnEpi): part is fp32
// (tiles_m + groups) * 2 * O, cnt int32 tiles_n * (groups + 1) zeroed; mean / rstd [O]
// and coef [3, O] out; running_mean / running_var / nbt updated when given.
void conv_fwd_bn(torch::Tensor x, torch::Tensor w, int64_t stride, int64_t pad, int64_t dil, torch::Tensor y,
                 int64_t splits, int64_t variant, OptT ws, OptT counters, torch::Tensor part, torch::Tensor cnt,
                 torch::Tensor bn_w, torch::Tensor bn_b, OptT run_mean, OptT run_var, OptT nbt, torch::Tensor mean,
                 torch::Tensor rstd, torch::Tensor coef, double eps, double momentum) {
  check_nhwc(x, "x");
  check_nhwc(w, "w");
  TORCH_CHECK(w.size(3) == x.size(3), "conv_fwd_bn: channel mismatch");
  const auto s = make_shape(x.size(0), x.size(1), x.size(2), x.size(3), w.size(0), w.size(1), w.size(2), stride, pad, dil);
  TORCH_CHECK(s.C % 64 == 0 && s.O % 8 == 0, "conv_fwd_bn: needs C % 64 == 0 and O % 8 == 0");
  const int64_t M = int64_t(s.N) * s.OH * s.OW;
  const auto k = make_splitk(splits, ws, counters, M, s.O, x, "conv_fwd_bn", variant);
  TORCH_CHECK(!(variant & p2::kConvT64), "conv_fwd_bn: the BatchNorm-statistics epilogue runs on 128x128 tiles only");
  TORCH_CHECK(k.splits == 1 || k.counters, "conv_fwd_bn: split-K needs the in-launch reduction (counters)");
  check_out(y, k, s.N, s.OH, s.OW, s.O, "conv_fwd_bn");
  const int64_t tiles_m = (M + 127) / 128, tiles_n = (s.O + 127) / 128, groups = bn_groups(tiles_m);
  auto f32v = [&](const torch::Tensor& t, int64_t n, const char* name) {
    TORCH_CHECK(t.is_cuda() && t.device() == x.device() && t.scalar_type() == torch::kFloat32 && t.is_contiguous() &&
                    t.numel() == n,
                "conv_fwd_bn: ", name, " must be a contiguous fp32 tensor of ", n, " elements on x's device");
    return t.data_ptr<float>();
  };
  p2::BnEpi e{};
  TORCH_CHECK(part.is_cuda() && part.device() == x.device() && part.scalar_type() == torch::kFloat32 &&
                  part.is_contiguous() && part.numel() >= (tiles_m + groups) * 2 * s.O,
              "conv_fwd_bn: part must hold (tiles_m + groups) * 2 * O fp32");
  TORCH_CHECK(cnt.is_cuda() && cnt.device() == x.device() && cnt.scalar_type() == torch::kInt32 && cnt.is_contiguous() &&
                  cnt.numel() >= tiles_n * (groups + 1),
              "conv_fwd_bn: cnt must hold tiles_n * (groups + 1) zeroed int32");
  e.part = part.data_ptr<float>();
  e.cnt = cnt.data_ptr<int>();
  e.w = f32v(bn_w, s.O, "bn weight");
  e.b = f32v(bn_b, s.O, "bn bias");
  const bool track = run_mean.has_value() && run_mean->defined();
  TORCH_CHECK(track == (run_var.has_value() && run_var->defined()), "conv_fwd_bn: running_mean and running_var go together");
  if (track) {
    e.run_mean = f32v(*run_mean, s.O, "running_mean");
    e.run_var = f32v(*run_var, s.O, "running_var");
  }
  if (nbt.has_value() && nbt->defined()) {
    TORCH_CHECK(nbt->device() == x.device() && nbt->scalar_type() == torch::kInt64 && nbt->numel() == 1,
                "conv_fwd_bn: num_batches_tracked must be an int64 scalar on x's device");
    e.nbt = nbt->data_ptr<int64_t>();
  }
  e.mean = f32v(mean, s.O, "mean");
  e.rstd = f32v(rstd, s.O, "rstd");
  e.coef = f32v(coef, 3 * s.O, "coef");
  e.eps = float(eps);
  e.momentum = float(momentum);
  TORCH_CHECK(x.device() == w.device() && y.device() == x.device(), "conv_fwd_bn: device mismatch");
  const c10::DeviceGuard g(x.device());
  p2::conv_fwd(s, reinterpret_cast<const uint16_t*>(x.data_ptr()), reinterpret_cast<const uint16_t*>(w.data_ptr()),
               y.data_ptr(), k, int(variant), stream_of(x), &e);
}

// conv_dgrad + the backward statistics of the BatchNorm(+ReLU) that produced this
// convolution's input (gemm.h BnEpi backward mode): bx / by = that BN's input /
// output [N, H, W, C] bf16 (by undefined: no ReLU), bmean / brstd its saved
// statistics, bn_w its weight; dgamma / dbeta [C] and coef [3, C] out.
void conv_dgrad_bn(torch::Tensor dy, torch::Tensor w, int64_t stride, int64_t pad, int64_t dil, torch::Tensor dx,
                   std::vector<int64_t> dx_shape, int64_t splits, int64_t variant, OptT ws, OptT counters,
                   torch::Tensor part, torch::Tensor cnt, torch::Tensor bn_w, torch::Tensor bx, OptT by,
                   torch::Tensor bmean, torch::Tensor brstd, torch::Tensor dgamma, torch::Tensor dbeta,
                   torch::Tensor coef) {
  check_nhwc(dy, "dy");
  check_nhwc(w, "w");
  TORCH_CHECK(dx_shape.size() == 4, "conv_dgrad_bn: dx_shape is (N, H, W, C)");
  const auto s =
      make_shape(dx_shape[0], dx_shape[1], dx_shape[2], dx_shape[3], w.size(0), w.size(1), w.size(2), stride, pad, dil);
  TORCH_CHECK(w.size(3) == s.C, "conv_dgrad_bn: channel mismatch");
  TORCH_CHECK(s.O % 64 == 0 && s.C % 8 == 0, "conv_dgrad_bn: needs O % 64 == 0 and C % 8 == 0");
  TORCH_CHECK(dy.size(0) == s.N && dy.size(1) == s.OH && dy.size(2) == s.OW && dy.size(3) == s.O, "conv_dgrad_bn: dy shape");
  const int64_t M = int64_t(s.N) * s.H * s.W;
  const auto k = make_splitk(splits, ws, counters, M, s.C, dy, "conv_dgrad_bn", variant);
  TORCH_CHECK(!(variant & p2::kConvT64), "conv_dgrad_bn: the BatchNorm-statistics epilogue runs on 128x128 tiles only");
  TORCH_CHECK(k.splits == 1 || k.counters, "conv_dgrad_bn: split-K needs the in-launch reduction (counters)");
  check_out(dx, k, s.N, s.H, s.W, s.C, "conv_dgrad_bn");
  const int64_t tiles_m = (M + 127) / 128, tiles_n = (s.C + 127) / 128, groups = bn_groups(tiles_m);
  auto f32v = [&](const torch::Tensor& t, int64_t n, const char* name) {
    TORCH_CHECK(t.is_cuda() && t.device() == dy.device() && t.scalar_type() == torch::kFloat32 && t.is_contiguous() &&
                    t.numel() == n,
                "conv_dgrad_bn: ", name, " must be a contiguous fp32 tensor of ", n, " elements on dy's device");
    return t.data_ptr<float>();
  };
  auto act = [&](const torch::Tensor& t, const char* name) {
    check_nhwc(t, name);
    TORCH_CHECK(t.device() == dy.device() && t.size(0) == s.N && t.size(1) == s.H && t.size(2) == s.W && t.size(3) == s.C,
                "conv_dgrad_bn: ", name, " must be [N, H, W, C] like dx");
    return reinterpret_cast<const uint16_t*>(t.data_ptr());
  };
  TORCH_CHECK(part.is_cuda() && part.device() == dy.device() && part.scalar_type() == torch::kFloat32 &&
                  part.is_contiguous() && part.numel() >= (tiles_m + groups) * 2 * s.C,
              "conv_dgrad_bn: part must hold (tiles_m + groups) * 2 * C fp32");
  TORCH_CHECK(cnt.is_cuda() && cnt.device() == dy.device() && cnt.scalar_type() == torch::kInt32 && cnt.is_contiguous() &&
                  cnt.numel() >= tiles_n * (groups + 1),
              "conv_dgrad_bn: cnt must hold tiles_n * (groups + 1) zeroed int32");
  p2::BnEpi e{};
  e.part = part.data_ptr<float>();
  e.cnt = cnt.data_ptr<int>();
  e.w = f32v(bn_w, s.C, "bn weight");
  e.bx = act(bx, "bx");
  if (by.has_value() && by->defined()) e.by = act(*by, "by");
  e.bmean = f32v(bmean, s.C, "bmean");
  e.brstd = f32v(brstd, s.C, "brstd");
  e.dw = f32v(dgamma, s.C, "dgamma");
  e.db = f32v(dbeta, s.C, "dbeta");
  e.coef = f32v(coef, 3 * s.C, "coef");
  TORCH_CHECK(dy.device() == w.device() && dx.device() == dy.device(), "conv_dgrad_bn: device mismatch");
  const c10::DeviceGuard g(dy.device());
  p2::conv_dgrad(s, reinterpret_cast<const uint16_t*>(dy.data_ptr()), reinterpret_cast<const uint16_t*>(w.data_ptr()),
                 dx.data_ptr(), k, int(variant), stream_of(dy), &e);
}

// dy [N, OH, OW, O], w [O, kh, kw, C]  ->  dx [N, H, W, C]  (dx_shape = (N, H, W, C), dx may hold slabs)
void conv_dgrad(torch::Tensor dy, torch::Tensor w, int64_t stride, int64_t pad, int64_t dil, torch::Tensor dx,
                std::vector<int64_t> dx_shape, int64_t splits, int64_t variant, OptT ws, OptT counters) {
  check_nhwc(dy, "dy");
  check_nhwc(w, "w");
  TORCH_CHECK(dx_shape.size() == 4, "conv_dgrad: dx_shape is (N, H, W, C)");
  const auto s =
      make_shape(dx_shape[0], dx_shape[1], dx_shape[2], dx_shape[3], w.size(0), w.size(1), w.size(2), stride, pad, dil);
  TORCH_CHECK(w.size(3) == s.C, "conv_dgrad: channel mismatch");
  TORCH_CHECK(s.O % 64 == 0 && s.C % 8 == 0, "conv_dgrad: needs O % 64 == 0 and C % 8 == 0 (C=", s.C, " O=", s.O, ")");
  TORCH_CHECK(dy.size(0) == s.N && dy.size(1) == s.OH && dy.size(2) == s.OW && dy.size(3) == s.O, "conv_dgrad: dy shape");
  const auto k = make_splitk(splits, ws, counters, int64_t(s.N) * s.H * s.W, s.C, dy, "conv_dgrad", variant);
  check_out(dx, k, s.N, s.H, s.W, s.C, "conv_dgrad");
  TORCH_CHECK(dy.device() == w.device() && dx.device() == dy.device(), "conv_dgrad: device mismatch");
  const c10::DeviceGuard g(dy.device());
  p2::conv_dgrad(s, reinterpret_cast<const uint16_t*>(dy.data_ptr()), reinterpret_cast<const uint16_t*>(w.data_ptr()),
                 dx.data_ptr(), k, int(variant), stream_of(dy));
}

// stride-2 input gradient by output phase: dy [N, OH, OW, O], w [O, kh, kw, C] -> out:
// phase-major [4 N (H/2) (W/2), C] bf16 (or split-K slabs / a counter-reduced bf16 out),
// for phase_interleave to scatter into dX; dx_shape (N, H, W, C) must pass conv_dgrad_s2_ok
void conv_dgrad_s2(torch::Tensor dy, torch::Tensor w, int64_t pad, torch::Tensor out, std::vector<int64_t> dx_shape,
                   int64_t splits, int64_t variant, OptT ws, OptT counters) {
  check_nhwc(dy, "dy");
  check_nhwc(w, "w");
  TORCH_CHECK(dx_shape.size() == 4, "conv_dgrad_s2: dx_shape is (N, H, W, C)");
  const auto s = make_shape(dx_shape[0], dx_shape[1], dx_shape[2], dx_shape[3], w.size(0), w.size(1), w.size(2), 2, pad, 1);
  TORCH_CHECK(p2::conv_dgrad_s2_ok(s), "conv_dgrad_s2: needs even H, W and N H W / 4 % 128 == 0");
  TORCH_CHECK(w.size(3) == s.C && s.O % 64 == 0 && s.C % 8 == 0, "conv_dgrad_s2: needs O % 64 == 0 and C % 8 == 0");
  TORCH_CHECK(dy.size(0) == s.N && dy.size(1) == s.OH && dy.size(2) == s.OW && dy.size(3) == s.O, "conv_dgrad_s2: dy shape");
  const int64_t rows = int64_t(p2::s2_phases(s)) * s.N * (s.H / 2) * (s.W / 2);  // phases with taps x N (H/2) (W/2)
  const auto k = make_splitk(splits, ws, counters, rows, s.C, dy, "conv_dgrad_s2", variant);
  if (k.splits == 1 || k.counters) {
    TORCH_CHECK(out.is_cuda() && out.scalar_type() == torch::kBFloat16 && out.is_contiguous() && out.numel() == rows * s.C &&
                    reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0,
                "conv_dgrad_s2: out must be contiguous bf16 with s2_phases N (H/2) (W/2) C elements");
  } else {
    TORCH_CHECK(out.is_cuda() && out.scalar_type() == torch::kFloat32 && out.is_contiguous() &&
                    out.numel() >= int64_t(k.splits) * slab_elems(rows, s.C) && reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0,
                "conv_dgrad_s2: split-K out must be contiguous fp32 with splits * slab_elems(rows, C) elements");
  }
  TORCH_CHECK(dy.device() == w.device() && out.device() == dy.device(), "conv_dgrad_s2: device mismatch");
  const c10::DeviceGuard g(dy.device());
  p2::conv_dgrad_s2(s, reinterpret_cast<const uint16_t*>(dy.data_ptr()), reinterpret_cast<const uint16_t*>(w.data_ptr()),
                    out.data_ptr(), k, int(variant), stream_of(dy));
}

// phase-major [s2_phases N (H/2) (W/2), C] bf16 -> dX [N, H, W, C] (conv_dgrad_s2's output
// order for a kh x kw kernel; the phases without taps are written as zeros)
void phase_interleave(torch::Tensor src, torch::Tensor dx, int64_t pad, int64_t kh, int64_t kw) {
  check_nhwc(dx, "dx");
  TORCH_CHECK(kh >= 1 && kw >= 1 && dx.size(1) + 2 * pad >= kh && dx.size(2) + 2 * pad >= kw, "phase_interleave: kernel size");
  const auto s = make_shape(dx.size(0), dx.size(1), dx.size(2), dx.size(3), 64, kh, kw, 2, pad, 1);
  TORCH_CHECK(p2::conv_dgrad_s2_ok(s) && s.C % 8 == 0, "phase_interleave: needs even H, W, N H W / 4 % 128 == 0, C % 8 == 0");
  const int64_t rows = int64_t(p2::s2_phases(s)) * s.N * (s.H / 2) * (s.W / 2);
  TORCH_CHECK(src.is_cuda() && src.device() == dx.device() && src.scalar_type() == torch::kBFloat16 && src.is_contiguous() &&
                  src.numel() == rows * s.C && reinterpret_cast<uintptr_t>(src.data_ptr()) % 16 == 0,
              "phase_interleave: src must be contiguous bf16 with s2_phases N (H/2) (W/2) C elements");
  const c10::DeviceGuard g(dx.device());
  p2::phase_interleave(s, reinterpret_cast<const uint16_t*>(src.data_ptr()), reinterpret_cast<uint16_t*>(dx.data_ptr()),
                       stream_of(dx));
}

// dy [N, OH, OW, O], x [N, H, W, C]  ->  out: [O, kh, kw, C] bf16/fp32, or raw fp32 slabs
// [splits, O*kh*kw*C] for a split-K launch without counters
void conv_wgrad(torch::Tensor dy, torch::Tensor x, int64_t kh, int64_t kw, int64_t stride, int64_t pad, int64_t dil,
                torch::Tensor out, int64_t splits, int64_t variant, OptT ws, OptT counters) {
  check_nhwc(dy, "dy");
  check_nhwc(x, "x");
  const auto s = make_shape(x.size(0), x.size(1), x.size(2), x.size(3), dy.size(3), kh, kw, stride, pad, dil);
  TORCH_CHECK(s.O % 8 == 0 && s.C % 8 == 0, "conv_wgrad: needs O % 8 == 0 and C % 8 == 0");
  TORCH_CHECK(dy.size(0) == s.N && dy.size(1) == s.OH && dy.size(2) == s.OW, "conv_wgrad: dy shape");
  TORCH_CHECK(out.is_cuda() && out.is_contiguous() && reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0,
              "conv_wgrad: out must be contiguous and 16-byte aligned");
  const int64_t n = int64_t(s.O) * kh * kw * s.C;
  const auto k = make_splitk(splits, ws, counters, s.O, kh * kw * s.C, x, "conv_wgrad", variant);
  int out_bf16 = 0;
  if (k.splits > 1 && !k.counters) {
    TORCH_CHECK(out.scalar_type() == torch::kFloat32 && out.is_contiguous() && out.numel() >= splits * slab_elems(s.O, kh * kw * s.C),
                "conv_wgrad: split-K out must be contiguous fp32 with splits * slab_elems elements");
  } else {
    TORCH_CHECK(out.numel() == n && (out.scalar_type() == torch::kFloat32 || out.scalar_type() == torch::kBFloat16),
                "conv_wgrad: out must be [O, kh, kw, C] bf16/fp32");
    out_bf16 = out.scalar_type() == torch::kBFloat16;
  }
  TORCH_CHECK(dy.device() == x.device() && out.device() == x.device(), "conv_wgrad: device mismatch");
  const c10::DeviceGuard g(x.device());
  p2::conv_wgrad(s, reinterpret_cast<const uint16_t*>(dy.data_ptr()), reinterpret_cast<const uint16_t*>(x.data_ptr()),
                 out.data_ptr(), out_bf16, k, int(variant), stream_of(x));
}

// out = sum over dim 0 of fp32 slabs [S, n]
void slab_sum(torch::Tensor slabs, torch::Tensor out) {
  TORCH_CHECK(slabs.is_cuda() && slabs.scalar_type() == torch::kFloat32 && slabs.dim() == 2 && slabs.is_contiguous(),
              "slab_sum: slabs must be contiguous fp32 [S, n]");
  const int64_t n = slabs.size(1);
  TORCH_CHECK(n % 4 == 0 && out.is_cuda() && out.is_contiguous() && out.numel() == n &&
                  (out.scalar_type() == torch::kFloat32 || out.scalar_type() == torch::kBFloat16),
              "slab_sum: out must be contiguous fp32/bf16 with n % 4 == 0 elements");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(slabs.data_ptr()) % 16 == 0,
              "slab_sum: alignment");
  TORCH_CHECK(slabs.size(0) >= 1 && slabs.device() == out.device(), "slab_sum: bad slabs");
  const c10::DeviceGuard g(out.device());
  p2::slab_sum(slabs.data_ptr<float>(), int(slabs.size(0)), n, out.data_ptr(), out.scalar_type() == torch::kBFloat16,
               stream_of(out));
}

// ---- small-C direct convolution (stem) ----------------------------------------------
p2::StemShape stem_shape(const torch::Tensor& x, const torch::Tensor& w, int64_t stride, int64_t pad, double xscale,
                         int& xtype, const char* who) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 4, who, ": x must be a 4-D GPU tensor (N, C, H, W) in any memory layout");
  TORCH_CHECK(x.scalar_type() == torch::kFloat32 || x.scalar_type() == torch::kBFloat16 || x.scalar_type() == torch::kUInt8,
              who, ": x must be fp32, bf16 or uint8");
  xtype = x.scalar_type() == torch::kFloat32 ? 0 : (x.scalar_type() == torch::kBFloat16 ? 1 : 2);
  check_nhwc(w, "w");
  TORCH_CHECK(w.size(3) == x.size(1), who, ": channel mismatch");
  TORCH_CHECK(stride >= 1 && stride <= 4 && pad >= 0 && pad <= 8, who, ": stride 1-4, pad 0-8");
  p2::StemShape s{};
  s.N = int(x.size(0));
  s.C = int(x.size(1));
  s.H = int(x.size(2));
  s.W = int(x.size(3));
  s.O = int(w.size(0));
  s.kh = int(w.size(1));
  s.kw = int(w.size(2));
  s.stride = int(stride);
  s.pad = int(pad);
  s.OH = out_size(s.H, s.kh, s.stride, s.pad, 1);
  s.OW = out_size(s.W, s.kw, s.stride, s.pad, 1);
  TORCH_CHECK(s.OH >= 1 && s.OW >= 1, who, ": empty output");
  TORCH_CHECK(s.kh * s.kw * s.C <= 160 && s.O % 16 == 0 && s.O <= 256, who, ": needs kh*kw*C <= 160, O % 16 == 0, O <= 256");
  TORCH_CHECK(s.kh * s.kw * s.C * s.O * 4 <= 40 * 1024, who, ": weight image exceeds the LDS budget");
  TORCH_CHECK(int64_t(s.N) * s.OH * s.OW < (int64_t(1) << 30) && x.numel() < (int64_t(1) << 31), who, ": size overflow");
  s.sn = x.stride(0);
  s.sc = x.stride(1);
  s.sh = x.stride(2);
  s.sw = x.stride(3);
  s.xscale = float(xscale);
  TORCH_CHECK(x.device() == w.device(), who, ": device mismatch");
  return s;
}

// x (N, C, H, W) any layout, w [O, kh, kw, C] bf16  ->  y [N, OH, OW, O] bf16
void stem_fwd(torch::Tensor x, torch::Tensor w, int64_t stride, int64_t pad, double xscale, torch::Tensor y) {
  int xtype = 0;
  const auto s = stem_shape(x, w, stride, pad, xscale, xtype, "stem_fwd");
  check_nhwc(y, "y");
  TORCH_CHECK(y.size(0) == s.N && y.size(1) == s.OH && y.size(2) == s.OW && y.size(3) == s.O && y.device() == x.device(),
              "stem_fwd: y must be [N, OH, OW, O]");
  const c10::DeviceGuard g(x.device());
  p2::stem_fwd(s, x.data_ptr(), xtype, reinterpret_cast<const uint16_t*>(w.data_ptr()),
               reinterpret_cast<uint16_t*>(y.data_ptr()), stream_of(x));
}

int64_t stem_wgrad_parts(int64_t N, int64_t OH, int64_t OW) { return p2::stem_wgrad_parts(int(N), int(OH), int(OW)); }

// dy [N, OH, OW, O] bf16, x (N, C, H, W) any layout; w only for its shape -> dw [O, kh, kw, C] bf16 / fp32
void stem_wgrad(torch::Tensor dy, torch::Tensor x, torch::Tensor w, int64_t stride, int64_t pad, double xscale,
                torch::Tensor part, torch::Tensor dw) {
  int xtype = 0;
  const auto s = stem_shape(x, w, stride, pad, xscale, xtype, "stem_wgrad");
  TORCH_CHECK(s.O == 32 || s.O == 64, "stem_wgrad: O must be 32 or 64");
  check_nhwc(dy, "dy");
  TORCH_CHECK(dy.size(0) == s.N && dy.size(1) == s.OH && dy.size(2) == s.OW && dy.size(3) == s.O, "stem_wgrad: dy shape");
  const int64_t n = int64_t(s.O) * s.kh * s.kw * s.C;
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == torch::kFloat32 && part.is_contiguous() &&
                  part.numel() >= p2::stem_wgrad_parts(s.N, s.OH, s.OW) * n,
              "stem_wgrad: part must be contiguous fp32 with stem_wgrad_parts * O * kh * kw * C elements");
  TORCH_CHECK(dw.is_cuda() && dw.is_contiguous() && dw.numel() == n &&
                  (dw.scalar_type() == torch::kFloat32 || dw.scalar_type() == torch::kBFloat16),
              "stem_wgrad: dw must be contiguous [O, kh, kw, C] bf16/fp32");
  TORCH_CHECK(dy.device() == x.device() && part.device() == x.device() && dw.device() == x.device(), "stem_wgrad: device");
  const c10::DeviceGuard g(x.device());
  p2::stem_wgrad(s, x.data_ptr(), xtype, reinterpret_cast<const uint16_t*>(dy.data_ptr()), part.data_ptr<float>(),
                 dw.data_ptr(), dw.scalar_type() == torch::kBFloat16, stream_of(x));
}

}  // namespace

void register_conv(pybind11::module& m) {
  using pybind11::arg;
  m.def("stem_fwd", &stem_fwd, "small-C direct convolution forward (stem)", pybind11::arg("x"), pybind11::arg("w"),
        pybind11::arg("stride"), pybind11::arg("pad"), pybind11::arg("xscale"), pybind11::arg("y"));
  m.def("conv_fwd_bn", &conv_fwd_bn, "implicit-GEMM conv forward + BatchNorm statistics in the launch", arg("x"),
        arg("w"), arg("stride"), arg("pad"), arg("dil"), arg("y"), arg("splits"), arg("variant"), arg("ws"),
        arg("counters"), arg("part"), arg("cnt"), arg("bn_w"), arg("bn_b"), arg("run_mean"), arg("run_var"), arg("nbt"),
        arg("mean"), arg("rstd"), arg("coef"), arg("eps"), arg("momentum"));
  m.def("conv_dgrad_bn", &conv_dgrad_bn, "implicit-GEMM conv input gradient + BatchNorm backward statistics",
        arg("dy"), arg("w"), arg("stride"), arg("pad"), arg("dil"), arg("dx"), arg("dx_shape"), arg("splits"),
        arg("variant"), arg("ws"), arg("counters"), arg("part"), arg("cnt"), arg("bn_w"), arg("bx"), arg("by"),
        arg("bmean"), arg("brstd"), arg("dgamma"), arg("dbeta"), arg("coef"));
  m.def("stem_wgrad_parts", &stem_wgrad_parts, "partial rows of the stem weight gradient");
  m.def("stem_wgrad", &stem_wgrad, "small-C direct convolution weight gradient (stem)", pybind11::arg("dy"),
        pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("stride"), pybind11::arg("pad"), pybind11::arg("xscale"),
        pybind11::arg("part"), pybind11::arg("dw"));
  m.def("conv_fwd", &conv_fwd, "implicit-GEMM conv forward (NHWC bf16)", arg("x"), arg("w"), arg("stride"), arg("pad"),
        arg("dil"), arg("y"), arg("splits") = 1, arg("variant") = 10, arg("ws") = pybind11::none(),
        arg("counters") = pybind11::none());
  m.def("conv_dgrad", &conv_dgrad, "implicit-GEMM conv input gradient", arg("dy"), arg("w"), arg("stride"), arg("pad"),
        arg("dil"), arg("dx"), arg("dx_shape"), arg("splits") = 1, arg("variant") = 10, arg("ws") = pybind11::none(),
        arg("counters") = pybind11::none());
  m.def("conv_dgrad_s2", &conv_dgrad_s2, "stride-2 conv input gradient by output phase (phase-major out)", arg("dy"),
        arg("w"), arg("pad"), arg("out"), arg("dx_shape"), arg("splits") = 1, arg("variant") = 10,
        arg("ws") = pybind11::none(), arg("counters") = pybind11::none());
  m.def("phase_interleave", &phase_interleave, "phase-major stride-2 input gradient -> NHWC dX", arg("src"), arg("dx"),
        arg("pad"), arg("kh") = 3, arg("kw") = 3);
  m.def("conv_wgrad", &conv_wgrad, "implicit-GEMM conv weight gradient", arg("dy"), arg("x"), arg("kh"), arg("kw"),
        arg("stride"), arg("pad"), arg("dil"), arg("out"), arg("splits") = 1, arg("variant") = 2,
        arg("ws") = pybind11::none(), arg("counters") = pybind11::none());
  m.def("slab_sum", &slab_sum, "sum of fp32 split-K slabs", arg("slabs"), arg("out"));
}
