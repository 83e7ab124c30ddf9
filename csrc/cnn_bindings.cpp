// PyTorch bindings of the fused MNIST-CNN training kernels (csrc/cnn_*.hip).
// Every binding checks dtypes, sizes and devices on the host before it
// launches, so a wrong call raises instead of faulting the GPU.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <c10/core/DeviceGuard.h>

#include "cnn.h"

namespace {

using p2cnn::AdamCfg;
using p2cnn::Offsets;

hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

template <typename T>
T* ptr(const torch::Tensor& t, c10::ScalarType st, int64_t min_numel, const char* name, int align = 16) {
  TORCH_CHECK(t.defined() && t.is_cuda(), name, ": expected a GPU tensor");
  TORCH_CHECK(t.scalar_type() == st, name, ": wrong dtype ", t.scalar_type());
  TORCH_CHECK(t.is_contiguous(), name, ": must be contiguous");
  TORCH_CHECK(t.numel() >= min_numel, name, ": needs >= ", min_numel, " elements, got ", t.numel());
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % align == 0, name, ": must be ", align, "-byte aligned");
  return reinterpret_cast<T*>(t.data_ptr());
}
template <typename T>
T* optr(const c10::optional<torch::Tensor>& t, c10::ScalarType st, int64_t min_numel, const char* name,
        int align = 16) {
  if (!t.has_value() || !t->defined()) return nullptr;
  return ptr<T>(*t, st, min_numel, name, align);
}

Offsets offsets(const std::vector<int64_t>& o) {
  TORCH_CHECK(o.size() == 8, "offsets: expected 8 entries");
  for (auto v : o) TORCH_CHECK(v >= 0, "offsets: negative");
  return Offsets{o[0], o[1], o[2], o[3], o[4], o[5], o[6], o[7]};
}

int64_t params_end(const Offsets& o) {
  return std::max({o.c1w + 800, o.c1b + 32, o.c2w + 51200, o.c2b + 64, o.l1w + int64_t(2048) * 3136, o.l1b + 2048,
                   o.l2w + 20480, o.l2b + 10});
}

void check_batch(int B, int mrows) {
  // 128-row launches exist for the forward-only (evaluation) kernels
  TORCH_CHECK(mrows == 32 || mrows == 64 || mrows == 128, "mrows must be 32, 64 or 128");
  TORCH_CHECK(B >= 1 && B <= mrows, "batch ", B, " exceeds mrows ", mrows);
}

const int64_t* idx_ptr(const c10::optional<torch::Tensor>& idx, int B) {
  return optr<int64_t>(idx, torch::kInt64, B, "idx", 8);
}

// NOTE: gathers through idx are bounds-checked on the host only by shape; the
// learner guarantees idx values are permutations of the dataset rows.

void k_conv1_fwd(torch::Tensor x, c10::optional<torch::Tensor> idx, torch::Tensor params, std::vector<int64_t> off,
                 torch::Tensor p1, torch::Tensor am1, c10::optional<torch::Tensor> p1s, int64_t B) {
  const c10::DeviceGuard g(params.device());
  // training launches (P1s wanted) hold <= 64 images; evaluation launches <= 128
  TORCH_CHECK(B >= 1 && B <= (p1s.has_value() && p1s->defined() ? 64 : 128), "bad batch");
  Offsets o = offsets(off);
  TORCH_CHECK(x.numel() % 784 == 0, "x must be [N,1,28,28] uint8");
  if (!idx.has_value()) TORCH_CHECK(x.numel() / 784 >= B, "x has fewer than B rows");
  p2cnn::conv1_fwd(ptr<uint8_t>(x, torch::kUInt8, 784, "x", 1), idx_ptr(idx, B),
                   ptr<float>(params, torch::kFloat32, params_end(o), "params"), o,
                   reinterpret_cast<uint16_t*>(ptr<at::BFloat16>(p1, torch::kBFloat16, B * 196 * 32, "p1")),
                   ptr<uint8_t>(am1, torch::kUInt8, B * 196 * 32, "am1"),
                   reinterpret_cast<uint16_t*>(optr<at::BFloat16>(p1s, torch::kBFloat16, B * p2cnn::kP1s, "p1s")),
                   int(B), stream());
}

void k_conv2_fwd(torch::Tensor p1, torch::Tensor w2r, torch::Tensor params, std::vector<int64_t> off,
                 torch::Tensor a1, torch::Tensor am2, int64_t B, int64_t mrows) {
  const c10::DeviceGuard g(params.device());
  check_batch(int(B), int(mrows));
  Offsets o = offsets(off);
  p2cnn::conv2_fwd(reinterpret_cast<uint16_t*>(ptr<at::BFloat16>(p1, torch::kBFloat16, B * 196 * 32, "p1")),
                   reinterpret_cast<uint16_t*>(ptr<at::BFloat16>(w2r, torch::kBFloat16, 51200, "w2r")),
                   ptr<float>(params, torch::kFloat32, params_end(o), "params"), o,
                   reinterpret_cast<uint16_t*>(ptr<at::BFloat16>(a1, torch::kBFloat16, mrows * 3136, "a1")),
                   ptr<uint8_t>(am2, torch::kUInt8, B * 3136, "am2"), int(B), stream());
}

void k_conv12_fwd(torch::Tensor x, c10::optional<torch::Tensor> idx, torch::Tensor params, std::vector<int64_t> off,
                  torch::Tensor w2r, c10::optional<torch::Tensor> p1, torch::Tensor am1, c10::optional<torch::Tensor> p1s,
                  torch::Tensor a1, torch::Tensor am2, int64_t B, int64_t mrows) {
  const c10::DeviceGuard g(params.device());
  check_batch(int(B), int(mrows));
  TORCH_CHECK(!(p1s.has_value() && p1s->defined()) || B <= 64, "conv12_fwd: training launches hold <= 64 images");
  Offsets o = offsets(off);
  TORCH_CHECK(x.numel() % 784 == 0, "x must be [N,1,28,28] uint8");
  if (!idx.has_value()) TORCH_CHECK(x.numel() / 784 >= B, "x has fewer than B rows");
  p2cnn::conv12_fwd(ptr<uint8_t>(x, torch::kUInt8, 784, "x", 1), idx_ptr(idx, int(B)),
                    ptr<float>(params, torch::kFloat32, params_end(o), "params"), o,
                    reinterpret_cast<uint16_t*>(ptr<at::BFloat16>(w2r, torch::kBFloat16, 51200, "w2r")),
                    reinterpret_cast<uint16_t*>(optr<at::BFloat16>(p1, torch::kBFloat16, B * 196 * 32, "p1")),
                    ptr<uint8_t>(am1, torch::kUInt8, B * 196 * 32, "am1"),
                    reinterpret_cast<uint16_t*>(optr<at::BFloat16>(p1s, torch::kBFloat16, B * p2cnn::kP1s, "p1s")),
                    reinterpret_cast<uint16_t*>(ptr<at::BFloat16>(a1, torch::kBFloat16, mrows * 3136, "a1")),
                    ptr<uint8_t>(am2, torch::kUInt8, B * 3136, "am2"), int(B), stream());
}

void k_gemm_skinny(torch::Tensor A, torch::Tensor Bt, torch::Tensor slabs, int64_t mrows, int64_t N, int64_t K,
                   int64_t S) {
  const c10::DeviceGuard g(A.device());
  TORCH_CHECK(N % 32 == 0 && K % 64 == 0 && S >= 1, "gemm_skinny: N%32, K%64 required");
  TORCH_CHECK(mrows == 32 || mrows == 64 || mrows == 128, "gemm_skinny: mrows must be 32, 64 or 128");
  p2cnn::gemm_skinny(reinterpret_cast<uint16_t*>(ptr<at::BFloat16>(A, torch::kBFloat16, mrows * K, "A")),
                     reinterpret_cast<uint16_t*>(ptr<at::BFloat16>(Bt, torch::kBFloat16, N * K, "Bt")),
                     ptr<float>(slabs, torch::kFloat32, S * mrows * N, "slabs"), int(mrows), int(N), int(K), int(S),
                     stream());
}

void k_head(torch::Tensor slabs, int64_t S, int64_t mrows, torch::Tensor params, std::vector<int64_t> off,
            torch::Tensor labels, c10::optional<torch::Tensor> idx, int64_t B, bool train, torch::Tensor H,
            torch::Tensor dH, torch::Tensor dlogits, torch::Tensor stats, c10::optional<torch::Tensor> w2bf) {
  const c10::DeviceGuard g(params.device());
  check_batch(int(B), int(mrows));
  Offsets o = offsets(off);
  if (!idx.has_value()) TORCH_CHECK(labels.numel() >= B, "labels has fewer than B rows");
  p2cnn::head(ptr<float>(slabs, torch::kFloat32, S * mrows * 2048, "slabs"), int(S), int(mrows),
              ptr<float>(params, torch::kFloat32, params_end(o), "params"), o,
              ptr<int64_t>(labels, torch::kInt64, 1, "labels", 8), idx_ptr(idx, B), int(B), train ? 1 : 0,
              reinterpret_cast<uint16_t*>(ptr<at::BFloat16>(H, torch::kBFloat16, mrows * 2048, "H")),
              reinterpret_cast<uint16_t*>(ptr<at::BFloat16>(dH, torch::kBFloat16, mrows * 2048, "dH")),
              ptr<float>(dlogits, torch::kFloat32, mrows * 10, "dlogits"), ptr<float>(stats, torch::kFloat32, 2, "stats", 4),
              reinterpret_cast<const uint16_t*>(optr<at::BFloat16>(w2bf, torch::kBFloat16, 10 * 2048, "w2bf")),
              stream());
}

AdamCfg cfg(double lr, double b1, double b2, double eps, double wd) {
  return AdamCfg{float(lr), float(b1), float(b2), float(eps), float(wd)};
}

void k_fc1_wgrad_adam(torch::Tensor dH, torch::Tensor a1, int64_t mrows, torch::Tensor params, torch::Tensor m,
                      torch::Tensor v, c10::optional<torch::Tensor> gdump, torch::Tensor w1bf, c10::optional<torch::Tensor> w1tbf,
                      std::vector<int64_t> off, torch::Tensor adam_t, int64_t t_off, double lr, double b1, double b2,
                      double eps, double wd) {
  const c10::DeviceGuard g(params.device());
  TORCH_CHECK(mrows == 32 || mrows == 64, "mrows must be 32 or 64");
  Offsets o = offsets(off);
  const int64_t n = params_end(o);
  p2cnn::fc1_wgrad_adam(reinterpret_cast<uint16_t*>(ptr<at::BFloat16>(dH, torch::kBFloat16, mrows * 2048, "dH")),
                        reinterpret_cast<uint16_t*>(ptr<at::BFloat16>(a1, torch::kBFloat16, mrows * 3136, "a1")),
                        int(mrows), ptr<float>(params, torch::kFloat32, n, "params"),
                        ptr<float>(m, torch::kFloat32, n, "m"), ptr<float>(v, torch::kFloat32, n, "v"),
                        optr<float>(gdump, torch::kFloat32, n, "gdump"),
                        reinterpret_cast<uint16_t*>(ptr<at::BFloat16>(w1bf, torch::kBFloat16, 2048 * 3136, "w1bf")),
                        reinterpret_cast<uint16_t*>(optr<at::BFloat16>(w1tbf, torch::kBFloat16, 2048 * 3136, "w1tbf")),
                        o, ptr<int>(adam_t, torch::kInt32, 1, "adam_t", 4), int(t_off), cfg(lr, b1, b2, eps, wd), stream());
}

void k_route_fc2(torch::Tensor dH, torch::Tensor w1, torch::Tensor am2, int64_t mrows, int64_t B,
                 torch::Tensor dc2m, torch::Tensor gb, torch::Tensor dlogits, torch::Tensor H, torch::Tensor params,
                 torch::Tensor m, torch::Tensor v, c10::optional<torch::Tensor> gdump, std::vector<int64_t> off,
                 torch::Tensor adam_t, int64_t t_off, double lr, double b1, double b2, double eps, double wd,
                 bool with_fc2, bool row_major, c10::optional<torch::Tensor> ws, c10::optional<torch::Tensor> ctr) {
  const c10::DeviceGuard g(dH.device());
  check_batch(int(B), int(mrows));
  TORCH_CHECK(mrows <= 64, "route_fc2: mrows must be 32 or 64");
  TORCH_CHECK(ws.has_value() == ctr.has_value(), "route_fc2: split-K needs both ws and ctr");
  TORCH_CHECK(!ws.has_value() || row_major, "route_fc2: split-K only on the row-major W1 kernel");
  Offsets o = offsets(off);
  const int64_t n = params_end(o);
  const auto dHp = reinterpret_cast<uint16_t*>(ptr<at::BFloat16>(dH, torch::kBFloat16, mrows * 2048, "dH"));
  const auto w1p = reinterpret_cast<uint16_t*>(ptr<at::BFloat16>(w1, torch::kBFloat16, 2048 * 3136, "w1"));
  const auto am2p = ptr<uint8_t>(am2, torch::kUInt8, B * 3136, "am2");
  const auto dc2p = reinterpret_cast<uint16_t*>(ptr<at::BFloat16>(dc2m, torch::kBFloat16, B * 64 * 224, "dc2m"));
  const auto gbp = ptr<float>(gb, torch::kFloat32, B * 3136, "gb");
  const auto dlp = ptr<float>(dlogits, torch::kFloat32, B * 10, "dlogits");
  const auto Hp = reinterpret_cast<uint16_t*>(ptr<at::BFloat16>(H, torch::kBFloat16, B * 2048, "H"));
  float* pp = ptr<float>(params, torch::kFloat32, n, "params");
  float* mp = ptr<float>(m, torch::kFloat32, n, "m");
  float* vp = ptr<float>(v, torch::kFloat32, n, "v");
  float* gd = optr<float>(gdump, torch::kFloat32, n, "gdump");
  const int* tp = ptr<int>(adam_t, torch::kInt32, 1, "adam_t", 4);
  if (row_major) {
    // split-K partials: [98 tiles][2 slices][mrows * 32] fp32; one ticket per tile
    float* wsp = optr<float>(ws, torch::kFloat32, 98 * 2 * mrows * 32, "ws");
    int* cp = optr<int>(ctr, torch::kInt32, 98, "ctr", 4);
    p2cnn::route_fc2_rm(dHp, w1p, am2p, int(mrows), int(B), dc2p, gbp, dlp, Hp, pp, mp, vp, gd, o, tp, int(t_off),
                        cfg(lr, b1, b2, eps, wd), with_fc2, wsp, cp, stream());
  } else {
    // w1 is the W1^T shadow [3136][2048]
    p2cnn::route_fc2(dHp, w1p, am2p, int(mrows), int(B), dc2p, gbp, dlp, Hp, pp, mp, vp, gd, o, tp, int(t_off),
                     cfg(lr, b1, b2, eps, wd), with_fc2, stream());
  }
}

void k_conv2_bwd(torch::Tensor dc2m, torch::Tensor p1s, torch::Tensor am1, torch::Tensor w2q, torch::Tensor x,
                 c10::optional<torch::Tensor> idx, torch::Tensor wslab1, torch::Tensor wslab2, int64_t B) {
  const c10::DeviceGuard g(dc2m.device());
  TORCH_CHECK(B >= 1 && B <= 64, "bad batch");
  TORCH_CHECK(x.numel() % 784 == 0, "x must be [N,1,28,28] uint8");
  if (!idx.has_value()) TORCH_CHECK(x.numel() / 784 >= B, "x has fewer than B rows");
  p2cnn::conv2_bwd(reinterpret_cast<uint16_t*>(ptr<at::BFloat16>(dc2m, torch::kBFloat16, B * 64 * 224, "dc2m")),
                   reinterpret_cast<uint16_t*>(ptr<at::BFloat16>(p1s, torch::kBFloat16, B * p2cnn::kP1s, "p1s")),
                   ptr<uint8_t>(am1, torch::kUInt8, B * 196 * 32, "am1"),
                   reinterpret_cast<uint16_t*>(ptr<at::BFloat16>(w2q, torch::kBFloat16, 51200, "w2q")),
                   ptr<uint8_t>(x, torch::kUInt8, 784, "x", 1), idx_ptr(idx, B),
                   ptr<float>(wslab1, torch::kFloat32, B * p2cnn::kDgTiles * p2cnn::kSlab1, "wslab1"),
                   ptr<float>(wslab2, torch::kFloat32, p2cnn::wgrad_groups(int(B)) * int64_t(p2cnn::kSlab2), "wslab2"),
                   int(B), stream());
}

void k_conv_adam(torch::Tensor wslab1, torch::Tensor wslab2, torch::Tensor gb, int64_t B, torch::Tensor params,
                 torch::Tensor m,
                 torch::Tensor v, c10::optional<torch::Tensor> gdump, torch::Tensor w2r, torch::Tensor w2q,
                 std::vector<int64_t> off, torch::Tensor adam_t, int64_t t_off, double lr, double b1, double b2,
                 double eps, double wd) {
  const c10::DeviceGuard g(params.device());
  Offsets o = offsets(off);
  const int64_t n = params_end(o);
  TORCH_CHECK(B >= 1 && B <= 64, "bad batch");
  p2cnn::conv_adam(ptr<float>(wslab1, torch::kFloat32, B * p2cnn::kDgTiles * p2cnn::kSlab1, "wslab1"),
                   ptr<float>(wslab2, torch::kFloat32, p2cnn::wgrad_groups(int(B)) * int64_t(p2cnn::kSlab2), "wslab2"),
                   ptr<float>(gb, torch::kFloat32, B * 3136, "gb"), int(B),
                   ptr<float>(params, torch::kFloat32, n, "params"), ptr<float>(m, torch::kFloat32, n, "m"),
                   ptr<float>(v, torch::kFloat32, n, "v"), optr<float>(gdump, torch::kFloat32, n, "gdump"),
                   reinterpret_cast<uint16_t*>(ptr<at::BFloat16>(w2r, torch::kBFloat16, 51200, "w2r")),
                   reinterpret_cast<uint16_t*>(ptr<at::BFloat16>(w2q, torch::kBFloat16, 51200, "w2q")), o,
                   ptr<int>(adam_t, torch::kInt32, 1, "adam_t", 4), int(t_off), cfg(lr, b1, b2, eps, wd), stream());
}

void k_fc1_conv_adam(torch::Tensor dH, torch::Tensor a1, int64_t mrows, torch::Tensor wslab1, torch::Tensor wslab2,
                     torch::Tensor gb, int64_t B, torch::Tensor params, torch::Tensor m, torch::Tensor v,
                     c10::optional<torch::Tensor> gdump, torch::Tensor w1bf, c10::optional<torch::Tensor> w1tbf, torch::Tensor w2r,
                     torch::Tensor w2q, std::vector<int64_t> off, torch::Tensor adam_t, int64_t t_off, double lr,
                     double b1, double b2, double eps, double wd, c10::optional<torch::Tensor> dlogits,
                     c10::optional<torch::Tensor> H, c10::optional<torch::Tensor> w2bf) {
  const c10::DeviceGuard g(params.device());
  check_batch(int(B), int(mrows));
  TORCH_CHECK(mrows <= 64, "fc1_conv_adam: mrows must be 32 or 64");
  TORCH_CHECK(dlogits.has_value() == H.has_value(), "fc1_conv_adam: pass both dlogits and H or neither");
  Offsets o = offsets(off);
  const int64_t n = params_end(o);
  p2cnn::fc1_conv_adam(
      reinterpret_cast<uint16_t*>(ptr<at::BFloat16>(dH, torch::kBFloat16, mrows * 2048, "dH")),
      reinterpret_cast<uint16_t*>(ptr<at::BFloat16>(a1, torch::kBFloat16, mrows * 3136, "a1")), int(mrows),
      ptr<float>(wslab1, torch::kFloat32, B * p2cnn::kDgTiles * p2cnn::kSlab1, "wslab1"),
      ptr<float>(wslab2, torch::kFloat32, p2cnn::wgrad_groups(int(B)) * int64_t(p2cnn::kSlab2), "wslab2"),
      ptr<float>(gb, torch::kFloat32, B * 3136, "gb"), int(B), ptr<float>(params, torch::kFloat32, n, "params"),
      ptr<float>(m, torch::kFloat32, n, "m"), ptr<float>(v, torch::kFloat32, n, "v"),
      optr<float>(gdump, torch::kFloat32, n, "gdump"),
      reinterpret_cast<uint16_t*>(ptr<at::BFloat16>(w1bf, torch::kBFloat16, 2048 * 3136, "w1bf")),
      reinterpret_cast<uint16_t*>(optr<at::BFloat16>(w1tbf, torch::kBFloat16, 2048 * 3136, "w1tbf")),
      reinterpret_cast<uint16_t*>(ptr<at::BFloat16>(w2r, torch::kBFloat16, 51200, "w2r")),
      reinterpret_cast<uint16_t*>(ptr<at::BFloat16>(w2q, torch::kBFloat16, 51200, "w2q")), o,
      ptr<int>(adam_t, torch::kInt32, 1, "adam_t", 4), int(t_off), cfg(lr, b1, b2, eps, wd),
      optr<float>(dlogits, torch::kFloat32, B * 10, "dlogits"),
      reinterpret_cast<const uint16_t*>(optr<at::BFloat16>(H, torch::kBFloat16, B * 2048, "H")),
      reinterpret_cast<uint16_t*>(optr<at::BFloat16>(w2bf, torch::kBFloat16, 10 * 2048, "w2bf")), stream());
}

// fc1_conv_adam + the next step's conv1 / conv2 (p2cnn::fc1_conv_adam_fwd): the same
// arguments, then the next step's x / idx / P1 / AM1 / P1s / A1 (the other parity
// buffer) / AM2, its batch size and 4 zero int32 (tickets + timeout flag)
void k_fc1_conv_adam_fwd(torch::Tensor dH, torch::Tensor a1, int64_t mrows, torch::Tensor wslab1, torch::Tensor wslab2,
                         torch::Tensor gb, int64_t B, torch::Tensor params, torch::Tensor m, torch::Tensor v,
                         c10::optional<torch::Tensor> gdump, torch::Tensor w1bf, c10::optional<torch::Tensor> w1tbf,
                         torch::Tensor w2r, torch::Tensor w2q, std::vector<int64_t> off, torch::Tensor adam_t,
                         int64_t t_off, double lr, double b1, double b2, double eps, double wd,
                         c10::optional<torch::Tensor> dlogits, c10::optional<torch::Tensor> H,
                         c10::optional<torch::Tensor> w2bf, torch::Tensor x, c10::optional<torch::Tensor> idx,
                         torch::Tensor p1, torch::Tensor am1, torch::Tensor p1s, torch::Tensor a1n, torch::Tensor am2,
                         int64_t Bn, torch::Tensor sync) {
  const c10::DeviceGuard g(params.device());
  check_batch(int(B), int(mrows));
  check_batch(int(Bn), int(mrows));
  TORCH_CHECK(mrows <= 64, "fc1_conv_adam_fwd: mrows must be 32 or 64");
  TORCH_CHECK(dlogits.has_value() == H.has_value(), "fc1_conv_adam_fwd: pass both dlogits and H or neither");
  TORCH_CHECK(x.numel() % 784 == 0, "x must be [N,1,28,28] uint8");
  if (!idx.has_value()) TORCH_CHECK(x.numel() / 784 >= Bn, "x has fewer than Bn rows");
  TORCH_CHECK(a1n.data_ptr() != a1.data_ptr(), "fc1_conv_adam_fwd: the next step's A1 must be the other buffer");
  Offsets o = offsets(off);
  const int64_t n = params_end(o);
  p2cnn::FwdNext f{};
  f.x = ptr<uint8_t>(x, torch::kUInt8, 784, "x", 1);
  f.idx = idx_ptr(idx, int(Bn));
  f.p1 = reinterpret_cast<uint16_t*>(ptr<at::BFloat16>(p1, torch::kBFloat16, Bn * 196 * 32, "p1"));
  f.am1 = ptr<uint8_t>(am1, torch::kUInt8, Bn * 196 * 32, "am1");
  f.p1s = reinterpret_cast<uint16_t*>(ptr<at::BFloat16>(p1s, torch::kBFloat16, Bn * p2cnn::kP1s, "p1s"));
  f.a1 = reinterpret_cast<uint16_t*>(ptr<at::BFloat16>(a1n, torch::kBFloat16, mrows * 3136, "a1n"));
  f.am2 = ptr<uint8_t>(am2, torch::kUInt8, Bn * 3136, "am2");
  f.B = int(Bn);
  f.sync = ptr<int>(sync, torch::kInt32, 4, "sync", 4);
  p2cnn::fc1_conv_adam_fwd(
      reinterpret_cast<uint16_t*>(ptr<at::BFloat16>(dH, torch::kBFloat16, mrows * 2048, "dH")),
      reinterpret_cast<uint16_t*>(ptr<at::BFloat16>(a1, torch::kBFloat16, mrows * 3136, "a1")), int(mrows),
      ptr<float>(wslab1, torch::kFloat32, B * p2cnn::kDgTiles * p2cnn::kSlab1, "wslab1"),
      ptr<float>(wslab2, torch::kFloat32, p2cnn::wgrad_groups(int(B)) * int64_t(p2cnn::kSlab2), "wslab2"),
      ptr<float>(gb, torch::kFloat32, B * 3136, "gb"), int(B), ptr<float>(params, torch::kFloat32, n, "params"),
      ptr<float>(m, torch::kFloat32, n, "m"), ptr<float>(v, torch::kFloat32, n, "v"),
      optr<float>(gdump, torch::kFloat32, n, "gdump"),
      reinterpret_cast<uint16_t*>(ptr<at::BFloat16>(w1bf, torch::kBFloat16, 2048 * 3136, "w1bf")),
      reinterpret_cast<uint16_t*>(optr<at::BFloat16>(w1tbf, torch::kBFloat16, 2048 * 3136, "w1tbf")),
      reinterpret_cast<uint16_t*>(ptr<at::BFloat16>(w2r, torch::kBFloat16, 51200, "w2r")),
      reinterpret_cast<uint16_t*>(ptr<at::BFloat16>(w2q, torch::kBFloat16, 51200, "w2q")), o,
      ptr<int>(adam_t, torch::kInt32, 1, "adam_t", 4), int(t_off), cfg(lr, b1, b2, eps, wd),
      optr<float>(dlogits, torch::kFloat32, B * 10, "dlogits"),
      reinterpret_cast<const uint16_t*>(optr<at::BFloat16>(H, torch::kBFloat16, B * 2048, "H")),
      reinterpret_cast<uint16_t*>(optr<at::BFloat16>(w2bf, torch::kBFloat16, 10 * 2048, "w2bf")), f, stream());
}

void k_pack_shadows(torch::Tensor params, std::vector<int64_t> off, torch::Tensor w2r, torch::Tensor w2q,
                    torch::Tensor w1bf, c10::optional<torch::Tensor> w1tbf, c10::optional<torch::Tensor> w2bf) {
  const c10::DeviceGuard g(params.device());
  Offsets o = offsets(off);
  p2cnn::pack_shadows(ptr<float>(params, torch::kFloat32, params_end(o), "params"), o,
                      reinterpret_cast<uint16_t*>(ptr<at::BFloat16>(w2r, torch::kBFloat16, 51200, "w2r")),
                      reinterpret_cast<uint16_t*>(ptr<at::BFloat16>(w2q, torch::kBFloat16, 51200, "w2q")),
                      reinterpret_cast<uint16_t*>(ptr<at::BFloat16>(w1bf, torch::kBFloat16, 2048 * 3136, "w1bf")),
                      reinterpret_cast<uint16_t*>(optr<at::BFloat16>(w1tbf, torch::kBFloat16, 2048 * 3136, "w1tbf")),
                      reinterpret_cast<uint16_t*>(optr<at::BFloat16>(w2bf, torch::kBFloat16, 10 * 2048, "w2bf")),
                      stream());
}

}  // namespace

namespace p2cnn {
void init_attributes();
}

void register_cnn(pybind11::module& m) {
  auto c = m.def_submodule("cnn", "fused MNIST-CNN training step kernels");
  c.def("init", &p2cnn::init_attributes, "set kernel attributes (call before HIP graph capture)");
  c.def("conv1_fwd", &k_conv1_fwd);
  c.def("conv2_fwd", &k_conv2_fwd);
  c.def("conv12_fwd", &k_conv12_fwd);
  c.def("gemm_skinny", &k_gemm_skinny);
  c.def("head", &k_head, pybind11::arg("slabs"), pybind11::arg("S"), pybind11::arg("mrows"), pybind11::arg("params"),
        pybind11::arg("off"), pybind11::arg("labels"), pybind11::arg("idx"), pybind11::arg("B"), pybind11::arg("train"),
        pybind11::arg("H"), pybind11::arg("dH"), pybind11::arg("dlogits"), pybind11::arg("stats"),
        pybind11::arg("w2bf") = pybind11::none());
  c.def("route_fc2", &k_route_fc2, pybind11::arg("dH"), pybind11::arg("w1"), pybind11::arg("am2"), pybind11::arg("mrows"), pybind11::arg("B"),
        pybind11::arg("dc2m"), pybind11::arg("gb"), pybind11::arg("dlogits"), pybind11::arg("H"), pybind11::arg("params"), pybind11::arg("m"), pybind11::arg("v"),
        pybind11::arg("gdump"), pybind11::arg("off"), pybind11::arg("adam_t"), pybind11::arg("t_off"), pybind11::arg("lr"), pybind11::arg("b1"),
        pybind11::arg("b2"), pybind11::arg("eps"), pybind11::arg("wd"), pybind11::arg("with_fc2") = true, pybind11::arg("row_major") = false,
        pybind11::arg("ws") = pybind11::none(), pybind11::arg("ctr") = pybind11::none());
  c.def("fc1_wgrad_adam", &k_fc1_wgrad_adam);
  c.def("conv2_bwd", &k_conv2_bwd);
  c.def("conv_adam", &k_conv_adam);
  c.def("fc1_conv_adam", &k_fc1_conv_adam, pybind11::arg("dH"), pybind11::arg("a1"), pybind11::arg("mrows"), pybind11::arg("wslab1"),
        pybind11::arg("wslab2"), pybind11::arg("gb"), pybind11::arg("B"), pybind11::arg("params"), pybind11::arg("m"), pybind11::arg("v"), pybind11::arg("gdump"),
        pybind11::arg("w1bf"), pybind11::arg("w1tbf"), pybind11::arg("w2r"), pybind11::arg("w2q"), pybind11::arg("off"), pybind11::arg("adam_t"),
        pybind11::arg("t_off"), pybind11::arg("lr"), pybind11::arg("b1"), pybind11::arg("b2"), pybind11::arg("eps"), pybind11::arg("wd"),
        pybind11::arg("dlogits") = pybind11::none(), pybind11::arg("H") = pybind11::none(),
        pybind11::arg("w2bf") = pybind11::none());
  c.def("fc1_conv_adam_fwd", &k_fc1_conv_adam_fwd);
  c.def("pack_shadows", &k_pack_shadows, pybind11::arg("params"), pybind11::arg("off"), pybind11::arg("w2r"),
        pybind11::arg("w2q"), pybind11::arg("w1bf"), pybind11::arg("w1tbf"), pybind11::arg("w2bf") = pybind11::none());
  c.def("wgrad_groups", [](int64_t B) { return int64_t(p2cnn::wgrad_groups(int(B))); },
        "conv2 weight-gradient partial slabs (of 51200 floats) written for a batch of B");
}
