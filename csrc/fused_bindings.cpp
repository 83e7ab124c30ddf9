// PyTorch bindings of the fused transformer / classifier ops (fused_ops.hip).
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

#include <cmath>

#include "attention.h"
#include "fused_ops.h"

namespace {

hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

bool act_dtype(const torch::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), name, " must be a contiguous GPU tensor");
  TORCH_CHECK(t.scalar_type() == torch::kBFloat16 || t.scalar_type() == torch::kFloat32, name, " must be bf16 or fp32");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name, " must be 16-byte aligned");
  return t.scalar_type() == torch::kBFloat16;
}

void check_f32(const torch::Tensor& t, int64_t n, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.scalar_type() == torch::kFloat32, name, " must be contiguous fp32 on GPU");
  TORCH_CHECK(t.numel() >= n, name, " too small");
}

// uint8 [B, C, H, W] -> bf16 [B, (H/P)(W/P), C P P] / 255
torch::Tensor patchify_u8(torch::Tensor x, int64_t P) {
  const c10::DeviceGuard g(x.device());
  TORCH_CHECK(x.is_cuda() && x.is_contiguous() && x.scalar_type() == torch::kUInt8 && x.dim() == 4,
              "patchify_u8: x must be a contiguous uint8 [B, C, H, W] GPU tensor");
  const int64_t B = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(P > 0 && P % 8 == 0 && H % P == 0 && W % P == 0, "patchify_u8: P % 8 == 0 and P | H, W");
  auto out = torch::empty({B, (H / P) * (W / P), C * P * P}, x.options().dtype(torch::kBFloat16));
  if (out.numel() > 0)
    p2fused::patchify_u8(x.data_ptr<uint8_t>(), reinterpret_cast<uint16_t*>(out.data_ptr()), int(B), int(C), int(H),
                         int(W), int(P), stream());
  return out;
}

void check_bf16(const torch::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.scalar_type() == torch::kBFloat16 &&
                  reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0,
              name, " must be a contiguous 16-byte aligned bf16 GPU tensor");
}

// y [B, N, D], cls [D], pos [N + 1, D] (bf16) -> h [B, N + 1, D]
torch::Tensor embed_tokens_fwd(torch::Tensor y, torch::Tensor cls, torch::Tensor pos) {
  const c10::DeviceGuard g(y.device());
  check_bf16(y, "y");
  check_bf16(cls, "cls");
  check_bf16(pos, "pos");
  TORCH_CHECK(y.dim() == 3, "embed_tokens: y must be [B, N, D]");
  const int64_t B = y.size(0), N = y.size(1), D = y.size(2);
  TORCH_CHECK(D % 8 == 0 && cls.numel() == D && pos.numel() == (N + 1) * D, "embed_tokens: shapes");
  TORCH_CHECK(cls.device() == y.device() && pos.device() == y.device(), "embed_tokens: devices");
  auto h = torch::empty({B, N + 1, D}, y.options());
  if (h.numel() > 0)
    p2fused::embed_tokens_fwd(reinterpret_cast<const uint16_t*>(y.data_ptr()), reinterpret_cast<const uint16_t*>(cls.data_ptr()),
                              reinterpret_cast<const uint16_t*>(pos.data_ptr()), reinterpret_cast<uint16_t*>(h.data_ptr()),
                              int(B), int(N), int(D), stream());
  return h;
}

// dh [B, N + 1, D] -> (dy [B, N, D], dpos [N + 1, D], dcls [D])
std::vector<torch::Tensor> embed_tokens_bwd(torch::Tensor dh) {
  const c10::DeviceGuard g(dh.device());
  check_bf16(dh, "dh");
  TORCH_CHECK(dh.dim() == 3 && dh.size(1) >= 1 && dh.size(2) % 8 == 0, "embed_tokens_bwd: dh must be [B, N + 1, D]");
  const int64_t B = dh.size(0), N = dh.size(1) - 1, D = dh.size(2);
  auto dy = torch::empty({B, N, D}, dh.options());
  auto dpos = torch::empty({N + 1, D}, dh.options());
  auto dcls = torch::empty({D}, dh.options());
  if (dpos.numel() > 0)
    p2fused::embed_tokens_bwd(reinterpret_cast<const uint16_t*>(dh.data_ptr()), reinterpret_cast<uint16_t*>(dy.data_ptr()),
                              reinterpret_cast<uint16_t*>(dpos.data_ptr()), reinterpret_cast<uint16_t*>(dcls.data_ptr()),
                              int(B), int(N), int(D), stream());
  return {dy, dpos, dcls};
}

std::vector<torch::Tensor> ln_fwd(torch::Tensor x, torch::Tensor w, torch::Tensor b, double eps,
                                  c10::optional<torch::Tensor> residual) {
  const c10::DeviceGuard g(x.device());
  TORCH_CHECK(x.dim() == 2, "x must be [N, C]");
  const int64_t N = x.size(0), C = x.size(1);
  TORCH_CHECK(C % 8 == 0 && C <= p2fused::kMaxLnCols, "C must be a multiple of 8 and <= 2048");
  const bool bf = act_dtype(x, "x");
  check_f32(w, C, "weight");
  check_f32(b, C, "bias");
  const bool has_res = residual.has_value() && residual->defined();
  if (has_res) {
    act_dtype(*residual, "residual");
    TORCH_CHECK(residual->sizes() == x.sizes() && residual->scalar_type() == x.scalar_type(), "residual must match x");
  }
  auto y = torch::empty_like(x);
  auto sum = has_res ? torch::empty_like(x) : torch::Tensor();
  auto opt = x.options().dtype(torch::kFloat32);
  auto mean = torch::empty({N}, opt), rstd = torch::empty({N}, opt);
  if (N > 0)
    p2fused::layer_norm_fwd(bf, x.data_ptr(), has_res ? residual->data_ptr() : nullptr, w.data_ptr<float>(),
                            b.data_ptr<float>(), y.data_ptr(), has_res ? sum.data_ptr() : nullptr,
                            mean.data_ptr<float>(), rstd.data_ptr<float>(), int(N), int(C), float(eps), stream());
  if (has_res) return {y, mean, rstd, sum};
  return {y, mean, rstd};
}

std::vector<torch::Tensor> ln_bwd(torch::Tensor dy, torch::Tensor x, torch::Tensor w, torch::Tensor mean,
                                  torch::Tensor rstd, c10::optional<torch::Tensor> gsum) {
  const c10::DeviceGuard g(x.device());
  const int64_t N = x.size(0), C = x.size(1);
  TORCH_CHECK(dy.sizes() == x.sizes() && dy.scalar_type() == x.scalar_type(), "dy must match x");
  const bool bf = act_dtype(x, "x");
  act_dtype(dy, "dy");
  check_f32(w, C, "weight");
  check_f32(mean, N, "mean");
  check_f32(rstd, N, "rstd");
  const bool has_gs = gsum.has_value() && gsum->defined();
  if (has_gs) {
    act_dtype(*gsum, "gsum");
    TORCH_CHECK(gsum->sizes() == x.sizes() && gsum->scalar_type() == x.scalar_type(), "gsum must match x");
  }
  auto dx = torch::empty_like(x);
  auto opt = x.options().dtype(torch::kFloat32);
  auto dw = torch::empty({C}, opt), db = torch::empty({C}, opt);  // col_reduce writes every column
  if (N > 0) {
    const int G = p2fused::layer_norm_bwd_blocks(int(N));
    auto pdw = torch::empty({G, C}, opt), pdb = torch::empty({G, C}, opt);
    p2fused::layer_norm_bwd(bf, dy.data_ptr(), x.data_ptr(), w.data_ptr<float>(), mean.data_ptr<float>(),
                            rstd.data_ptr<float>(), has_gs ? gsum->data_ptr() : nullptr, dx.data_ptr(),
                            pdw.data_ptr<float>(), pdb.data_ptr<float>(), dw.data_ptr<float>(), db.data_ptr<float>(),
                            int(N), int(C), stream());
  } else {
    dw.zero_();
    db.zero_();
  }
  return {dx, dw, db};
}

// The backward passes above without their column reduction: the partials are returned
// and reduced later, many at a time, by col_reduce_multi (a training step's deferred
// parameter-gradient reductions, ops/fused.py deferred_param_grads).
std::vector<torch::Tensor> ln_bwd_parts(torch::Tensor dy, torch::Tensor x, torch::Tensor w, torch::Tensor mean,
                                        torch::Tensor rstd, c10::optional<torch::Tensor> gsum) {
  const c10::DeviceGuard g(x.device());
  const int64_t N = x.size(0), C = x.size(1);
  TORCH_CHECK(N > 0, "ln_bwd_parts: empty input");
  TORCH_CHECK(dy.sizes() == x.sizes() && dy.scalar_type() == x.scalar_type(), "dy must match x");
  const bool bf = act_dtype(x, "x");
  act_dtype(dy, "dy");
  check_f32(w, C, "weight");
  check_f32(mean, N, "mean");
  check_f32(rstd, N, "rstd");
  const bool has_gs = gsum.has_value() && gsum->defined();
  if (has_gs)
    TORCH_CHECK(gsum->sizes() == x.sizes() && gsum->scalar_type() == x.scalar_type(), "gsum must match x");
  auto dx = torch::empty_like(x);
  auto opt = x.options().dtype(torch::kFloat32);
  const int G = p2fused::layer_norm_bwd_blocks(int(N));
  auto pdw = torch::empty({G, C}, opt), pdb = torch::empty({G, C}, opt);
  p2fused::layer_norm_bwd(bf, dy.data_ptr(), x.data_ptr(), w.data_ptr<float>(), mean.data_ptr<float>(),
                          rstd.data_ptr<float>(), has_gs ? gsum->data_ptr() : nullptr, dx.data_ptr(),
                          pdw.data_ptr<float>(), pdb.data_ptr<float>(), nullptr, nullptr, int(N), int(C), stream());
  return {dx, pdw, pdb};
}

std::vector<torch::Tensor> bias_gelu_bwd_parts(torch::Tensor dy, torch::Tensor x, torch::Tensor b) {
  const c10::DeviceGuard g(x.device());
  const int64_t H = x.size(-1), N = x.numel() / H;
  TORCH_CHECK(N > 0, "bias_gelu_bwd_parts: empty input");
  TORCH_CHECK(dy.sizes() == x.sizes() && dy.scalar_type() == x.scalar_type(), "dy must match x");
  const bool bf = act_dtype(x, "x");
  act_dtype(dy, "dy");
  check_f32(b, H, "bias");
  auto dx = torch::empty_like(x);
  auto pdb = torch::empty({p2fused::bias_gelu_bwd_splits(int(N)), H}, x.options().dtype(torch::kFloat32));
  p2fused::bias_gelu_bwd(bf, dy.data_ptr(), x.data_ptr(), b.data_ptr<float>(), dx.data_ptr(), pdb.data_ptr<float>(),
                         nullptr, int(N), int(H), stream());
  return {dx, pdb};
}

torch::Tensor column_sum_parts(torch::Tensor x) {
  const c10::DeviceGuard g(x.device());
  TORCH_CHECK(x.dim() == 2 && x.size(0) > 0, "x must be a non-empty [N, H]");
  const int64_t N = x.size(0), H = x.size(1);
  TORCH_CHECK(H % 8 == 0, "H must be a multiple of 8");
  const bool bf = act_dtype(x, "x");
  auto part = torch::empty({p2fused::bias_gelu_bwd_splits(int(N)), H}, x.options().dtype(torch::kFloat32));
  p2fused::column_sum(bf, x.data_ptr(), part.data_ptr<float>(), nullptr, nullptr, int(N), int(H), stream());
  return part;
}

// parts[i] = the [S, H] column partials of xs[i] (bf16 [N, H], N > 0), many per launch
void column_sum_parts_multi(std::vector<torch::Tensor> xs, std::vector<torch::Tensor> parts) {
  TORCH_CHECK(xs.size() == parts.size(), "column_sum_parts_multi: xs / parts length mismatch");
  if (xs.empty()) return;
  const c10::DeviceGuard g(xs[0].device());
  p2fused::CsJobs jobs{};
  for (size_t i = 0; i < xs.size(); ++i) {
    const auto& x = xs[i];
    const auto& pt = parts[i];
    TORCH_CHECK(x.is_cuda() && x.scalar_type() == torch::kBFloat16 && x.dim() == 2 && x.stride(1) == 1 &&
                    x.stride(0) == x.size(1) && x.size(0) > 0 && x.size(1) % 8 == 0 &&
                    reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0,
                "column_sum_parts_multi: xs must be contiguous, 16-byte aligned bf16 [N, H] (H % 8 == 0)");
    const int N = int(x.size(0)), H = int(x.size(1)), S = p2fused::bias_gelu_bwd_splits(N);
    TORCH_CHECK(pt.is_cuda() && pt.scalar_type() == torch::kFloat32 && pt.is_contiguous() && pt.dim() == 2 &&
                    pt.size(0) == S && pt.size(1) == H && pt.device() == x.device() && x.device() == xs[0].device(),
                "column_sum_parts_multi: parts[i] must be contiguous fp32 [bias_gelu_bwd_splits(N), H] on xs' device");
    jobs.j[jobs.n++] = p2fused::CsJob{reinterpret_cast<const uint16_t*>(x.data_ptr<at::BFloat16>()),
                                      pt.data_ptr<float>(), N, H, S, 0};
    if (jobs.n == p2fused::kCsMaxJobs || i + 1 == xs.size()) {
      p2fused::colsum_multi(jobs, stream());
      jobs.n = 0;
    }
  }
}

int64_t colsum_splits(int64_t N) { return p2fused::bias_gelu_bwd_splits(int(N)); }

// outs[i] (fp32 or bf16 [C]) = column sums of parts[i] (fp32 [R, C]), up to kCrMaxJobs per launch
void col_reduce_multi(std::vector<torch::Tensor> parts, std::vector<torch::Tensor> outs) {
  TORCH_CHECK(parts.size() == outs.size(), "col_reduce_multi: parts / outs length mismatch");
  if (parts.empty()) return;
  const c10::DeviceGuard g(parts[0].device());
  p2fused::CrJobs jobs{};
  for (size_t i = 0; i < parts.size(); ++i) {
    const auto& a = parts[i];
    const auto& o = outs[i];
    TORCH_CHECK(a.is_cuda() && a.scalar_type() == torch::kFloat32 && a.dim() == 2 && a.is_contiguous() && a.size(0) > 0,
                "col_reduce_multi: parts must be non-empty contiguous fp32 [R, C] GPU tensors");
    TORCH_CHECK(a.device() == parts[0].device() && o.device() == a.device(), "col_reduce_multi: one device");
    TORCH_CHECK(o.is_contiguous() && o.numel() == a.size(1) &&
                    (o.scalar_type() == torch::kFloat32 || o.scalar_type() == torch::kBFloat16),
                "col_reduce_multi: outs must be contiguous fp32 / bf16 [C] matching their partials");
    const bool bf = o.scalar_type() == torch::kBFloat16;
    jobs.j[jobs.n++] = p2fused::CrJob{a.data_ptr<float>(), bf ? nullptr : o.data_ptr<float>(), nullptr, nullptr,
                                      bf ? reinterpret_cast<uint16_t*>(o.data_ptr<at::BFloat16>()) : nullptr,
                                      int(a.size(0)), int(a.size(1)), 0, 0};
    if (jobs.n == p2fused::kCrMaxJobs || i + 1 == parts.size()) {
      p2fused::col_reduce_multi(jobs, stream());
      jobs.n = 0;
    }
  }
}

torch::Tensor split_sum_bf16(torch::Tensor parts) {
  const c10::DeviceGuard g(parts.device());
  TORCH_CHECK(parts.is_cuda() && parts.scalar_type() == torch::kBFloat16 && parts.is_contiguous() && parts.dim() >= 2,
              "parts must be a contiguous bf16 [S, ...] GPU tensor");
  const int64_t S = parts.size(0), n = parts.numel() / std::max<int64_t>(S, 1);
  TORCH_CHECK(S >= 1 && n % 8 == 0, "split_sum_bf16: S >= 1 and a multiple-of-8 slice required");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(parts.data_ptr()) % 16 == 0, "parts must be 16-byte aligned");
  auto out = torch::empty(parts.sizes().slice(1), parts.options());
  if (n > 0)
    p2fused::split_sum_bf16(reinterpret_cast<const uint16_t*>(parts.data_ptr<at::BFloat16>()),
                            reinterpret_cast<uint16_t*>(out.data_ptr<at::BFloat16>()), n, int(S), stream());
  return out;
}

torch::Tensor column_sum(torch::Tensor x, bool bf16_out) {
  const c10::DeviceGuard g(x.device());
  TORCH_CHECK(x.dim() == 2, "x must be [N, H]");
  const int64_t N = x.size(0), H = x.size(1);
  TORCH_CHECK(H % 8 == 0, "H must be a multiple of 8");
  const bool bf = act_dtype(x, "x");
  auto opt = x.options().dtype(torch::kFloat32);
  auto out = torch::empty({H}, bf16_out ? x.options().dtype(torch::kBFloat16) : opt);
  if (N > 0) {
    auto part = torch::empty({p2fused::bias_gelu_bwd_splits(int(N)), H}, opt);
    p2fused::column_sum(bf, x.data_ptr(), part.data_ptr<float>(), bf16_out ? nullptr : out.data_ptr<float>(),
                        bf16_out ? reinterpret_cast<uint16_t*>(out.data_ptr<at::BFloat16>()) : nullptr, int(N), int(H),
                        stream());
  } else {
    out.zero_();
  }
  return out;
}

torch::Tensor bias_gelu_fwd(torch::Tensor x, torch::Tensor b) {
  const c10::DeviceGuard g(x.device());
  const int64_t H = x.size(-1);
  TORCH_CHECK(H % 8 == 0, "last dim must be a multiple of 8");
  const bool bf = act_dtype(x, "x");
  check_f32(b, H, "bias");
  auto y = torch::empty_like(x);
  if (x.numel() > 0) p2fused::bias_gelu_fwd(bf, x.data_ptr(), b.data_ptr<float>(), y.data_ptr(), x.numel(), int(H), stream());
  return y;
}

std::vector<torch::Tensor> bias_gelu_bwd(torch::Tensor dy, torch::Tensor x, torch::Tensor b) {
  const c10::DeviceGuard g(x.device());
  const int64_t H = x.size(-1), N = x.numel() / H;
  TORCH_CHECK(dy.sizes() == x.sizes() && dy.scalar_type() == x.scalar_type(), "dy must match x");
  const bool bf = act_dtype(x, "x");
  act_dtype(dy, "dy");
  check_f32(b, H, "bias");
  auto dx = torch::empty_like(x);
  auto db = torch::empty({H}, x.options().dtype(torch::kFloat32));  // col_reduce writes every column
  if (N > 0) {
    auto pdb = torch::empty({p2fused::bias_gelu_bwd_splits(int(N)), H}, x.options().dtype(torch::kFloat32));
    p2fused::bias_gelu_bwd(bf, dy.data_ptr(), x.data_ptr(), b.data_ptr<float>(), dx.data_ptr(), pdb.data_ptr<float>(),
                           db.data_ptr<float>(), int(N), int(H), stream());
  } else {
    db.zero_();
  }
  return {dx, db};
}

std::vector<torch::Tensor> xent_fwd(torch::Tensor z, torch::Tensor y) {
  const c10::DeviceGuard g(z.device());
  TORCH_CHECK(z.dim() == 2, "logits must be [N, K]");
  TORCH_CHECK(y.is_cuda() && y.scalar_type() == torch::kInt64 && y.is_contiguous() && y.numel() == z.size(0),
              "labels must be int64 [N] on the GPU");
  const bool bf = act_dtype(z, "logits");
  const int64_t N = z.size(0), K = z.size(1);
  auto opt = z.options().dtype(torch::kFloat32);
  auto loss = torch::empty({N}, opt), lse = torch::empty({N}, opt);
  if (N > 0) p2fused::xent_fwd(bf, z.data_ptr(), y.data_ptr<int64_t>(), loss.data_ptr<float>(), lse.data_ptr<float>(), int(N), int(K), stream());
  return {loss, lse};
}

torch::Tensor xent_bwd(torch::Tensor z, torch::Tensor y, torch::Tensor lse, torch::Tensor gscale) {
  const c10::DeviceGuard g(z.device());
  const bool bf = act_dtype(z, "logits");
  const int64_t N = z.size(0), K = z.size(1);
  check_f32(lse, N, "lse");
  check_f32(gscale, 1, "grad");
  auto dz = torch::empty_like(z);
  if (N > 0)
    p2fused::xent_bwd(bf, z.data_ptr(), y.data_ptr<int64_t>(), lse.data_ptr<float>(), gscale.data_ptr<float>(),
                      dz.data_ptr(), int(N), int(K), stream());
  return dz;
}

// ---- fused attention over the QKV projection output --------------------------
p2attn::AttnShape attn_shape(const torch::Tensor& qkv, int64_t heads) {
  TORCH_CHECK(qkv.is_cuda() && qkv.is_contiguous() && qkv.scalar_type() == torch::kBFloat16 && qkv.dim() == 3,
              "qkv must be a contiguous bf16 [B, T, 3C] GPU tensor");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(qkv.data_ptr()) % 16 == 0, "qkv must be 16-byte aligned");
  const int64_t B = qkv.size(0), T = qkv.size(1), C3 = qkv.size(2);
  TORCH_CHECK(C3 % 3 == 0 && heads > 0 && (C3 / 3) == heads * p2attn::kHeadDim, "qkv last dim must be 3 * heads * 64");
  TORCH_CHECK(T >= 1 && T <= p2attn::kMaxT, "attention kernel supports 1..256 tokens");
  TORCH_CHECK(B <= 65535 && heads <= 65535, "grid limits");
  p2attn::AttnShape sh{};
  sh.B = int(B);
  sh.H = int(heads);
  sh.T = int(T);
  sh.C = int(C3 / 3);
  sh.qkv_row = C3;
  sh.qkv_batch = T * C3;
  sh.o_row = sh.C;
  sh.o_batch = T * sh.C;
  sh.scale = float(1.0 / std::sqrt(double(p2attn::kHeadDim)));
  return sh;
}

std::vector<torch::Tensor> attn_fwd(torch::Tensor qkv, int64_t heads) {
  const c10::DeviceGuard g(qkv.device());
  const auto sh = attn_shape(qkv, heads);
  auto o = torch::empty({qkv.size(0), qkv.size(1), int64_t(sh.C)}, qkv.options());
  auto lse = torch::empty({qkv.size(0), heads, qkv.size(1)}, qkv.options().dtype(torch::kFloat32));
  if (sh.B > 0)
    p2attn::attention_fwd(reinterpret_cast<const uint16_t*>(qkv.data_ptr()), reinterpret_cast<uint16_t*>(o.data_ptr()),
                          lse.data_ptr<float>(), sh, stream());
  return {o, lse};
}

torch::Tensor attn_bwd(torch::Tensor qkv, torch::Tensor o, torch::Tensor dout, torch::Tensor lse, int64_t heads) {
  const c10::DeviceGuard g(qkv.device());
  const auto sh = attn_shape(qkv, heads);
  for (auto* t : {&o, &dout}) {
    TORCH_CHECK(t->is_cuda() && t->is_contiguous() && t->scalar_type() == torch::kBFloat16 && t->dim() == 3 &&
                    t->size(0) == sh.B && t->size(1) == sh.T && t->size(2) == sh.C,
                "o / dout must be contiguous bf16 [B, T, C]");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "o / dout must be 16-byte aligned");
  }
  TORCH_CHECK(lse.is_cuda() && lse.is_contiguous() && lse.scalar_type() == torch::kFloat32 &&
                  lse.numel() == int64_t(sh.B) * sh.H * sh.T,
              "lse must be the forward's fp32 [B, H, T]");
  auto dqkv = torch::empty_like(qkv);
  if (sh.B > 0)
    p2attn::attention_bwd(reinterpret_cast<const uint16_t*>(qkv.data_ptr()), reinterpret_cast<const uint16_t*>(o.data_ptr()),
                          reinterpret_cast<const uint16_t*>(dout.data_ptr()), lse.data_ptr<float>(),
                          reinterpret_cast<uint16_t*>(dqkv.data_ptr()), sh, stream());
  return dqkv;
}

// dsts[i] <- srcs[i] for every pair, one launch (same byte size per pair, any dtype)
void multi_copy(std::vector<torch::Tensor> dsts, std::vector<torch::Tensor> srcs) {
  TORCH_CHECK(dsts.size() == srcs.size() && !dsts.empty() && int(dsts.size()) <= p2fused::kMaxCopies,
              "multi_copy: 1..", p2fused::kMaxCopies, " (dst, src) pairs");
  const c10::DeviceGuard g(dsts[0].device());
  p2fused::CopyList cl{};
  cl.n = int(dsts.size());
  for (int i = 0; i < cl.n; ++i) {
    const auto &d = dsts[i], &s = srcs[i];
    TORCH_CHECK(d.is_cuda() && s.is_cuda() && d.device() == s.device() && d.device() == dsts[0].device(),
                "multi_copy: tensors must be on one GPU");
    TORCH_CHECK(d.is_contiguous() && s.is_contiguous(), "multi_copy: tensors must be contiguous");
    const int64_t nb = d.numel() * d.element_size();
    TORCH_CHECK(nb == s.numel() * s.element_size() && nb % 4 == 0, "multi_copy: pair ", i, " byte sizes differ or not % 4");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(d.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(s.data_ptr()) % 16 == 0,
                "multi_copy: pair ", i, " not 16-byte aligned");
    cl.dst[i] = d.data_ptr();
    cl.src[i] = s.data_ptr();
    cl.bytes[i] = nb;
  }
  p2fused::multi_copy(cl, stream());
}

}  // namespace

void register_fused(pybind11::module& m) {
  auto f = m.def_submodule("fused", "fused LayerNorm / bias+GELU / softmax cross-entropy kernels");
  f.def("patchify_u8", &patchify_u8, "uint8 images -> bf16 ViT patch rows / 255", pybind11::arg("x"), pybind11::arg("P"));
  f.def("embed_tokens_fwd", &embed_tokens_fwd, "cat(cls, y) + pos in one pass (bf16)");
  f.def("embed_tokens_bwd", &embed_tokens_bwd, "dy = dh[:, 1:], dpos = sum_b dh, dcls = dpos[0]");
  f.def("ln_fwd", &ln_fwd, pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("b"), pybind11::arg("eps"),
        pybind11::arg("residual") = pybind11::none());
  f.def("ln_bwd", &ln_bwd, pybind11::arg("dy"), pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("mean"),
        pybind11::arg("rstd"), pybind11::arg("gsum") = pybind11::none());
  f.def("column_sum", &column_sum, "column sums of a [N, H] bf16/fp32 activation (linear bias gradient), fp32 or bf16 out",
        pybind11::arg("x"), pybind11::arg("bf16_out") = false);
  f.def("ln_bwd_parts", &ln_bwd_parts, "LayerNorm backward: dx and the [G, C] dgamma / dbeta partials");
  f.def("bias_gelu_bwd_parts", &bias_gelu_bwd_parts, "bias+GELU backward: dx and the [S, H] dbias partials");
  f.def("column_sum_parts", &column_sum_parts, "[S, H] partial column sums of a [N, H] activation");
  f.def("col_reduce_multi", &col_reduce_multi, "outs[i] = column sums of parts[i], many per launch");
  f.def("column_sum_parts_multi", &column_sum_parts_multi, "parts[i] = column_sum partials of xs[i], many per launch");
  f.def("colsum_splits", &colsum_splits, "row splits S of column_sum's [S, H] partials for N rows");
  f.def("multi_copy", &multi_copy, "dsts[i] <- srcs[i] for up to 12 pairs in one launch");
  f.def("split_sum_bf16", &split_sum_bf16, "bf16 sum over dim 0 of [S, ...] bf16 partials, fp32 accumulation");
  f.def("bias_gelu_fwd", &bias_gelu_fwd);
  f.def("bias_gelu_bwd", &bias_gelu_bwd);
  f.def("xent_fwd", &xent_fwd);
  f.def("xent_bwd", &xent_bwd);
  f.def("attn_fwd", &attn_fwd, "fused MHSA forward over [B, T, 3C] qkv (head dim 64, T <= 256) -> (o, lse)");
  f.def("attn_bwd", &attn_bwd, "fused MHSA backward -> dqkv [B, T, 3C]");
}
