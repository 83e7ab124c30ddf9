// PyTorch bindings of the hand-written MFMA GEMM (p2pfl_amd._C.gemm).
// Shapes, strides, dtypes and alignment are validated on the host before the
// launch: a mismatched call is a Python exception, never a GPU fault.
#include <algorithm>

#include <torch/extension.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>

#include "gemm.h"

namespace {

// fp32 elements of one split-K slice: the fragment-native tiles of the kernel the
// variant selects (gemm_core.h SlabGeom; 256 x 256 for the 256 tile and the
// ping-pong kernel's in-launch reduction), or the ping-pong kernel's row-major
// M x N slabs of a separately reduced launch
int64_t slab_elems(int64_t M, int64_t N, int64_t variant) {
  const int64_t t = (variant & (64 | 2048)) ? 256 : 128;
  return std::max(M * N, ((M + t - 1) / t) * ((N + t - 1) / t) * t * t);
}

void check_bf16_2d(const torch::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == torch::kBFloat16, name, " must be a bf16 GPU tensor");
  TORCH_CHECK(t.dim() == 2 && t.stride(1) == 1, name, " must be 2-D with unit column stride");
  TORCH_CHECK(t.stride(0) % 8 == 0 && reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name,
              " rows must be 16-byte aligned");
}

// a: [M, K] (a_kmajor) or [K, M];  b: [N, K] (b_kmajor) or [K, N];  out: [M, N] bf16/fp32,
// or [splits, M, N] fp32 when splits > 1.
void gemm(torch::Tensor a, torch::Tensor b, bool a_kmajor, bool b_kmajor, torch::Tensor out,
          c10::optional<torch::Tensor> bias, bool gelu, c10::optional<torch::Tensor> z,
          c10::optional<torch::Tensor> residual, int64_t splits, int64_t variant, c10::optional<torch::Tensor> ws,
          c10::optional<torch::Tensor> counters) {
  check_bf16_2d(a, "a");
  check_bf16_2d(b, "b");
  const int64_t M = a_kmajor ? a.size(0) : a.size(1), K = a_kmajor ? a.size(1) : a.size(0);
  const int64_t N = b_kmajor ? b.size(0) : b.size(1), Kb = b_kmajor ? b.size(1) : b.size(0);
  TORCH_CHECK(K == Kb, "gemm: reduction sizes differ (", K, " vs ", Kb, ")");
  TORCH_CHECK(M >= 1 && N >= 8 && K >= 8, "gemm: degenerate shape");
  TORCH_CHECK(N % 8 == 0, "gemm: N must be a multiple of 8 (M=", M, " N=", N, " K=", K, ")");
  TORCH_CHECK((!a_kmajor && !b_kmajor) || K % 8 == 0, "gemm: a k-major operand needs K % 8 == 0 (M=", M, " N=", N,
              " K=", K, ")");
  TORCH_CHECK(a_kmajor || M % 8 == 0, "gemm: an m-major A needs M % 8 == 0");
  TORCH_CHECK(M < (int64_t(1) << 31) && N < (int64_t(1) << 31) && K < (int64_t(1) << 31), "gemm: size overflow");
  TORCH_CHECK(a.device() == b.device() && out.device() == a.device(), "gemm: device mismatch");
  // stream-K schedule of the ping-pong kernel (variant bits 11 + 17): `splits` is its grid size
  const bool sk = (variant & 2048) && (variant & (1 << 17));
  const int64_t sk_iters = ((M + 255) / 256) * ((N + 255) / 256) * ((K + 63) / 64);
  if (variant & 2048) {
    TORCH_CHECK(!((variant & (1 << 21)) && (splits > 1 || sk)), "gemm: the 256 x 128 ping-pong tile takes no split-K / stream-K");
  }
  if (sk) {
    TORCH_CHECK(splits >= 1 && splits <= sk_iters && splits <= 4096,
                "gemm: stream-K grid must be 1..min(4096, tiles x K-tiles = ", sk_iters, ")");
    TORCH_CHECK(counters.has_value() && counters->defined(), "gemm: stream-K needs counters and a workspace");
  } else {
    TORCH_CHECK(splits >= 1 && splits <= 64, "gemm: 1 <= splits <= 64");
  }
  p2::GemmParams p{};
  p.a = reinterpret_cast<const uint16_t*>(a.data_ptr());
  p.b = reinterpret_cast<const uint16_t*>(b.data_ptr());
  p.lda = a.stride(0);
  p.ldb = b.stride(0);
  p.M = int(M);
  p.N = int(N);
  p.K = int(K);
  p.a_kmajor = a_kmajor;
  p.b_kmajor = b_kmajor;
  p.splits = int(splits);
  p.variant = int(variant);
  const bool in_launch = counters.has_value() && counters->defined();
  if (in_launch) {  // split-K reduced inside the launch: slabs in ws, epilogue into out
    TORCH_CHECK(splits > 1 || sk, "gemm: counters only with splits > 1 or stream-K");
    const int64_t tiles = ((M + 127) / 128) * ((N + 127) / 128);
    TORCH_CHECK(counters->is_cuda() && counters->scalar_type() == torch::kInt32 && counters->is_contiguous() &&
                    counters->numel() >= tiles && counters->device() == a.device(),
                "gemm: counters must be a contiguous int32 GPU tensor with one entry per 128x128 tile");
    // stream-K: two 256 x 256 fp32 slabs per workgroup (its first and last tile)
    const int64_t ws_need = sk ? 2 * splits * 65536 : splits * slab_elems(M, N, variant);
    TORCH_CHECK(ws.has_value() && ws->defined() && ws->is_cuda() && ws->scalar_type() == torch::kFloat32 &&
                    ws->is_contiguous() && ws->numel() >= ws_need && ws->device() == a.device() &&
                    reinterpret_cast<uintptr_t>(ws->data_ptr()) % 16 == 0,
                "gemm: split-K workspace must be contiguous fp32 with splits * slab_elems(M, N) elements");
    p.ws = ws->data_ptr<float>();
    p.counters = counters->data_ptr<int>();
  }
  if (splits > 1 && !in_launch && !sk) {
    TORCH_CHECK(out.scalar_type() == torch::kFloat32 && out.is_contiguous() && out.numel() >= splits * slab_elems(M, N, variant),
                "gemm: split-K output must be contiguous fp32 with splits * slab_elems(M, N) elements (reduce with tile_slab_reduce)");
    TORCH_CHECK(!bias.has_value() && !gelu && !residual.has_value(), "gemm: no epilogue with split-K");
    p.ldc = N;
  } else {
    TORCH_CHECK(out.dim() == 2 && out.size(0) == M && out.size(1) == N && out.stride(1) == 1, "gemm: out must be [M, N]");
    TORCH_CHECK(out.scalar_type() == torch::kBFloat16 || out.scalar_type() == torch::kFloat32, "gemm: out bf16 or fp32");
    TORCH_CHECK(out.stride(0) % 4 == 0 && reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0, "gemm: out alignment");
    p.ldc = out.stride(0);
  }
  p.c = out.data_ptr();
  p.c_bf16 = out.scalar_type() == torch::kBFloat16;
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(bias->is_cuda() && bias->is_contiguous() && bias->numel() == N &&
                    (bias->scalar_type() == torch::kFloat32 || bias->scalar_type() == torch::kBFloat16),
                "gemm: bias must be a contiguous fp32/bf16 [N] tensor");
    p.bias = bias->data_ptr();
    p.bias_bf16 = bias->scalar_type() == torch::kBFloat16;
  }
  p.gelu = gelu;
  if (z.has_value() && z->defined()) {
    TORCH_CHECK(gelu, "gemm: z (pre-activation) only with gelu");
    TORCH_CHECK(z->scalar_type() == torch::kBFloat16 && z->dim() == 2 && z->size(0) == M && z->size(1) == N &&
                    z->stride(0) == p.ldc && z->stride(1) == 1,
                "gemm: z must be bf16 [M, N] with out's row stride");
    p.z = reinterpret_cast<uint16_t*>(z->data_ptr());
  }
  if (residual.has_value() && residual->defined()) {
    TORCH_CHECK(residual->scalar_type() == torch::kBFloat16 && residual->dim() == 2 && residual->size(0) == M &&
                    residual->size(1) == N && residual->stride(0) == p.ldc && residual->stride(1) == 1,
                "gemm: residual must be bf16 [M, N] with out's row stride");
    p.residual = reinterpret_cast<const uint16_t*>(residual->data_ptr());
  }
  // the ping-pong kernel does not range-check a k-major K tail: a plain ping-pong request
  // for such a shape runs on the 128 x 128 core kernel (gemm_bf16), but the stream-K
  // schedule has no such fallback (its workspace is sized per workgroup), so refuse it
  TORCH_CHECK(!sk || p2::gemm_pp_supported(p),
              "gemm: the stream-K schedule needs K % 64 == 0 with a k-major operand (M=", M, " N=", N, " K=", K, ")");
  const c10::DeviceGuard guard(a.device());
  p2::gemm_bf16(p, c10::hip::getCurrentHIPStream().stream());
}

// C[M, N] (bf16 / fp32, contiguous) = sum of the `splits` fragment-native slabs in `ws`
// written by a split-K gemm / conv launch without counters with this `variant`.
void tile_slab_reduce(torch::Tensor ws, int64_t splits, int64_t M, int64_t N, torch::Tensor out, int64_t variant) {
  TORCH_CHECK(ws.is_cuda() && ws.scalar_type() == torch::kFloat32 && ws.is_contiguous() &&
                  ws.numel() >= splits * slab_elems(M, N, variant) && reinterpret_cast<uintptr_t>(ws.data_ptr()) % 16 == 0,
              "tile_slab_reduce: ws must be contiguous fp32 with splits * slab_elems(M, N) elements");
  TORCH_CHECK(!(variant & 2048), "tile_slab_reduce: the ping-pong kernel writes row-major slabs");
  TORCH_CHECK(splits >= 1 && M >= 1 && N >= 8 && N % 4 == 0, "tile_slab_reduce: bad shape");
  TORCH_CHECK(out.is_cuda() && out.is_contiguous() && out.numel() == M * N && out.device() == ws.device() &&
                  (out.scalar_type() == torch::kFloat32 || out.scalar_type() == torch::kBFloat16) &&
                  reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0,
              "tile_slab_reduce: out must be contiguous fp32/bf16 with M * N elements");
  const c10::DeviceGuard guard(ws.device());
  p2::tile_slab_reduce(ws.data_ptr<float>(), int(splits), int(M), int(N), N, out.data_ptr(),
                       out.scalar_type() == torch::kBFloat16, int(variant), c10::hip::getCurrentHIPStream().stream());
}

}  // namespace

void register_gemm(pybind11::module& m) {
  m.def("tile_slab_reduce", &tile_slab_reduce, "sum of fragment-native split-K slabs into C", pybind11::arg("ws"),
        pybind11::arg("splits"), pybind11::arg("M"), pybind11::arg("N"), pybind11::arg("out"), pybind11::arg("variant"));
  m.def("gemm", &gemm, "bf16 MFMA GEMM with fused bias/GELU/residual epilogue and split-K",
        pybind11::arg("a"), pybind11::arg("b"), pybind11::arg("a_kmajor"), pybind11::arg("b_kmajor"),
        pybind11::arg("out"), pybind11::arg("bias") = pybind11::none(), pybind11::arg("gelu") = false,
        pybind11::arg("z") = pybind11::none(), pybind11::arg("residual") = pybind11::none(),
        pybind11::arg("splits") = 1, pybind11::arg("variant") = 0, pybind11::arg("ws") = pybind11::none(),
        pybind11::arg("counters") = pybind11::none());
}
