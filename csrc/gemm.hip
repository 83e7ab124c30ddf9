// Hand-written bf16 MFMA GEMM for the Linear layers (ViT blocks, MLP), gfx950.
//
// One kernel covers the three products of a Linear layer -- forward
// (x . W^T), input gradient (dY . W) and weight gradient (dY^T . x) -- by
// letting each operand be "k-major" (the reduction index contiguous in
// memory) or "mn-major" (the row/column index contiguous), so no operand is
// ever transposed in memory:
//
// * 128 x 128 output tile per 256-thread workgroup, 4 waves as 2 x 2, each
//   wave 64 x 64 = 2 x 2 tiles of v_mfma_f32_32x32x16_bf16, BK = 64; or
//   (variant bit 6) 256 x 256 per 512-thread workgroup, 8 waves as 2 x 4,
//   each 128 x 64 -- half the operand bytes per FLOP, for large products;
//   (variant bit 12) the 128 x 128 tile on a 4-stage LDS ring (3 K-tiles in
//   flight, one workgroup per CU): short-K products, where a double buffer
//   pays the L2/HBM round trip once per K-tile;
// * the pipeline itself lives in gemm_core.h (shared with the implicit-GEMM
//   convolutions of conv.hip); this file instantiates it with plain loaders;
// * operands go HBM -> LDS with global_load_lds (16 B per lane, no VGPR
//   round trip) into a double buffer: the next K-tile's loads are issued
//   before the current tile's MFMAs (one vmcnt(0) + barrier per K-tile);
// * k-major tiles are [128 rows][64 k] (128-B rows) read with ds_read_b128,
//   chunk XOR-swizzled by (row >> 1) & 7 (conflict-free 16-lane reads);
//   mn-major tiles are [64 k][128] (256-B rows) read with the gfx950
//   transpose read ds_read_b64_tr_b16, chunk XOR-swizzled by
//   ((row & 3) << 2 | (row >> 2) & 3) -- the swizzle is applied to the
//   per-lane GLOBAL address so the LDS image stays lane-linear for the DMA;
// * the MFMA is issued as (B, A) so the accumulator holds C with m on the
//   lane and 4 consecutive n per register group: the epilogue writes 8-B
//   (bf16) / 16-B (fp32) vectors along rows, with bias, GELU (+ its
//   pre-activation) and residual add fused;
// * workgroups are remapped so each XCD gets a contiguous run of tiles
//   (bijective for any grid size), and consecutive tiles share a B panel;
// * split-K (fp32 slabs) fills the chip when M x N has few tiles (weight
//   gradients reduce over the 6304 token rows).
//
// The reference has no GEMM of its own (Lightning/torch.nn.Linear); shapes
// from /root/reference/p2pfl/learning/pytorch/mnist_examples/models/mlp.py:53-69
// and the ViT-B config of BASELINE.json.
#include "gemm_core.h"

namespace p2gemm {

template <int NBUF, class LA, class LB, int EPI>
__global__ __launch_bounds__(NT, NBUF == 1 ? 4 : (NBUF == 2 ? 2 : 1)) void gemm_kernel(GemmParams p, LA la, LB lb, int tiles_m, int tiles_n) {
  __shared__ __attribute__((aligned(16))) char smem[smem_bytes<Tile128, NBUF>()];  // [buf][A | B]
  gemm_body<Tile128, NBUF, LA, LB, 0, EPI>(p, la, lb, tiles_m, tiles_n, smem);
}

// 256 x 256 tile, 8 waves, one workgroup per CU (132 KB of LDS, up to 256
// registers per lane at two waves per SIMD).
template <class LA, class LB, int EPI>
__global__ __launch_bounds__(Tile256::NT) void gemm256_kernel(GemmParams p, LA la, LB lb, int tiles_m, int tiles_n) {
  __shared__ __attribute__((aligned(16))) char smem[smem_bytes<Tile256, 2>()];
  gemm_body<Tile256, 2, LA, LB, 0, EPI>(p, la, lb, tiles_m, tiles_n, smem);
}

template <int EPI, class LA, class LB>
static void launch_e(const GemmParams& p, const LA& la, const LB& lb, hipStream_t s) {
  int tm, tn;
  if (p.variant & 64) {
    const int grid = gemm_grid<Tile256>(p, tm, tn);
    hipLaunchKernelGGL((gemm256_kernel<LA, LB, EPI>), dim3(grid), dim3(Tile256::NT), 0, s, p, la, lb, tm, tn);
    return;
  }
  const int grid = gemm_grid<Tile128>(p, tm, tn);
  if (p.variant & 4096)  // 4-stage ring (3 K-tiles in flight), one workgroup per CU: short-K products
    hipLaunchKernelGGL((gemm_kernel<4, LA, LB, EPI>), dim3(grid), dim3(NT), 0, s, p, la, lb, tm, tn);
  else if (p.variant & 8)
    hipLaunchKernelGGL((gemm_kernel<1, LA, LB, EPI>), dim3(grid), dim3(NT), 0, s, p, la, lb, tm, tn);
  else
    hipLaunchKernelGGL((gemm_kernel<2, LA, LB, EPI>), dim3(grid), dim3(NT), 0, s, p, la, lb, tm, tn);
}

template <class LA, class LB>
static void launch(const GemmParams& p, const LA& la, const LB& lb, hipStream_t s) {
  switch (epilogue_kind(p)) {
    case 0: launch_e<0>(p, la, lb, s); break;
    case 2: launch_e<2>(p, la, lb, s); break;
    default: launch_e<1>(p, la, lb, s);
  }
}

}  // namespace p2gemm

namespace p2 {

void gemm_bf16(const GemmParams& p, hipStream_t s) {
  using namespace p2gemm;
  GemmParams q = p;
  if (q.splits < 1) q.splits = 1;
  if ((q.variant & 2048) && gemm_pp_supported(q)) {
    gemm_bf16_pp(q, s);
    return;
  }
  if (p.a_kmajor && p.b_kmajor)
    launch(q, PlainK{p.a, p.lda, p.M, p.K}, PlainK{p.b, p.ldb, p.N, p.K}, s);
  else if (p.a_kmajor)
    launch(q, PlainK{p.a, p.lda, p.M, p.K}, PlainMN{p.b, p.ldb, p.N, p.K}, s);
  else if (p.b_kmajor)
    launch(q, PlainMN{p.a, p.lda, p.M, p.K}, PlainK{p.b, p.ldb, p.N, p.K}, s);
  else
    launch(q, PlainMN{p.a, p.lda, p.M, p.K}, PlainMN{p.b, p.ldb, p.N, p.K}, s);
}

void tile_slab_reduce(const float* ws, int splits, int M, int N, int64_t ldc, void* out, int out_bf16, int variant,
                      hipStream_t s) {
  using namespace p2gemm;
  if (variant & 64) {
    const int tm = (M + 255) / 256, tn = (N + 255) / 256;
    const int64_t groups = int64_t(tm) * tn * (256 * 256 / 4);
    hipLaunchKernelGGL(tile_slab_reduce_kernel<Tile256>, dim3(int((groups + 255) / 256)), dim3(256), 0, s, ws, splits, M,
                       N, ldc, out, out_bf16, variant, tm, tn);
  } else if ((variant & kConvT64) && !(variant & 2048)) {  // the convolutions' 64 x 64 tiles (conv.hip)
    const int tm = (M + 63) / 64, tn = (N + 63) / 64;
    const int64_t groups = int64_t(tm) * tn * (64 * 64 / 4);
    hipLaunchKernelGGL(tile_slab_reduce_kernel<Tile64>, dim3(int((groups + 255) / 256)), dim3(256), 0, s, ws, splits, M,
                       N, ldc, out, out_bf16, variant, tm, tn);
  } else {
    const int tm = (M + 127) / 128, tn = (N + 127) / 128;
    const int64_t groups = int64_t(tm) * tn * (128 * 128 / 4);
    hipLaunchKernelGGL(tile_slab_reduce_kernel<Tile128>, dim3(int((groups + 255) / 256)), dim3(256), 0, s, ws, splits, M,
                       N, ldc, out, out_bf16, variant, tm, tn);
  }
}

}  // namespace p2
