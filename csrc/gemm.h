// Host launch API of the hand-written MFMA GEMM (csrc/gemm.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace p2 {

// C[M][N] = sum_k A(m, k) * B(n, k) over bf16 operands, fp32 accumulation.
//   A(m, k) = a[m * lda + k] when a_kmajor, else a[k * lda + m]
//   B(n, k) = b[n * ldb + k] when b_kmajor, else b[k * ldb + n]
// (nn.Linear forward: A = x [M][K], B = W [N][K], both k-major; dgrad:
//  B = W read n-major; wgrad: both operands m/n-major.)
// Epilogue, in order: + bias[n] (fp32 or bf16), GELU (writes the
// pre-activation to `z` if given), + residual[m][n] (bf16); C is bf16 or
// fp32.  With splits > 1 every K-slice writes its raw fp32 partial to
// c + slice * M * N instead (no epilogue; reduce afterwards) -- or, when
// `counters` is given, to the workspace `ws` ([splits][M][N] fp32), and the
// last slice to finish a tile reduces the tile in the same launch and runs
// the epilogue into c.  `counters` holds one int per output tile, zero
// before the launch; the kernel leaves it zero again.
// BatchNorm training statistics emitted by a GEMM / convolution epilogue (bf16 C
// only): every output tile writes per-column (mean, M2) of its bf16-rounded
// values as a partial; the last tile of a group of 16 tile-rows combines its
// group (Chan's parallel formula, fixed order), the last group finalizes the
// column: batch mean / rstd, the apply coefficients [mean | w * rstd | b] of
// csrc/batchnorm.hip, running statistics (momentum, unbiased variance) and
// num_batches_tracked.  `part` holds (tiles_m + groups) * 2 * N floats; `cnt`
// tiles_n * (groups + 1) ints, zero before the launch and left zero.
struct BnEpi {
  float* part;
  int* cnt;
  const float* w;
  const float* b;
  float* run_mean;  // optional (no running statistics when null)
  float* run_var;
  int64_t* nbt;     // optional
  float* mean;      // [N] out
  float* rstd;      // [N] out
  float* coef;      // [3N] out
  float eps, momentum;
  // Backward mode (bx != null): C is dz, the gradient w.r.t. the output of an
  // act(bn(x)) whose input x = bx and output (for the ReLU mask) = by (null: no
  // ReLU) are bf16 [M][N]; the launch reduces s1 = sum dz', s2 = sum dz' (x -
  // bmean) with dz' = dz * (by > 0), and the finalize writes dw = rstd * s2,
  // db = s1 and coef = [A | B | D] of csrc/batchnorm.hip's apply_bwd
  // (dx = A dz' + B (x - mean) + D) instead of the forward outputs.
  const uint16_t* bx;
  const uint16_t* by;
  const float* bmean;
  const float* brstd;
  float* dw;
  float* db;
  // measurement knob (P2_BN_EPI_MODE, read once by the conv launcher): 0 = full
  // epilogue; 1 = per-tile statistics only (no cross-tile reduction: outputs are
  // not finalized); 2 = statistics + partial stores + first-level ticket only
  int mode;
};

struct GemmParams {
  const uint16_t* a;
  const uint16_t* b;
  void* c;
  int64_t lda, ldb, ldc;
  int M, N, K;
  int a_kmajor, b_kmajor;
  int c_bf16;
  const void* bias;
  int bias_bf16;
  int gelu;
  uint16_t* z;  // GELU pre-activation output (bf16, ldc), optional
  const uint16_t* residual;  // bf16 [M][ldc], optional
  int splits;
  float* ws;      // split-K workspace for the in-launch reduction
  int* counters;  // per-tile arrival counters (see above), or null
  BnEpi bn;       // BatchNorm statistics epilogue when bn.part != null
  int variant;  // tuning experiments: bit0 setprio around MFMAs, bit1 A-panel tile order, bit2 no XCD remap, bit3 single LDS buffer (4 workgroups / CU), bit4/bit5 timing probes (no stores / no K loop), bit6 256 x 256 tile (8 waves), bit7 no DMA after the prologue (probe), bit8 legacy panel tile order instead of grouped (bit1 then picks A- vs B-panel order), bits 9-10 where the double-buffer prefetch is issued (0 before the K-tile's fragment reads, 1 after the first ones, 2 one chunk per k-substep), bit11 the ping-pong 256 x 256 pipeline of gemm_pp.hip (continuous per-phase DMA, staggered wave halves); with bit 11, bits 12-15 are the ping-pong kernel's timing probes (gemm_pp.hip).  Bit 12 is also the conv kernels' 4-stage ring (conv.hip), whose split-K slabs are 128 x 128 tiles
};

// conv.hip variant bit 14: 64 x 64 output tiles (gemm_core.h Tile64; split-K slabs of that
// geometry, reduced by tile_slab_reduce with the same bit).  The convolutions only -- with
// bit 11 (the ping-pong GEMM) bit 14 is one of its timing probes.
constexpr int kConvT64 = 1 << 14;

void gemm_bf16(const GemmParams& p, hipStream_t s);
// out[M][ldc] = sum of the `splits` fragment-native split-K slabs (gemm_core.h SlabGeom)
// that a launch without counters wrote to `ws`; `variant` = that launch's (tile shape, order)
void tile_slab_reduce(const float* ws, int splits, int M, int N, int64_t ldc, void* out, int out_bf16, int variant,
                      hipStream_t s);
// the ping-pong pipeline (gemm_pp.hip); gemm_bf16 routes variant bit 11 here
bool gemm_pp_supported(const GemmParams& p);
void gemm_bf16_pp(const GemmParams& p, hipStream_t s);

}  // namespace p2
