// Shared helpers for p2pfl_amd HIP kernels (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>
#include <stdexcept>

#define P2_DEVICE __device__ __forceinline__

namespace p2 {

constexpr int kWave = 64;

// clang vector types: usable with __builtin_nontemporal_* and MFMA builtins
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

// 16-byte streaming (non-temporal) load: for data read once (weights streamed
// through a GEMM) so it does not evict reused operands from L2/MALL.
P2_DEVICE uint4 ld_nt16(const void* p) {
  const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  return __builtin_bit_cast(uint4, v);
}

// bf16 <-> f32.  f32 -> bf16 is the gfx950 conversion instruction
// (v_cvt_pk_bf16_f32: round-to-nearest-even, NaN stays NaN; MI355X_MICROARCH.md
// correctness table): one instruction per pair.  The bit-level sequence used
// before (add 0x7fff + lsb, plus a branch for NaN) cost ~8 instructions and an
// exec-masked branch per value -- in an unrolled 256 x 256 GEMM epilogue that
// was ~6 KB of code fetched cold by every workgroup.
typedef __bf16 p2_bf16x2_t __attribute__((ext_vector_type(2)));
P2_DEVICE float bf16_to_f32(uint16_t h) { return __uint_as_float(uint32_t(h) << 16); }
P2_DEVICE uint16_t f32_to_bf16(float f) { return __builtin_bit_cast(uint16_t, static_cast<__bf16>(f)); }
P2_DEVICE uint32_t pack_bf16x2(float lo, float hi) {
  const p2_bf16x2_t v = {static_cast<__bf16>(lo), static_cast<__bf16>(hi)};
  return __builtin_bit_cast(uint32_t, v);
}

// Grid size for a grid-stride memory-bound kernel: enough blocks to cover the
// 256 CUs several times over, capped (Guideline 11).
inline int stream_grid(int64_t work_items, int block) {
  int64_t g = (work_items + block - 1) / block;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return int(g);
}

// erf, branch-free: Abramowitz & Stegun 7.1.26, |error| <= 1.5e-7 (plus fp32
// rounding) -- ~12 VALU instructions against ~80 for the library erff, which
// makes GELU epilogues VALU-bound (same form as fused_ops.hip's bias+GELU).
P2_DEVICE float erf_fast(float x) {
  const float a = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, a, 1.f));
  float q = fmaf(1.061405429f, t, -1.453152027f);
  q = fmaf(q, t, 1.421413741f);
  q = fmaf(q, t, -0.284496736f);
  q = fmaf(q, t, 0.254829592f);
  const float r = 1.f - q * t * __expf(-a * a);
  return copysignf(r, x);
}

// Whole-wave reductions, every lane gets the result (call with all 64 lanes active).
// Within each row of 16 lanes by DPP (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror,
// row_mirror: register-to-register, a few cycles each), then the four row results by
// v_readlane into scalar registers -- instead of six dependent ds_bpermute round trips
// through the LDS crossbar.  Fixed combination order: deterministic.
template <int CTRL>
P2_DEVICE float dpp_mov(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
P2_DEVICE float row_lane(float v, int l) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l)); }
P2_DEVICE float wave_sum(float v) {
  v += dpp_mov<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_mov<0x141>(v);  // row_half_mirror
  v += dpp_mov<0x140>(v);  // row_mirror: every lane holds its row's sum
  return (row_lane(v, 0) + row_lane(v, 16)) + (row_lane(v, 32) + row_lane(v, 48));
}
P2_DEVICE float wave_max(float v) {
  v = fmaxf(v, dpp_mov<0xB1>(v));
  v = fmaxf(v, dpp_mov<0x4E>(v));
  v = fmaxf(v, dpp_mov<0x141>(v));
  v = fmaxf(v, dpp_mov<0x140>(v));
  return fmaxf(fmaxf(row_lane(v, 0), row_lane(v, 16)), fmaxf(row_lane(v, 32), row_lane(v, 48)));
}

}  // namespace p2

#define P2_CHECK(expr)                                                        \
  do {                                                                        \
    hipError_t _e = (expr);                                                   \
    if (_e != hipSuccess) throw std::runtime_error(hipGetErrorString(_e));    \
  } while (0)
