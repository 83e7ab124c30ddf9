// 256 x 256 bf16 MFMA GEMM with FOUR waves of 128 x 128 (gfx950), for the ViT-B
// Linear products (BASELINE config 4).
//
// Why another tile: the round-3 kernels split a 256 x 256 tile over 8 waves of
// 128 x 64 (gemm256 / ping-pong).  Every fragment a wave reads from LDS then
// feeds 2 MFMAs on one side, and the 8 waves synchronise twice per phase; the
// PMC comparison with hipBLASLt (profiles/r3_gemm_pingpong.md) showed 1.8x the
// LDS instructions and 31 % of wave cycles parked at barriers.  Here each wave
// owns 128 x 128 = 4 x 4 v_mfma_f32_32x32x16_bf16 tiles: 256 fp32 accumulators
// per lane, which the compiler keeps in AGPRs at one wave per SIMD (512-register
// budget), 8 fragment reads feed 16 MFMAs per k-substep, and there is ONE
// barrier per K-tile:
//
//   iteration it:  s_waitcnt vmcnt(0); barrier      (K-tile it landed in LDS, and every
//                                                    wave finished reading K-tile it-1)
//                  DMA K-tile it+1 -> the other buffer (last read at it-1: free)
//                  4 k-substeps x 16 MFMAs on K-tile it, the fragments of substep
//                  ks+1 read under the MFMAs of ks
//
// Operands go HBM/L2 -> LDS by global_load_lds (the loaders and swizzled LDS
// images of gemm_core.h: k-major ds_read_b128, mn-major ds_read_b64_tr_b16),
// so a K-tile costs no VGPR round trip.  2 stages x (A 32 KB + B 32 KB) = 128 KB
// of LDS; one workgroup per CU.  Split-K slices are reduced inside the launch by
// the last slice to reach a tile (the hand-off of gemm_core.h, same hardware
// note), so the weight-gradient products (9-36 tiles over K = 6304 tokens) fill
// the chip without a second launch.
//
// Epilogue: + bias (fp32 / bf16), GELU (+ pre-activation z), + residual, bf16
// (LDS-staged, 16-byte row stores) or fp32 output -- the same contract as
// gemm_core.h (GemmParams), selected by ops.gemm with variant bit 12.
//
// Reference: the Linear layers the reference trains through torch.nn.Linear
// (/root/reference/p2pfl/learning/pytorch/mnist_examples/models/mlp.py:53-55);
// the ViT-B/16 shapes of BASELINE.json config 4.
#include "gemm_core.h"

#include <utility>

namespace p2w4 {
using namespace p2gemm;

// f(std::integral_constant<int, I>) for I = 0 .. N-1, expanded at compile time: the
// accumulator indices stay constant expressions, so the accumulator array is never
// demoted to scratch memory (a plain unrolled loop over 64 groups was, 1088 B/lane)
template <class F, int... I>
P2_DEVICE void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
P2_DEVICE void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

constexpr int TM = 256, TN = 256, NTH = 256;
constexpr int STAGE4 = 4 * TILE;  // A halves 0,1 | B halves 2,3 (16 KB each)
constexpr int QN = 64;            // 16-byte groups per lane of a 128 x 128 wave tile
constexpr int TILEF = TM * TN;    // fp32 elements of one split-K slab tile

template <class LA, class LB, bool SPLIT>
__global__ __launch_bounds__(NTH, 1) void gemm_w4_kernel(GemmParams p, LA la, LB lb, int tiles_m, int tiles_n) {
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int bid = (p.variant & 4) ? int(blockIdx.x) : xcd_remap(blockIdx.x, gridDim.x);
  const int tiles = tiles_m * tiles_n;
  const int split = bid / tiles, t = bid % tiles;
  int tm, tn;
  tile_coords(p.variant, t, tiles_m, tiles_n, tm, tn);
  const int m0 = tm * TM, n0 = tn * TN;
  int kper = (p.K + p.splits - 1) / p.splits;
  kper = (kper + BK - 1) / BK * BK;
  const int kb = split * kper, ke = min(p.K, kb + kper);
  const int nt = ke > kb ? (ke - kb + BK - 1) / BK : 0;

  f32x16 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const typename LA::St sa0 = la.prep(m0, tid), sa1 = la.prep(m0 + 128, tid);
  const typename LB::St sb0 = lb.prep(n0, tid), sb1 = lb.prep(n0 + 128, tid);
  auto stage_all = [&](int k0, char* dst) {
    stage(la, sa0, k0, dst, tid);
    stage(la, sa1, k0, dst + TILE, tid);
    stage(lb, sb0, k0, dst + 2 * TILE, tid);
    stage(lb, sb1, k0, dst + 3 * TILE, tid);
  };
  const char* a_half = smem + wm * TILE;        // this wave's 128 A rows
  const char* b_half = smem + (2 + wn) * TILE;  // and 128 B rows
  if (nt > 0) stage_all(kb, smem);
  for (int it = 0; it < nt; ++it) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const int cur = (it & 1) * STAGE4;
    if (it + 1 < nt) stage_all(kb + (it + 1) * BK, smem + (STAGE4 - cur));
    uint4 fa[2][4], fb[2][4];
#pragma unroll
    for (int i = 0; i < 4; ++i) fa[0][i] = frag<LA::KMAJ>(a_half + cur, 32 * i, 0, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j) fb[0][j] = frag<LB::KMAJ>(b_half + cur, 32 * j, 0, lane);
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      const int cb = ks & 1;
      if (ks + 1 < BK / 16) {
#pragma unroll
        for (int i = 0; i < 4; ++i) fa[cb ^ 1][i] = frag<LA::KMAJ>(a_half + cur, 32 * i, ks + 1, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) fb[cb ^ 1][j] = frag<LB::KMAJ>(b_half + cur, 32 * j, ks + 1, lane);
      }
      // the 8 fragment reads of substep ks + 1 are issued before the 16 MFMAs of ks
      // (left alone, the scheduler sank each read next to its first use and exposed
      // the LDS latency 4x per substep at one wave per SIMD)
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma(fb[cb][j], fa[cb][i], acc[i][j]);
      __builtin_amdgcn_sched_barrier(0);
    }
  }

  // ---- epilogue: lane holds C[m0 + 128 wm + 32 i + (lane & 31)][n0 + 128 wn + 32 j + 8 g + 4 h + e]
  // in acc[i][j][4 g + e].  The accumulators stay in AGPRs: every 4-value group
  // is read out, finished and stored on its own (a VALU pass over all 256 at once
  // would need them in VGPRs).
  const int h = lane >> 5;
  // explicit AGPR reads, one 4-value group at a time: left to itself the compiler
  // copies all 256 accumulators to VGPRs before the epilogue and spills
  auto rd = [&](auto qc) __attribute__((always_inline)) {
    constexpr int q = decltype(qc)::value, i = q >> 4, j = (q >> 2) & 3, g = q & 3;
    f32x4 r;
    asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(r[0]) : "a"(acc[i][j][4 * g + 0]));
    asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(r[1]) : "a"(acc[i][j][4 * g + 1]));
    asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(r[2]) : "a"(acc[i][j][4 * g + 2]));
    asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(r[3]) : "a"(acc[i][j][4 * g + 3]));
    return r;
  };
  const uint32_t lane_off = uint32_t(((wave * QN) * 64 + lane) * 16);
  float* slabs = p.counters ? p.ws : reinterpret_cast<float*>(p.c);
  auto rsrc = [&](int s) __attribute__((always_inline)) {
    return __builtin_amdgcn_make_buffer_rsrc(slabs + (int64_t(s) * tiles + t) * TILEF, 0, TILEF * 4, 0x00020000);
  };
  if (SPLIT) {
    // this slice's fragment-native fp32 slab (sc1 stores when reduced in the launch)
    const auto rs = rsrc(split);
    static_for<QN>([&](auto qc) __attribute__((always_inline)) {
      constexpr int q = decltype(qc)::value;
      const f32x4 v = rd(qc);
      if (p.counters)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rs, lane_off + q * 1024, 0, 16);
      else
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rs, lane_off + q * 1024, 0, 0);
      __builtin_amdgcn_sched_barrier(0);  // keep the AGPR reads next to their store
    });
    if (!p.counters) return;
    // the last slice to reach the tile reduces it (hand-off of gemm_core.h)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = reinterpret_cast<int*>(smem);
    if (tid == 0) {
      const int old = __hip_atomic_fetch_add(p.counters + t, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      flag[0] = old == p.splits - 1;
      if (old == p.splits - 1) __hip_atomic_store(p.counters + t, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!flag[0]) return;
  }
  constexpr int LROW = TN * 2 + 16, CPR = TN / 8;
  static_assert(128 * LROW <= 2 * STAGE4, "epilogue image must fit the LDS");
  // bias, GELU (+ pre-activation), residual; fp32 C stored directly, bf16 C into the
  // LDS image of this wave row
  auto finish = [&](int i, int j, int g, f32x4 a) __attribute__((always_inline)) {
    const int m = m0 + 128 * wm + 32 * i + (lane & 31), n = n0 + 128 * wn + 32 * j + 8 * g + 4 * h;
    if (m >= p.M || n >= p.N) return;
    float v[4] = {a[0], a[1], a[2], a[3]};
    if (p.bias) {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        v[e] += p.bias_bf16 ? bf16_to_f32(reinterpret_cast<const uint16_t*>(p.bias)[n + e])
                            : reinterpret_cast<const float*>(p.bias)[n + e];
    }
    const int64_t off = int64_t(m) * p.ldc + n;
    if (p.gelu) {
      if (p.z) *reinterpret_cast<uint2*>(p.z + off) = uint2{pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3])};
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = gelu_f(v[e]);
    }
    if (p.residual) {
      const uint2 rr = *reinterpret_cast<const uint2*>(p.residual + off);
      v[0] += __uint_as_float(rr.x << 16);
      v[1] += __uint_as_float(rr.x & 0xffff0000u);
      v[2] += __uint_as_float(rr.y << 16);
      v[3] += __uint_as_float(rr.y & 0xffff0000u);
    }
    if (!p.c_bf16) {
      *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(p.c) + off) = f32x4{v[0], v[1], v[2], v[3]};
      return;
    }
    const int r = 32 * i + (lane & 31), c = 128 * wn + 32 * j + 8 * g + 4 * h;
    *reinterpret_cast<uint2*>(smem + r * LROW + c * 2) = uint2{pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3])};
  };
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    __syncthreads();  // LDS free (main loop / previous pass / the ticket flag)
    if (wm == pass) {
      if (SPLIT) {
        // sum of every slice in slice order (own slab included), 8 groups in flight
        constexpr int GF = 8;
#pragma unroll 1
        for (int qc = 0; qc < QN; qc += GF) {
          f32x4 sum[GF];
#pragma unroll
          for (int u = 0; u < GF; ++u) sum[u] = f32x4{0.f, 0.f, 0.f, 0.f};
          for (int s = 0; s < p.splits; ++s) {
            const auto rs = rsrc(s);
            f32x4 v[GF];
#pragma unroll
            for (int u = 0; u < GF; ++u)
              v[u] = __builtin_bit_cast(f32x4,
                                        __builtin_amdgcn_raw_buffer_load_b128(rs, lane_off + (qc + u) * 1024, 0, 16));
#pragma unroll
            for (int u = 0; u < GF; ++u) sum[u] += v[u];
          }
#pragma unroll
          for (int u = 0; u < GF; ++u) {
            const int q = qc + u;
            finish(q >> 4, (q >> 2) & 3, q & 3, sum[u]);
          }
        }
      } else {
        static_for<QN>([&](auto qc) __attribute__((always_inline)) {
          constexpr int q = decltype(qc)::value;
          finish(q >> 4, (q >> 2) & 3, q & 3, rd(qc));
        });
      }
    }
    if (!p.c_bf16) continue;
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 128 * CPR / NTH; ++q) {
      const int chunk = q * NTH + tid, r = chunk / CPR, c = chunk % CPR;
      const int m = m0 + 128 * pass + r, n = n0 + c * 8;
      if (m < p.M && n < p.N)
        *reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(p.c) + int64_t(m) * p.ldc + n) =
            *reinterpret_cast<const uint4*>(smem + r * LROW + c * 16);
    }
  }
}

template <class LA, class LB>
void launch(const GemmParams& p, const LA& la, const LB& lb, hipStream_t s) {
  const int tm = (p.M + TM - 1) / TM, tn = (p.N + TN - 1) / TN;
  const int grid = tm * tn * (p.splits > 1 ? p.splits : 1);
  if (p.splits > 1)
    hipLaunchKernelGGL((gemm_w4_kernel<LA, LB, true>), dim3(grid), dim3(NTH), 0, s, p, la, lb, tm, tn);
  else
    hipLaunchKernelGGL((gemm_w4_kernel<LA, LB, false>), dim3(grid), dim3(NTH), 0, s, p, la, lb, tm, tn);
}

}  // namespace p2w4

namespace p2 {

// fp32 elements of one split-K slice of this kernel (whole 256 x 256 tiles)
int64_t gemm_w4_slab_elems(int M, int N) { return int64_t((M + 255) / 256) * ((N + 255) / 256) * 256 * 256; }

void gemm_bf16_w4(const GemmParams& p, hipStream_t s) {
  using namespace p2gemm;
  if (p.a_kmajor && p.b_kmajor)
    p2w4::launch(p, PlainK{p.a, p.lda, p.M, p.K}, PlainK{p.b, p.ldb, p.N, p.K}, s);
  else if (p.a_kmajor)
    p2w4::launch(p, PlainK{p.a, p.lda, p.M, p.K}, PlainMN{p.b, p.ldb, p.N, p.K}, s);
  else if (p.b_kmajor)
    p2w4::launch(p, PlainMN{p.a, p.lda, p.M, p.K}, PlainK{p.b, p.ldb, p.N, p.K}, s);
  else
    p2w4::launch(p, PlainMN{p.a, p.lda, p.M, p.K}, PlainMN{p.b, p.ldb, p.N, p.K}, s);
}

}  // namespace p2
