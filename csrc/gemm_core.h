// MFMA GEMM core shared by the Linear GEMM (gemm.hip) and the implicit-GEMM
// convolutions (conv.hip): C[M][N] = sum_k A(m, k) B(n, k), bf16 operands,
// fp32 accumulation, gfx950 v_mfma_f32_32x32x16_bf16.
//
// The operands come through LOADER policies: a loader maps one 16-byte chunk
// of an operand tile to a global address, so the same pipeline serves plain
// matrices and the gathers of an implicit-GEMM convolution (im2col rows,
// transposed-convolution taps).  A k-major loader returns 8 consecutive k of
// one row (m or n); an mn-major loader 8 consecutive m / n of one k.  Any
// element outside the operand (rows past M / N, k past K, zero padding of a
// convolution) points at a 16-byte zero page, so tails need no masking.
//
// Pipeline (see gemm.hip for the full rationale): 128 x 128 tile per 256-thread
// workgroup, 4 waves as 2 x 2 (64 x 64 each, 2 x 2 MFMA tiles), BK = 64,
// global_load_lds into a double buffer (next tile's DMA issued before the
// current tile's MFMAs, one vmcnt(0) + barrier per K-tile), XOR-swizzled LDS
// images (ds_read_b128 for k-major, ds_read_b64_tr_b16 transpose reads for
// mn-major), XCD-aware tile order, split-K into fp32 slabs.
#pragma once
#include "common.h"
#include "gemm.h"

namespace p2gemm {
using namespace p2;

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

constexpr int BM = 128, BN = 128, BK = 64, NT = 256;
constexpr int TILE = BM * BK * 2;  // bytes per 128-row operand half-tile (16 KB)

// Output tile shape.  Operands are staged as 128-row halves (TILE bytes each,
// the loader geometry above: 256 threads x 4 chunks); a workgroup of NT
// threads is GROUPS = NT / 256 staging groups, group g filling the halves
// h = g, g + GROUPS, ... of A and of B.  Waves are WAVES_M x WAVES_N, each
// owning FM x FN 32 x 32 MFMA tiles.
//   Tile128: 128 x 128, 4 waves (2 x 2), 64 x 64 per wave -- up to 4
//            workgroups per CU (single-buffer schedule), the small-grid shape;
//   Tile256: 256 x 256, 8 waves (2 x 4), 128 x 64 per wave, 128 accumulator
//            registers, one workgroup per CU: half the L2 -> LDS bytes per
//            FLOP of Tile128, for the large products.
template <int BM_, int BN_, int WAVES_M_, int WAVES_N_>
struct TileCfg {
  static constexpr int BM = BM_, BN = BN_, WAVES_M = WAVES_M_, WAVES_N = WAVES_N_;
  static constexpr int NT = 64 * WAVES_M * WAVES_N;
  static constexpr int GROUPS = NT / 256;
  static constexpr int HA = (BM + 127) / 128, HB = (BN + 127) / 128;  // operand halves (Tile64: one partial half)
  static constexpr int FM = BM / WAVES_M / 32, FN = BN / WAVES_N / 32;
  static constexpr int STAGE = (HA + HB) * TILE;  // bytes per pipeline stage
  static_assert(NT % 256 == 0 && HA % GROUPS == 0 && HB % GROUPS == 0, "staging groups must split the halves");
};
using Tile128 = TileCfg<128, 128, 2, 2>;
using Tile256 = TileCfg<256, 256, 2, 4>;
//   Tile64:  64 x 64, 4 waves (2 x 2), one 32 x 32 MFMA tile per wave -- for
//            the CIFAR ResNet's 16x16 / 8x8 / 4x4 stages and 64-channel
//            products, where 128 x 128 tiles leave most CUs idle (or half of
//            every MFMA on zero columns) and needed split-K slabs + a reduce.
using Tile64 = TileCfg<64, 64, 2, 2>;

// Zero page for out-of-operand chunks (one copy per translation unit).  It is
// 64 KB, not 16 B: a tile whose rows or taps fall outside the operand sends
// every lane of every CU to it, and one hot 16-byte line serialises on a
// single L2 channel (measured ~1 us per K-tile on a 64-wide conv); each lane
// of each workgroup takes its own 16-byte slot instead.
static __device__ __attribute__((aligned(16))) uint16_t g_zero_page[32768] = {};
P2_DEVICE const void* zero_chunk() {
  return g_zero_page + ((threadIdx.x & 63) + 64 * (blockIdx.x & 63)) * 8;
}

P2_DEVICE f32x16 mfma(uint4 a, uint4 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c,
                                                  0, 0, 0);
}

P2_DEVICE int swz_k(int row) { return (row >> 1) & 7; }                       // k-major: 8 chunks / 128-B row
P2_DEVICE int swz_mn(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }  // mn-major: 16 chunks / 256-B row

// ---- loader protocol -----------------------------------------------------------
// A loader is a small struct passed by value into the kernel.  `prep(r0, tid)`
// runs once per workgroup and returns the lane's state: within one operand
// tile a lane always moves the same four chunks (i = 0..3), whose row (k-major)
// or column (mn-major) coordinate does not change along K, so everything that
// depends on it is decoded once.  `src(st, i, k0, tid)` returns the global
// address of chunk i of the K-tile starting at k0 (or a zero-page chunk).
//
// Chunk geometry (cid = 256 i + tid):
//   k-major : row = 32 i + (tid >> 3), k = k0 + 8 ((tid & 7) ^ ((tid >> 4) & 7))
//   mn-major: k = k0 + 16 i + (tid >> 4),
//             col = 8 ((tid & 15) ^ (((tid >> 4) & 3) << 2 | (tid >> 6) & 3))
// (the XOR terms are swz_k / swz_mn of the LDS row, which do not depend on i).
P2_DEVICE int kmaj_row(int i, int tid) { return 32 * i + (tid >> 3); }
P2_DEVICE int kmaj_k(int tid) { return 8 * ((tid & 7) ^ ((tid >> 4) & 7)); }
P2_DEVICE int mnmaj_k(int i, int tid) { return 16 * i + (tid >> 4); }
P2_DEVICE int mnmaj_col(int tid) { return 8 * ((tid & 15) ^ ((((tid >> 4) & 3) << 2) | ((tid >> 6) & 3))); }

struct PlainK {  // element (r, k) at g[r * ld + k]
  static constexpr bool KMAJ = true;
  const uint16_t* g;
  int64_t ld;
  int nrows, K;
  struct St {
    const uint16_t* row[4];
    int kk;
  };
  P2_DEVICE St prep(int r0, int tid) const {
    St st;
    st.kk = kmaj_k(tid);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = r0 + kmaj_row(i, tid);
      st.row[i] = r < nrows ? g + r * ld + st.kk : nullptr;
    }
    return st;
  }
  P2_DEVICE const void* src(const St& st, int i, int k0, int) const {
    return (st.row[i] && k0 + st.kk < K) ? static_cast<const void*>(st.row[i] + k0) : zero_chunk();
  }
};
struct PlainMN {  // element (r, k) at g[k * ld + r]
  static constexpr bool KMAJ = false;
  const uint16_t* g;
  int64_t ld;
  int nrows, K;
  struct St {
    const uint16_t* col;
    int kr;
  };
  P2_DEVICE St prep(int r0, int tid) const {
    const int c = r0 + mnmaj_col(tid);
    return St{c < nrows ? g + c : nullptr, tid >> 4};
  }
  P2_DEVICE const void* src(const St& st, int i, int k0, int) const {
    const int k = k0 + 16 * i + st.kr;
    return (st.col && k < K) ? static_cast<const void*>(st.col + k * ld) : zero_chunk();
  }
};

// Issue the DMA of one operand tile (K-tile starting at k0) into `lds`; every
// lane moves 16 B four times.  The LDS image is lane-linear per wave; the
// swizzle lives in the chunk -> source-address mapping above.
//
// The load is issued from inline asm, not __builtin_amdgcn_global_load_lds:
// hipcc cannot tell which LDS bytes a builtin DMA writes, so it drains every
// outstanding DMA (s_waitcnt vmcnt(0)) before the next ds_read -- including
// the prefetch of the OTHER buffer, issued just before this K-tile's
// fragment reads, which serialised the double buffer.  Hidden in asm, the
// DMA is waited for only where the pipeline says so: the explicit
// vmcnt(0) + barrier ahead of the buffer's first read.
P2_DEVICE void dma16(const void* gsrc, char* lds_dst) {
  const uint32_t m0v = __builtin_amdgcn_readfirstlane(uint32_t(reinterpret_cast<uintptr_t>(lds_dst)));
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(m0v)
      : "memory");
}

// NCH chunks per thread (4: a full 128-row half; a k-major operand of a 64-row
// tile stages chunks 0-1 = its rows 0-63 only, into the first 8 KB)
template <int NCH, class L>
P2_DEVICE void stage(const L& ld, const typename L::St& st, int k0, char* lds, int tid) {
  const int wave = tid >> 6;
#pragma unroll
  for (int i = 0; i < NCH; ++i) dma16(ld.src(st, i, k0, tid), lds + (i * NT + wave * 64) * 16);  // lane L writes dst + 16 L
}

// Chunks per thread of one staged half of an operand with `rows` tile rows: a
// k-major image is row-linear (128 B per row), so a narrow tile stages (and
// keeps) only its rows; an mn-major image is k-linear over 128 columns (its
// fragment reads address columns inside that 256-B row) and stays whole.
template <int ROWS, bool KMAJ>
constexpr int half_chunks() {
  return (KMAJ && ROWS < 128) ? ROWS / 32 : 4;
}
// LDS bytes of one pipeline stage (A halves, then B halves) for these loaders
template <class CFG, class LA, class LB>
constexpr int stage_bytes() {
  return CFG::HA * half_chunks<(CFG::BM < 128 ? CFG::BM : 128), LA::KMAJ>() * NT * 16 +
         CFG::HB * half_chunks<(CFG::BN < 128 ? CFG::BN : 128), LB::KMAJ>() * NT * 16;
}

// Fragment of a 32-row block (rows rb..rb+31 of the tile) for k-substep ks:
// lane l holds element (rb + (l & 31), 16 ks + 8 (l >> 5) + j), j = 0..7.
template <bool KMAJ>
P2_DEVICE uint4 frag(const char* lds, int rb, int ks, int lane) {
  if constexpr (KMAJ) {
    const int row = rb + (lane & 31), c = 2 * ks + (lane >> 5);
    return *reinterpret_cast<const uint4*>(lds + row * 128 + ((c ^ swz_k(row)) << 4));
  } else {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int col = rb + 16 * (g & 1) + 4 * p;  // this lane supplies 4 columns of row q
    const int ch = col >> 3, sub = (col & 7) * 2;
    uint4 out;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int row = 16 * ks + 8 * (g >> 1) + 4 * t + q;
      const char* addr = lds + row * 256 + ((ch ^ swz_mn(row)) << 4) + sub;
      const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(addr));
      const uint2 u = __builtin_bit_cast(uint2, v);
      if (t == 0) {
        out.x = u.x;
        out.y = u.y;
      } else {
        out.z = u.x;
        out.w = u.y;
      }
    }
    return out;
  }
}

P2_DEVICE float gelu_f(float z) { return 0.5f * z * (1.f + erf_fast(z * 0.70710678118654752f)); }

// XCD-aware bijective remap of a linear workgroup id (blocks sharing an XCD get consecutive ids).
P2_DEVICE int xcd_remap(int orig, int nwg) {
  const int xcd = orig % 8, q = nwg / 8, r = nwg % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

// LDS bytes a kernel of this shape declares: the pipeline stages, and for the
// 8-wave tile at least the whole bf16 output tile (padded rows), so its
// epilogue stages C in one pass (132 KB; still one workgroup per CU).
template <class CFG, int NBUF>
constexpr int smem_bytes() {  // NBUF: LDS stages of the K loop (1, 2, or a 3-5 stage ring)
  constexpr int pipe = NBUF * CFG::STAGE, epi = CFG::BM * (CFG::BN * 2 + 16);
  return (CFG::NT >= 512 && epi > pipe) ? epi : pipe;
}
// the same for a kernel that knows its loaders (narrow k-major halves staged compactly);
// equal to smem_bytes for the 128- and 256-row tiles
template <class CFG, int NBUF, class LA, class LB>
constexpr int smem_bytes_l() {
  constexpr int pipe = NBUF * stage_bytes<CFG, LA, LB>(), epi = CFG::BM * (CFG::BN * 2 + 16);
  return (CFG::NT >= 512 && epi > pipe) ? epi : pipe;
}

// s_waitcnt vmcnt(LPT * n) for a runtime n in [0, MAXN] (the count must be an
// immediate): waits until at most n K-tiles of LPT DMAs each are in flight.
template <int LPT, int MAXN>
P2_DEVICE void vmcnt_tiles(int n) {
  static_assert(LPT * MAXN <= 63, "vmcnt is 6 bits");
  if constexpr (MAXN >= 3) {
    if (n >= 3) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LPT * 3) : "memory");
      return;
    }
  }
  if constexpr (MAXN >= 2) {
    if (n == 2) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LPT * 2) : "memory");
      return;
    }
  }
  if constexpr (MAXN >= 1) {
    if (n == 1) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LPT) : "memory");
      return;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// A launch whose epilogue is a plain store of C (no split-K, bias, GELU,
// residual or BatchNorm statistics): kernels instantiate a compact epilogue for it.
inline bool plain_epilogue(const GemmParams& p) {
  return p.splits <= 1 && !p.bias && !p.gelu && !p.residual && !p.bn.part;
}
// 0: plain store, 2: + bias only (the Linear forward), 1: everything behind runtime flags
inline int epilogue_kind(const GemmParams& p) {
  if (plain_epilogue(p)) return 0;
  return (p.splits <= 1 && !p.gelu && !p.residual && !p.bn.part) ? 2 : 1;
}

// Output tile (tm, tn) of linear tile index t (see the tile-order note in gemm_body).
P2_DEVICE void tile_coords(int variant, int t, int tiles_m, int tiles_n, int& tm, int& tn) {
  if (variant & 256) {
    tm = (variant & 2) ? t / tiles_n : t % tiles_m;
    tn = (variant & 2) ? t % tiles_n : t / tiles_m;
  } else {
    constexpr int GROUP_M = 8;
    const int per_group = GROUP_M * tiles_n, g0 = (t / per_group) * GROUP_M;
    const int gsize = min(tiles_m - g0, GROUP_M), r = t % per_group;
    tm = g0 + r % gsize;
    tn = r / gsize;
  }
}

// Split-K partial tiles are stored fragment-native: slice s of tile t is one
// contiguous block of TILEF = NT * FM * FN * 16 floats (= BM * BN), group q of
// lane l of wave w at ((w * QN + q) * 64 + l) * 4 (QN = 4 FM FN groups per lane),
// so every store / load instruction moves 1 KB contiguous (a row-major slab
// scattered each wave's 16-byte groups over 32 rows).  Only the reducers read
// this layout: the in-launch last arriver and tile_slab_reduce_kernel.
template <class CFG>
struct SlabGeom {
  static constexpr int QN = CFG::FM * CFG::FN * 4;
  static constexpr int TILEF = CFG::NT * CFG::FM * CFG::FN * 16;
  static_assert(TILEF == CFG::BM * CFG::BN, "fragment slab covers the tile");
};

// ---- BatchNorm statistics epilogue (GemmParams::bn) -------------------------------
// Running (count, mean, M2) of one column; Chan et al.'s pairwise update.
struct Moments {
  float n, mean, m2;
};
P2_DEVICE Moments moments_merge(Moments a, const Moments& b) {
  if (b.n <= 0.f) return a;
  if (a.n <= 0.f) return b;
  const float n = a.n + b.n, d = b.mean - a.mean, f = b.n / n;
  a.mean = fmaf(d, f, a.mean);
  a.m2 = a.m2 + b.m2 + d * d * a.n * f;
  a.n = n;
  return a;
}
// forward statistics merge by Chan's formula; backward sums (s1, s2 in the mean /
// m2 slots) simply add
P2_DEVICE Moments bn_merge(bool bwd, Moments a, const Moments& b) {
  if (bwd) return Moments{a.n + b.n, a.mean + b.mean, a.m2 + b.m2};
  return moments_merge(a, b);
}
P2_DEVICE void st_sc1(float* base, int n, int idx, float v) {
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(base, 0, n * 4, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rs, idx * 4, 0, 16);
}
P2_DEVICE float ld_sc1(const float* base, int n, int idx) {
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, n * 4, 0x00020000);
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, idx * 4, 0, 16));
}
// Arrival ticket of a workgroup whose sc1 stores must be visible to the last
// arriver (same hand-off as the split-K reduction; see the hardware note
// there).  True in the last of `total` arrivals, which resets the counter.
P2_DEVICE bool last_arrival(int* ctr, int total, int* flag_lds) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const int old = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    flag_lds[0] = old == total - 1;
    if (old == total - 1) __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  return flag_lds[0] != 0;
}

constexpr int kBnGroup = 16;  // tile rows per first-level group

// The tile's column moments (`mo`, held by threads tid < BN for column n0 + tid)
// go out as this tile's partial; the two-level reduction finalizes the columns.
template <class CFG, bool bwd>
P2_DEVICE void bn_epilogue_reduce(const GemmParams& p, Moments mo, int tm, int tn, int tiles_m, char* smem) {
  const BnEpi& e = p.bn;
  const int tid = threadIdx.x, N = p.N, n0 = tn * CFG::BN;
  const int groups = (tiles_m + kBnGroup - 1) / kBnGroup, g = tm / kBnGroup;
  const int gsize = min(kBnGroup, tiles_m - g * kBnGroup);
  const int nparts = (tiles_m + groups) * 2 * N;
  const int n = n0 + tid;
  const bool col = tid < CFG::BN && n < N;
  if (col) {
    st_sc1(e.part, nparts, (tm * 2) * N + n, mo.mean);
    st_sc1(e.part, nparts, (tm * 2 + 1) * N + n, mo.m2);
  }
  int* flag = reinterpret_cast<int*>(smem);
  auto tile_rows = [&](int t) { return float(min(CFG::BM, p.M - t * CFG::BM)); };
  if (!last_arrival(e.cnt + tn * (groups + 1) + g, gsize, flag)) return;
  if (e.mode == 2) return;
  // level 1: combine the group's tile partials in tile order
  Moments acc{0.f, 0.f, 0.f};
  if (col) {
    float mv[kBnGroup], m2v[kBnGroup];
#pragma unroll
    for (int i = 0; i < kBnGroup; ++i) {
      const int t = g * kBnGroup + i;
      mv[i] = i < gsize ? ld_sc1(e.part, nparts, (t * 2) * N + n) : 0.f;
      m2v[i] = i < gsize ? ld_sc1(e.part, nparts, (t * 2 + 1) * N + n) : 0.f;
    }
#pragma unroll
    for (int i = 0; i < kBnGroup; ++i)
      if (i < gsize) acc = bn_merge(bwd, acc, Moments{tile_rows(g * kBnGroup + i), mv[i], m2v[i]});
  }
  if (groups > 1) {
    if (col) {
      st_sc1(e.part, nparts, ((tiles_m + g) * 2) * N + n, acc.mean);
      st_sc1(e.part, nparts, ((tiles_m + g) * 2 + 1) * N + n, acc.m2);
    }
    if (!last_arrival(e.cnt + tn * (groups + 1) + groups, groups, flag)) return;
    acc = Moments{0.f, 0.f, 0.f};
    if (col) {
      for (int g0 = 0; g0 < groups; g0 += kBnGroup) {
        float mv[kBnGroup], m2v[kBnGroup];
#pragma unroll
        for (int i = 0; i < kBnGroup; ++i) {
          const int gg = g0 + i;
          mv[i] = gg < groups ? ld_sc1(e.part, nparts, ((tiles_m + gg) * 2) * N + n) : 0.f;
          m2v[i] = gg < groups ? ld_sc1(e.part, nparts, ((tiles_m + gg) * 2 + 1) * N + n) : 0.f;
        }
#pragma unroll
        for (int i = 0; i < kBnGroup; ++i) {
          const int gg = g0 + i;
          if (gg >= groups) continue;
          float rows = 0.f;
          for (int t = gg * kBnGroup; t < min(tiles_m, (gg + 1) * kBnGroup); ++t) rows += tile_rows(t);
          acc = bn_merge(bwd, acc, Moments{rows, mv[i], m2v[i]});
        }
      }
    }
  }
  if (!col) return;
  const float M = float(p.M);
  if (bwd) {  // same outputs as bn_finalize_bwd_kernel
    const float rs = e.brstd[n], A = e.w[n] * rs, s1 = acc.mean, s2 = acc.m2;
    e.db[n] = s1;
    e.dw[n] = s2 * rs;
    e.coef[n] = A;
    e.coef[N + n] = -A * rs * rs * s2 / M;
    e.coef[2 * N + n] = -A * s1 / M;
    return;
  }
  // finalize column n (same outputs as bn_finalize_fwd_kernel)
  const float var = fmaxf(acc.m2 / M, 0.f);
  const float rs = rsqrtf(var + e.eps);
  e.mean[n] = acc.mean;
  e.rstd[n] = rs;
  e.coef[n] = acc.mean;
  e.coef[N + n] = e.w[n] * rs;
  e.coef[2 * N + n] = e.b[n];
  if (e.run_mean) {
    const float unb = p.M > 1 ? acc.m2 / (M - 1.f) : var;
    e.run_mean[n] = (1.f - e.momentum) * e.run_mean[n] + e.momentum * acc.mean;
    e.run_var[n] = (1.f - e.momentum) * e.run_var[n] + e.momentum * unb;
  }
  if (e.nbt && n == 0) e.nbt[0] += 1;
}

// The whole kernel body.  `p` carries M/N/K, split-K and the epilogue.
// BN: compile the BatchNorm statistics epilogue in (GemmParams::bn; the conv
// kernels that produce a BN input instantiate it, the Linear GEMMs do not)
// EPI (epilogue_kind): 0 compact epilogue for plain stores, 2 bias only (see
// gemm_pp.hip's note on instruction fetch); 1 every epilogue feature behind
// runtime flags.
// A loader sees the output tile it serves through tile_bound (default: itself);
// a loader whose gather depends on the tile's rows -- the stride-2 input
// gradient's B operand takes the taps of its tile's output phase (conv.hip) --
// overloads it to return a copy bound to the tile's first row.
template <class L>
P2_DEVICE const L& tile_bound(const L& l, int) {
  return l;
}

template <class CFG, int NBUF, class LA, class LB, int BN = 0, int EPI = 1>
P2_DEVICE void gemm_body(const GemmParams& p, const LA& la0, const LB& lb0, int tiles_m, int tiles_n, char* smem) {
  constexpr int FM = CFG::FM, FN = CFG::FN, HA = CFG::HA, HB = CFG::HB, G = CFG::GROUPS;
  // chunks per thread and bytes of one staged half of A / B, bytes of a pipeline stage
  constexpr int CHA = half_chunks<(CFG::BM < 128 ? CFG::BM : 128), LA::KMAJ>();
  constexpr int CHB = half_chunks<(CFG::BN < 128 ? CFG::BN : 128), LB::KMAJ>();
  constexpr int HALF_A = CHA * NT * 16, HALF_B = CHB * NT * 16, STG = HA * HALF_A + HB * HALF_B;
  constexpr int SMEM = smem_bytes_l<CFG, NBUF, LA, LB>();
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / CFG::WAVES_N, wn = wave % CFG::WAVES_N;
  const int grp = tid >> 8, gt = tid & 255;  // staging group, thread within it
  const int bid = (p.variant & 4) ? int(blockIdx.x) : xcd_remap(blockIdx.x, gridDim.x);
  const int tiles = tiles_m * tiles_n;
  const int split = bid / tiles, t = bid % tiles;
  // Tile order: the workgroups resident on one XCD at a time are a run of
  // consecutive ids (xcd_remap), and that XCD's L2 serves them only the
  // operand panels they share.  Grouped order (default) walks GROUP_M tile
  // rows before moving one tile column, so a run of R resident tiles covers
  // about GROUP_M x R / GROUP_M tiles: 8 A + 4 B panels for Tile256's 32 per
  // XCD, where a single-row run reads 1 A + 32 B panels (measured at 8192^3:
  // L2 hit rate 48 % -> the bound on the K loop).  Variant bit 8: legacy
  // panel order, consecutive tiles sharing the B panel (bit 1: the A panel).
  int tm, tn;
  tile_coords(p.variant, t, tiles_m, tiles_n, tm, tn);
  const int m0 = tm * CFG::BM, n0 = tn * CFG::BN;
  const LA la = tile_bound(la0, m0);
  const LB lb = tile_bound(lb0, m0);
  int kper = (p.K + p.splits - 1) / p.splits;
  kper = (kper + BK - 1) / BK * BK;
  const int kb = split * kper, ke = min(p.K, kb + kper);
  const int nt = (ke > kb && !(p.variant & 32)) ? (ke - kb + BK - 1) / BK : 0;  // bit 5: skip the K loop (timing probe)

  f32x16 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  // loader state of the halves this thread's group stages
  typename LA::St sta[HA / G];
  typename LB::St stb[HB / G];
#pragma unroll
  for (int q = 0; q < HA / G; ++q) sta[q] = la.prep(m0 + 128 * (grp + G * q), gt);
#pragma unroll
  for (int q = 0; q < HB / G; ++q) stb[q] = lb.prep(n0 + 128 * (grp + G * q), gt);
  auto stage_all = [&](int k0, char* dst) {
#pragma unroll
    for (int q = 0; q < HA / G; ++q) stage<CHA>(la, sta[q], k0, dst + (grp + G * q) * HALF_A, gt);
#pragma unroll
    for (int q = 0; q < HB / G; ++q) stage<CHB>(lb, stb[q], k0, dst + HA * HALF_A + (grp + G * q) * HALF_B, gt);
  };
  // chunk c (0..3) of every half this group stages: stage_all split in four
  auto stage_chunk = [&](int c, int k0, char* dst) {
    const int wo = (c * NT + (gt >> 6) * 64) * 16;
    if (c < CHA)
#pragma unroll
      for (int q = 0; q < HA / G; ++q) dma16(la.src(sta[q], c, k0, gt), dst + (grp + G * q) * HALF_A + wo);
    if (c < CHB)
#pragma unroll
      for (int q = 0; q < HB / G; ++q) dma16(lb.src(stb[q], c, k0, gt), dst + HA * HALF_A + (grp + G * q) * HALF_B + wo);
  };
  // where the next K-tile's DMA is issued (variant bits 9-10): 0 before this
  // K-tile's first fragment reads, 1 right after them, 2 spread over the four
  // k-substeps (one chunk each)
  const int dma_mode = (p.variant >> 9) & 3;
  // fragment rows: wave (wm, wn) owns A rows wm * 32 FM + 32 i, B rows wn * 32 FN + 32 j
  auto frag_a = [&](const char* s, int i, int ks) {
    const int r = wm * 32 * FM + 32 * i;
    return frag<LA::KMAJ>(s + (r >> 7) * HALF_A, r & 127, ks, lane);
  };
  auto frag_b = [&](const char* s, int j, int ks) {
    const int r = wn * 32 * FN + 32 * j;
    return frag<LB::KMAJ>(s + HA * HALF_A + (r >> 7) * HALF_B, r & 127, ks, lane);
  };
  if constexpr (NBUF == 2) {
    if (nt > 0) {
      stage_all(kb, smem);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  }
  // One K-tile: MFMAs over the LDS image at `s`; fragments of sub-step ks + 1
  // are read from LDS while the MFMAs of ks run (one block per CU is common
  // for the small convolution / split-K grids, where the LDS read latency is
  // otherwise exposed four times per K-tile).
  auto compute = [&](const char* s, int k_next, char* dst) {  // k_next < 0: no DMA
    if (k_next >= 0 && dma_mode == 0) stage_all(k_next, dst);
    uint4 fa[2][FM], fb[2][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i) fa[0][i] = frag_a(s, i, 0);
#pragma unroll
    for (int j = 0; j < FN; ++j) fb[0][j] = frag_b(s, j, 0);
    if (k_next >= 0 && dma_mode == 1) stage_all(k_next, dst);
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      const int cb = ks & 1;
      if (k_next >= 0 && dma_mode >= 2) stage_chunk(ks, k_next, dst);
      if (ks + 1 < BK / 16) {
#pragma unroll
        for (int i = 0; i < FM; ++i) fa[cb ^ 1][i] = frag_a(s, i, ks + 1);
#pragma unroll
        for (int j = 0; j < FN; ++j) fb[cb ^ 1][j] = frag_b(s, j, ks + 1);
      }
      if (p.variant & 1) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mfma(fb[cb][j], fa[cb][i], acc[i][j]);
      if (p.variant & 1) __builtin_amdgcn_s_setprio(0);
    }
  };
  if constexpr (NBUF >= 3) {
    // NBUF-stage ring for short-K, small-grid products (the CIFAR convolutions:
    // one workgroup per CU, 9-72 K-tiles): NBUF - 1 K-tiles are in flight while
    // one is consumed, so the HBM/L2 round trip is paid about once per
    // NBUF - 1 tiles instead of once per tile.  One raw barrier per K-tile;
    // the counted vmcnt retires exactly the tile read next (never vmcnt(0)
    // until the tail); the buffer restaged at iteration it is the one read at
    // it - 1, which every wave finished before passing this barrier.
    constexpr int LPT = (HA / G) * CHA + (HB / G) * CHB;  // DMAs per thread per K-tile
    auto buf = [&](int t) { return smem + (t % NBUF) * STG; };
    for (int j = 0; j < NBUF - 1 && j < nt; ++j) stage_all(kb + j * BK, buf(j));
    for (int it = 0; it < nt; ++it) {
      const int ahead = min(nt - it - 1, NBUF - 2);  // K-tiles allowed to stay in flight
      vmcnt_tiles<LPT, NBUF - 2>(ahead);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      if (it + NBUF - 1 < nt) stage_all(kb + (it + NBUF - 1) * BK, buf(it + NBUF - 1));
      compute(buf(it), -1, smem);
    }
  } else if constexpr (NBUF == 2) {
    // Two K-tiles per iteration so both LDS buffers sit at constant offsets:
    // the compiler can then tell the DMA into one buffer from the ds_reads of
    // the other and does not drain the in-flight prefetch (vmcnt(0)) before
    // every K-tile's first fragment read -- with a runtime buffer index it
    // did, which serialised load and compute.
    const bool dma = !(p.variant & 128);  // bit 7: no DMA after the prologue (timing probe: compute only)
    for (int it = 0; it < nt; it += 2) {
      compute(smem, (dma && it + 1 < nt) ? kb + (it + 1) * BK : -1, smem + STG);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (it + 1 < nt) {
        compute(smem + STG, (dma && it + 2 < nt) ? kb + (it + 2) * BK : -1, smem);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      }
    }
  } else {  // one buffer: latency hidden by the other resident workgroups
    for (int it = 0; it < nt; ++it) {
      stage_all(kb + it * BK, smem);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      compute(smem, -1, smem);
      __syncthreads();
    }
  }

  // ---- epilogue: lane holds C[m][n0 + wn*32FN + j*32 + 8 g + 4 h + e] for its m
  if (p.variant & 16) {  // bit 4: no stores (timing probe); keep acc alive
    if (acc[0][0][0] == 12345.f && acc[FM - 1][FN - 1][15] == -1.f) reinterpret_cast<float*>(p.c)[0] = 0.f;
    return;
  }
  const int h = lane >> 5;
  auto row_of = [&](int i) { return m0 + wm * 32 * FM + i * 32 + (lane & 31); };
  auto col_of = [&](int j, int g) { return n0 + wn * 32 * FN + j * 32 + 8 * g + 4 * h; };
  if (EPI == 1 && p.splits > 1) {
    // every K-slice writes its raw fp32 partial tile, fragment-native (SlabGeom)
    using SG = SlabGeom<CFG>;
    float* slabs = p.counters ? p.ws : reinterpret_cast<float*>(p.c);
    const int tiles = tiles_m * tiles_n;
    const uint32_t lane_off = uint32_t(((wave * SG::QN) * 64 + lane) * 16);
    auto tile_rsrc = [&](int s) __attribute__((always_inline)) {
      return __builtin_amdgcn_make_buffer_rsrc(slabs + (int64_t(s) * tiles + t) * SG::TILEF, 0, SG::TILEF * 4, 0x00020000);
    };
    {
      const auto rs = tile_rsrc(split);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int q = (i * FN + j) * 4 + g;
            const f32x4 v = {acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]};
            // in-launch: sc1 (write-through) stores, so the hand-off needs no
            // release fence (an agent release wrote back the whole L2 per slice)
            if (p.counters)
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rs, lane_off + q * 1024, 0, 16);
            else
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rs, lane_off + q * 1024, 0, 0);
          }
    }
    if (!p.counters) return;
    // In-launch reduction: the slice that arrives last at this tile's counter
    // sums all slices' slabs and runs the epilogue.  Every wave drains its sc1
    // stores, then one relaxed agent-scope ticket; the last arriver reads the
    // slabs with sc1 loads (every one of them), so no acquire fence either.
    // The counter is reset for the next launch.
    //
    // HARDWARE ASSUMPTION (gfx950, not the HIP memory model): the slab stores
    // and loads carry the device-scope cache-policy bit (aux = 16, "sc1"), so a
    // store is written through the issuing XCD's L2 before its vmcnt retires,
    // and a load is served from the device coherence point, never from a stale
    // line in the reading XCD's L2.  The s_waitcnt vmcnt(0) + barrier before the
    // ticket therefore orders every slab store before the atomic at device
    // scope, which is what an agent release fence would give (at the cost of a
    // whole-L2 write-back per slice).  Slices of one tile land on different XCDs
    // (round-robin workgroup dispatch), and the workspace is re-used by the
    // next launch, so tests/test_gpu_gemm.py::test_in_launch_splitk_reused_workspace
    // runs many back-to-back split-K launches over one workspace against the
    // separate-launch reducer to pin this assumption.
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
    // acc := sum of all slices (own slab included), all groups of a slice in
    // flight at once (two slices when the register budget allows)
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
    auto ld = [&](const __amdgpu_buffer_rsrc_t& rs, int q) __attribute__((always_inline)) {
      return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, lane_off + q * 1024, 0, 16));
    };
    int s2 = 0;
    for (; NBUF >= 2 && SG::QN <= 16 && s2 + 2 <= p.splits; s2 += 2) {
      const auto r0 = tile_rsrc(s2), r1 = tile_rsrc(s2 + 1);
      f32x4 v0[SG::QN], v1[SG::QN];
#pragma unroll
      for (int q = 0; q < SG::QN; ++q) {
        v0[q] = ld(r0, q);
        v1[q] = ld(r1, q);
      }
#pragma unroll
      for (int q = 0; q < SG::QN; ++q)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[q / (4 * FN)][(q / 4) % FN][4 * (q % 4) + e] += v0[q][e] + v1[q][e];
    }
    for (; s2 < p.splits; ++s2) {
      const auto r0 = tile_rsrc(s2);
      f32x4 v0[SG::QN];
#pragma unroll
      for (int q = 0; q < SG::QN; ++q) v0[q] = ld(r0, q);
#pragma unroll
      for (int q = 0; q < SG::QN; ++q)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[q / (4 * FN)][(q / 4) % FN][4 * (q % 4) + e] += v0[q][e];
    }
  }
  // BatchNorm statistics (p.bn) of this tile, from the accumulators: each lane
  // holds 4 consecutive columns x FM rows per (j, g); the bf16-rounded values (what
  // is stored) are summed over the lane's rows, then lanes r and r ^ 16 are added
  // (one independent shuffle per value), the 16 row-pair partials of every column
  // go through LDS and one thread per (wave row, column) adds them in fixed order;
  // the WAVES_M wave rows sharing a column are merged last.  (A 5-step xor-shuffle
  // tree per value was 352 dependent LDS-crossbar round trips per wave: +12 us per
  // launch, scripts/bn_epi_probe.py.)  Forward: sums shifted by the column's value
  // in the wave's first row (v_readlane, no LDS) -> (count, mean, M2); backward:
  // dz' = dz (bn output > 0) and dz' (x - mean) from the BN's input / output
  // tensors, read in the accumulator layout (8-byte vectors).
  if (BN && p.bn.part != nullptr && p.bn.mode != 3) {
    const BnEpi& e = p.bn;
    constexpr bool bwd = BN == 2;  // compiled per direction: no runtime branches on it
    const int h = lane >> 5;
    const int mrow0 = m0 + wm * 32 * FM;  // first row of this wave
    constexpr int CW = CFG::WAVES_N * 32;  // columns of one pass (one j per wave)
    float* s1p = reinterpret_cast<float*>(smem);          // [WAVES_M][16][CW]
    float* s2p = s1p + CFG::WAVES_M * 16 * CW;            // [WAVES_M][16][CW]
    float* shp = s2p + CFG::WAVES_M * 16 * CW;            // [WAVES_M][CW]
    static_assert(!BN || (2 * 16 + 1) * CFG::WAVES_M * CW * 4 <= SMEM, "BN pass buffers fit the LDS");
    static_assert(!BN || CFG::WAVES_M * CFG::BN * 3 * 4 <= SMEM, "BN merge buffer fits the LDS");
    float keep[FN][3];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      float s1[4][4], s2[4][4], sh[4][4];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int n = n0 + wn * 32 * FN + j * 32 + 8 * g + 4 * h;
        const bool ncol = n < p.N;
        float mu[4] = {0.f, 0.f, 0.f, 0.f};
        if (bwd && ncol) {
          const f32x4 mv = *reinterpret_cast<const f32x4*>(e.bmean + n);
          mu[0] = mv[0], mu[1] = mv[1], mu[2] = mv[2], mu[3] = mv[3];
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          s1[g][q] = 0.f;
          s2[g][q] = 0.f;
          const int v0 = __float_as_int(bf16_to_f32(f32_to_bf16(acc[0][j][4 * g + q])));
          const float a = __int_as_float(__builtin_amdgcn_readlane(v0, 0));
          const float b = __int_as_float(__builtin_amdgcn_readlane(v0, 32));
          sh[g][q] = bwd ? 0.f : (h ? b : a);
        }
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int m = mrow0 + i * 32 + (lane & 31);
          if (m >= p.M || !ncol) continue;
          float xv[4] = {0.f, 0.f, 0.f, 0.f}, yv[4] = {1.f, 1.f, 1.f, 1.f};
          if (bwd) {
            const int64_t off = int64_t(m) * p.N + n;
            const uint2 xr = *reinterpret_cast<const uint2*>(e.bx + off);
            xv[0] = __uint_as_float(xr.x << 16), xv[1] = __uint_as_float(xr.x & 0xffff0000u);
            xv[2] = __uint_as_float(xr.y << 16), xv[3] = __uint_as_float(xr.y & 0xffff0000u);
            if (e.by) {
              const uint2 yr = *reinterpret_cast<const uint2*>(e.by + off);
              yv[0] = __uint_as_float(yr.x << 16), yv[1] = __uint_as_float(yr.x & 0xffff0000u);
              yv[2] = __uint_as_float(yr.y << 16), yv[3] = __uint_as_float(yr.y & 0xffff0000u);
            }
          }
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float v = bf16_to_f32(f32_to_bf16(acc[i][j][4 * g + q]));
            if (bwd) {
              const float gz = yv[q] > 0.f ? v : 0.f;
              s1[g][q] += gz;
              s2[g][q] = fmaf(gz, xv[q] - mu[q], s2[g][q]);
            } else {
              const float d = v - sh[g][q];
              s1[g][q] += d;
              s2[g][q] = fmaf(d, d, s2[g][q]);
            }
          }
        }
      }
      // rows r and r ^ 16 of each column: 32 independent shuffles, one wait
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          s1[g][q] += __shfl_xor(s1[g][q], 16, 64);
          s2[g][q] += __shfl_xor(s2[g][q], 16, 64);
        }
      __syncthreads();  // LDS free (main loop, or the previous pass's reads)
      if ((lane & 16) == 0) {
        const int r16 = lane & 15;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int c = wn * 32 + 8 * g + 4 * h;
          *reinterpret_cast<f32x4*>(s1p + (wm * 16 + r16) * CW + c) = f32x4{s1[g][0], s1[g][1], s1[g][2], s1[g][3]};
          *reinterpret_cast<f32x4*>(s2p + (wm * 16 + r16) * CW + c) = f32x4{s2[g][0], s2[g][1], s2[g][2], s2[g][3]};
          if (r16 == 0)
            *reinterpret_cast<f32x4*>(shp + wm * CW + c) = f32x4{sh[g][0], sh[g][1], sh[g][2], sh[g][3]};
        }
      }
      __syncthreads();
      if (tid < CFG::WAVES_M * CW) {
        const int w = tid / CW, c = tid % CW;
        float a1 = 0.f, a2 = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          a1 += s1p[(w * 16 + r) * CW + c];
          a2 += s2p[(w * 16 + r) * CW + c];
        }
        keep[j][0] = shp[w * CW + c];
        keep[j][1] = a1;
        keep[j][2] = a2;
      }
    }
    __syncthreads();  // pass buffers dead -> merge buffer
    float* red = reinterpret_cast<float*>(smem);  // [WAVES_M][BN] x (shift, s1, s2)
    if (tid < CFG::WAVES_M * CW) {
      const int w = tid / CW, c = tid % CW, wcol = c / 32, cc = c % 32;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        float* dst = red + (w * CFG::BN + wcol * 32 * FN + j * 32 + cc) * 3;
        dst[0] = keep[j][0];
        dst[1] = keep[j][1];
        dst[2] = keep[j][2];
      }
    }
    __syncthreads();
    Moments mo{0.f, 0.f, 0.f};
    if (tid < CFG::BN) {
#pragma unroll
      for (int w = 0; w < CFG::WAVES_M; ++w) {
        const float* src = red + (w * CFG::BN + tid) * 3;
        const float cnt = float(max(0, min(32 * FM, p.M - (m0 + w * 32 * FM))));
        if (bwd) {
          mo = bn_merge(true, mo, Moments{cnt, src[1], src[2]});
        } else if (cnt > 0.f) {
          const float mu = src[1] / cnt;
          mo = moments_merge(mo, Moments{cnt, src[0] + mu, fmaxf(src[2] - src[1] * mu, 0.f)});
        }
      }
    }
    __syncthreads();
    if (e.mode != 1) bn_epilogue_reduce<CFG, bwd>(p, mo, tm, tn, tiles_m, smem);
    __syncthreads();  // the bf16 staging below reuses the LDS
  }
  // bias, GELU (+ pre-activation, stored directly), residual: in place on acc
  if constexpr (EPI != 0)
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int m = row_of(i), n = col_of(j, g);
        if (m >= p.M || n >= p.N) continue;
        float v[4] = {acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]};
        if (p.bias) {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            v[e] += p.bias_bf16 ? bf16_to_f32(reinterpret_cast<const uint16_t*>(p.bias)[n + e])
                                : reinterpret_cast<const float*>(p.bias)[n + e];
        }
        const int64_t off = int64_t(m) * p.ldc + n;
        if constexpr (EPI == 1) {
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
        }
        if (!p.c_bf16)
          *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(p.c) + off) = f32x4{v[0], v[1], v[2], v[3]};
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[i][j][4 * g + e] = v[e];
      }
  if constexpr (EPI == 0) {
    if (!p.c_bf16) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int m = row_of(i), n = col_of(j, g);
            if (m < p.M && n < p.N)
              *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(p.c) + int64_t(m) * p.ldc + n) =
                  f32x4{acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]};
          }
      return;
    }
  }
  if (!p.c_bf16) return;
  // bf16 C goes out through LDS: a lane's 4-column groups sit on 32 different
  // rows, so direct 8-byte stores scatter over 32 rows per instruction; staged
  // through a padded [32 FM][BN] image (rows padded by 16 B: 2-way bank
  // conflicts at most), each thread then stores whole 16-byte row chunks, a
  // wave writing contiguous row segments per instruction.  One pass per wave
  // row (32 FM rows), so the image fits the single-buffer LDS of the
  // 4-workgroup/CU Tile128 schedule (17 KB) and Tile256's 128 KB (68 KB).
  constexpr int LROW = CFG::BN * 2 + 16, CPR = CFG::BN / 8;
  // one pass over the whole tile when the kernel's LDS holds its image
  // (smem_bytes), else one pass per wave row
  constexpr bool ONE = CFG::BM * LROW <= SMEM;
  constexpr int PASSES = ONE ? 1 : CFG::WAVES_M, ROWS = CFG::BM / PASSES;
  static_assert(ROWS * LROW <= SMEM, "epilogue image must fit the kernel's LDS");
  static_assert((ROWS * CPR) % CFG::NT == 0, "whole chunks per thread");
#pragma unroll
  for (int pass = 0; pass < PASSES; ++pass) {
    __syncthreads();  // LDS free: main loop (or previous pass) done
    if (ONE || wm == pass) {
      const int rbase = ONE ? wm * 32 * FM : 0;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int r = rbase + i * 32 + (lane & 31), c = wn * 32 * FN + j * 32 + 8 * g + 4 * h;
            *reinterpret_cast<uint2*>(smem + r * LROW + c * 2) =
                uint2{pack_bf16x2(acc[i][j][4 * g], acc[i][j][4 * g + 1]),
                      pack_bf16x2(acc[i][j][4 * g + 2], acc[i][j][4 * g + 3])};
          }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < ROWS * CPR / CFG::NT; ++q) {
      const int chunk = q * CFG::NT + tid, r = chunk / CPR, c = chunk % CPR;
      const int m = m0 + pass * ROWS + r, n = n0 + c * 8;
      if (m < p.M && n < p.N)
        *reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(p.c) + int64_t(m) * p.ldc + n) =
            *reinterpret_cast<const uint4*>(smem + r * LROW + c * 16);
    }
  }
}

// Reduce the fragment-native split-K slabs of a launch without counters
// (`splits` slices of every tile) into C (bf16 or fp32, row stride ldc).  One
// thread per 4-value group, spread over the whole chip (a workgroup per tile
// left most CUs idle); consecutive threads read consecutive 16-byte groups of
// each slice, four slices in flight.
template <class CFG>
__global__ __launch_bounds__(256) void tile_slab_reduce_kernel(const float* __restrict__ slabs, int splits, int M, int N,
                                                               int64_t ldc, void* out, int out_bf16, int variant,
                                                               int tiles_m, int tiles_n) {
  using SG = SlabGeom<CFG>;
  constexpr int FN = CFG::FN, FM = CFG::FM, GPT = SG::TILEF / 4;  // 4-value groups per tile
  const int tiles = tiles_m * tiles_n;
  const int64_t e = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (e >= int64_t(tiles) * GPT) return;
  const int t = int(e / GPT), r = int(e % GPT);
  const int wave = r / (SG::QN * 64), q = (r / 64) % SG::QN, lane = r % 64;
  const f32x4* src = reinterpret_cast<const f32x4*>(slabs) + e;
  const int64_t stride = int64_t(tiles) * GPT;  // groups per slice
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  int s = 0;
  for (; s + 4 <= splits; s += 4) {
    f32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = src[(s + u) * stride];
#pragma unroll
    for (int u = 0; u < 4; ++u) acc += v[u];
  }
  for (; s < splits; ++s) acc += src[s * stride];
  int tm, tn;
  tile_coords(variant, t, tiles_m, tiles_n, tm, tn);
  const int wm = wave / CFG::WAVES_N, wn = wave % CFG::WAVES_N;
  const int i = q / (4 * FN), j = (q / 4) % FN, g = q % 4;
  const int m = tm * CFG::BM + wm * 32 * FM + i * 32 + (lane & 31);
  const int n = tn * CFG::BN + wn * 32 * FN + j * 32 + 8 * g + 4 * (lane >> 5);
  if (m < M && n < N) {
    const int64_t off = int64_t(m) * ldc + n;
    if (out_bf16)
      *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(out) + off) =
          uint2{pack_bf16x2(acc[0], acc[1]), pack_bf16x2(acc[2], acc[3])};
    else
      *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(out) + off) = acc;
  }
}

template <class CFG>
inline int gemm_grid(const GemmParams& p, int& tiles_m, int& tiles_n) {
  tiles_m = (p.M + CFG::BM - 1) / CFG::BM;
  tiles_n = (p.N + CFG::BN - 1) / CFG::BN;
  return tiles_m * tiles_n * (p.splits > 1 ? p.splits : 1);
}

}  // namespace p2gemm
