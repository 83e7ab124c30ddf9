// Ping-pong GEMM for the Linear layers: 256 x 256 output tile, 8 waves, one
// workgroup per CU, operands streamed HBM -> LDS continuously (gfx950).
//
// Why a second pipeline next to gemm_core.h's: that one stages a whole K-tile
// (64 KB) per iteration and waits for it with vmcnt(0) + a full barrier, so
// at one workgroup per CU every K-tile starts with the waves parked on the
// DMA (27 % of the 8192^3 run, profiles/r2_gemm_256.md) and nothing overlaps
// the LDS fragment reads with the matrix pipe.  Here:
//
// * Each K-tile (BK = 64) is consumed in four PHASES, one 64 x 32 quadrant of
//   the wave's 128 x 64 output per phase (8 x v_mfma_f32_32x32x16_bf16):
//     ph1 (a-lo, b-lo)  ph2 (a-lo, b-hi)  ph3 (a-hi, b-hi)  ph4 (a-hi, b-lo)
//   (b-lo is read again in ph4 rather than held: 16 fewer VGPRs) where a-lo / a-hi are the A rows of the tile's two 128-row halves and
//   b-lo / b-hi the B rows of its two halves.  A wave (wr, wc) owns A rows
//   {64 wr, 128 + 64 wr} + [0, 64) and B rows {32 wc, 128 + 32 wc} + [0, 32),
//   so each operand half is one contiguous 16 KB LDS piece.
// * The LDS holds two K-tiles (buffers) of four pieces.  Every phase issues
//   the DMA of ONE piece (16 KB: 2 x global_load_lds_dwordx4 per lane) into a
//   piece whose last fragment read has retired, so the loads stream
//   continuously, ~3 pieces in flight; the counted `s_waitcnt vmcnt(6)` at
//   phases 4 and 8 retires exactly the K-tile read next, never vmcnt(0)
//   inside the loop.  Piece schedule (tile t in buffer 0, t+1 in buffer 1):
//     ph1 Blo(t+1)->b1   ph2 Alo(t+2)->b0   ph3 Bhi(t+2)->b0  ph4 Ahi(t+2)->b0
//     ph5 Blo(t+2)->b0   ph6 Alo(t+3)->b1   ph7 Bhi(t+3)->b1  ph8 Ahi(t+3)->b1
//   (a piece is restaged one phase after the phase that read it; those reads
//   are retired by the lgkmcnt(0) ahead of that phase's first barrier).
// * Two barriers per phase and the waves 4-7 one barrier behind waves 0-3:
//   each SIMD holds one wave of each half, so while one wave runs its MFMA
//   cluster the other issues its fragment reads and DMA -- the matrix pipe is
//   never waiting on LDS latency (ping-pong).  Raw s_barrier, never
//   __syncthreads(): its fence would drain the in-flight DMA.
// * Operand chunks, swizzles and fragment reads are gemm_core.h's (k-major
//   ds_read_b128, m/n-major ds_read_b64_tr_b16 transpose reads); rows past M /
//   N are clamped onto the last row (their outputs are never stored), k past
//   K reads the zero page.  Epilogue (split-K reduction, bias / GELU /
//   residual, LDS-staged bf16 stores) is gemm_core.h's.
//
// Selected by GemmParams::variant bit 11 (ops/gemm.py).  Reference layer
// shapes: /root/reference/p2pfl/learning/pytorch/mnist_examples/models/mlp.py:53-69
// and the ViT-B/16 of BASELINE config 4.
#include "gemm_core.h"

namespace p2gemm {

using PPCfg = Tile256;  // 256 x 256, 8 waves as 2 x 4, FM = 4, FN = 2

typedef int i32x4 __attribute__((ext_vector_type(4)));

// One 16-byte-per-lane LDS DMA through a raw buffer resource: `desc` (SGPRs)
// covers the bytes from the chunk row's start to the end of the operand, so
// any lane whose offset falls past the operand (rows past M / N of a k-major
// operand, k rows past K of an m/n-major one) receives zeros from the
// hardware range check -- no per-lane zero-page select.  soffset stays 0 (it
// is not range-checked).
P2_DEVICE void dma_buf16(const i32x4& desc, uint32_t voff, char* lds_dst) {
  const uint32_t m0v = __builtin_amdgcn_readfirstlane(uint32_t(reinterpret_cast<uintptr_t>(lds_dst)));
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %3\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(desc), "s"(m0v)
      : "memory");
}

P2_DEVICE i32x4 buf_desc(const char* base, int64_t bytes) {
  const uint64_t b = reinterpret_cast<uint64_t>(base);
  i32x4 d;
  d.x = __builtin_amdgcn_readfirstlane(int(uint32_t(b)));
  d.y = __builtin_amdgcn_readfirstlane(int(uint32_t(b >> 32)));  // stride 0: raw buffer
  d.z = __builtin_amdgcn_readfirstlane(int(bytes > 0 ? uint32_t(bytes) : 0u));
  d.w = 0x00020000;  // gfx9 raw-buffer dword 3 (dword loads, no swizzle)
  return d;
}

// One operand's DMA sources for this thread: both 128-row halves, the thread's
// two chunks (i = 2 grp + c of gemm_core.h's 256-thread chunk geometry).  The
// per-lane part of a chunk's address is one VGPR (k-major: both halves and
// chunks differ by whole rows, folded into the wave-uniform descriptor base;
// m/n-major: one per half, columns past the operand clamped onto its last
// chunk -- their outputs are never stored).
template <bool KMAJ>
struct PPSrc {
  const char* g;
  int64_t total;        // operand bytes
  int64_t ub0[2][2];    // [half][chunk] wave-uniform byte offset of the chunk row at k0 = 0
  int64_t kstep;        // bytes per unit of k0 (2 for k-major, 2 ld for m/n-major)
  uint32_t voff[2];     // per-lane byte offset ([half] for m/n-major)

  P2_DEVICE void init(const uint16_t* g_, int64_t ld, int nrows, int K, int r0, int grp, int gt) {
    g = reinterpret_cast<const char*>(g_);
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int i = 2 * grp + c;
#pragma unroll
      for (int h = 0; h < 2; ++h)
        ub0[h][c] = KMAJ ? int64_t(r0 + 128 * h + 32 * i) * ld * 2 : int64_t(16 * i) * ld * 2;
    }
    if constexpr (KMAJ) {
      total = int64_t(nrows) * ld * 2;
      kstep = 2;
      voff[0] = voff[1] = uint32_t(((gt >> 3) * ld + kmaj_k(gt)) * 2);
    } else {
      total = int64_t(K) * ld * 2;
      kstep = ld * 2;
#pragma unroll
      for (int h = 0; h < 2; ++h) voff[h] = uint32_t(((gt >> 4) * ld + min(r0 + 128 * h + mnmaj_col(gt), nrows - 8)) * 2);
    }
  }
  // chunk c of half h for the K-tile at k0 into LDS `dst`
  P2_DEVICE void dma(int h, int c, int k0, char* dst) const {
    const int64_t ub = ub0[h][c] + int64_t(k0) * kstep;
    dma_buf16(buf_desc(g + ub, total - ub), voff[KMAJ ? 0 : h], dst);
  }
};

// Per-lane byte offset, within an m/n-major piece ([64 k][128] bf16, 256-B
// rows), of transpose read t (0, 1) of the 32-column fragment at column rb for
// k-substep 0 (gemm_core.h frag<false>; k-substep ks adds 16 rows = 4096 B).
P2_DEVICE uint32_t mn_base(int rb, int t, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int col = rb + 16 * (g & 1) + 4 * p;
  const int row = 8 * (g >> 1) + 4 * t + q;
  return row * 256 + (((col >> 3) ^ swz_mn(row)) << 4) + (col & 7) * 2;
}

// EPI (epilogue_kind): 0 = plain product (no split-K, bias, GELU, residual),
// 2 = bias only, 1 = every epilogue feature behind runtime flags.  The plain instance's epilogue is a few hundred
// instructions instead of ~60 KB of unrolled bias / GELU / split-K code: run once
// per tile, straight-line, that code is fetched cold from L2 by every workgroup,
// and on the short-K ViT products the fetch stalls cost more than the stores
// (scripts/gemm_anatomy.py: 12.5 us for a launch with the K loop switched off).
template <class SA, class SB, bool KA, bool KB, int EPI>
__global__ __launch_bounds__(512) void gemm_pp_kernel(GemmParams p, int tiles_m, int tiles_n) {
  __shared__ __attribute__((aligned(16))) char smem[smem_bytes<PPCfg, 2>()];
  constexpr int FM = PPCfg::FM, FN = PPCfg::FN, STG = PPCfg::STAGE;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;  // waves 0-3: wr = 0 (one per SIMD), 4-7: wr = 1
  const int grp = __builtin_amdgcn_readfirstlane(tid >> 8), gt = tid & 255;  // staging group (wave-uniform)
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tiles = tiles_m * tiles_n;
  const int split = bid / tiles, t = bid % tiles;
  int tm, tn;
  {  // grouped tile order (8 tile rows per column step), as gemm_body
    constexpr int GROUP_M = 8;
    const int per_group = GROUP_M * tiles_n, g0 = (t / per_group) * GROUP_M;
    const int gsize = min(tiles_m - g0, GROUP_M), r = t % per_group;
    tm = g0 + r % gsize;
    tn = r / gsize;
  }
  const int m0 = tm * 256, n0 = tn * 256;
  int kper = (p.K + p.splits - 1) / p.splits;
  kper = (kper + BK - 1) / BK * BK;
  const int kb = split * kper, ke = min(p.K, kb + kper);
  // timing probes (variant bits): 12 no DMA after the prologue, 13 no stagger,
  // 14 no C stores, 15 no K loop
  const int probe = p.variant >> 12;
  const int nt = (ke > kb && !(probe & 8)) ? (ke - kb + BK - 1) / BK : 0;
  const bool dma_on = !(probe & 1), stag = !(probe & 2);

  SA sa;
  SB sb;
  sa.init(p.a, p.lda, p.M, p.K, m0, grp, gt);
  sb.init(p.b, p.ldb, p.N, p.K, n0, grp, gt);

  f32x16 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  // LDS: piece q (0 Alo, 1 Ahi, 2 Blo, 3 Bhi) of buffer b at (2 q + b) x 16 KB,
  // so every fragment read below is one per-lane base VGPR + an immediate
  // offset below 64 KB (A pieces in the first 64 KB, B pieces in the second)
  auto stage = [&](int q, int tile, int buf) __attribute__((always_inline)) {
    const int k0 = kb + tile * BK;
    char* dst = smem + (2 * q + buf) * TILE;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      char* d = dst + ((2 * grp + c) * 256 + (wave & 3) * 64) * 16;  // lane L writes d + 16 L
      if (q < 2)
        sa.dma(q, c, k0, d);
      else
        sb.dma(q - 2, c, k0, d);
    }
  };
  // per-lane LDS base addresses (bytes from smem) of the fragment reads:
  //   k-major: [k-substep], mn-major (two transpose reads per fragment): [row block][t]
  const int l31 = lane & 31, hi = lane >> 5;
  uint32_t va[4], vb[4];
  if constexpr (KA) {
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) va[ks] = (64 * wr + l31) * 128 + ((((2 * ks) | hi) ^ ((l31 >> 1) & 7)) << 4);
  } else {
#pragma unroll
    for (int u = 0; u < 4; ++u) va[u] = mn_base(64 * wr + 32 * (u >> 1), u & 1, lane);
  }
  if constexpr (KB) {
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) vb[ks] = 4 * TILE + (32 * wc + l31) * 128 + ((((2 * ks) | hi) ^ ((l31 >> 1) & 7)) << 4);
  } else {
#pragma unroll
    for (int u = 0; u < 2; ++u) vb[u] = 4 * TILE + mn_base(32 * wc, u, lane);
  }
  // fragment (row block i, k-substep ks) of piece `half` in buffer `buf`
  auto frag_pp = [&](const uint32_t* v, bool kmaj, int half, int buf, int i, int ks) __attribute__((always_inline)) {
    const int cst = (2 * half + buf) * TILE;
    if (kmaj) return *reinterpret_cast<const uint4*>(smem + v[ks] + cst + i * 32 * 128);
    uint4 out;
    const s16x4 x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4*)(smem + v[2 * i] + cst + ks * 4096));
    const s16x4 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4*)(smem + v[2 * i + 1] + cst + ks * 4096));
    const uint2 u0 = __builtin_bit_cast(uint2, x0), u1 = __builtin_bit_cast(uint2, x1);
    out.x = u0.x;
    out.y = u0.y;
    out.z = u1.x;
    out.w = u1.y;
    return out;
  };
  uint4 fa[2][4], fb[4];  // fa[row block][k-substep], fb[k-substep]
  auto read_a = [&](int buf, int h) __attribute__((always_inline)) {
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int i = 0; i < 2; ++i) fa[i][ks] = frag_pp(va, KA, h, buf, i, ks);
  };
  auto read_b = [&](int buf, int h) __attribute__((always_inline)) {
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) fb[ks] = frag_pp(vb, KB, h, buf, 0, ks);
  };
  auto mma = [&](int h, int g) __attribute__((always_inline)) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int i = 0; i < 2; ++i) acc[2 * h + i][g] = mfma(fb[ks], fa[i][ks], acc[2 * h + i][g]);
    __builtin_amdgcn_s_setprio(0);
  };
  // phase boundaries: reads retired before the first barrier (so the piece
  // can be restaged next phase), MFMA cluster between the two barriers
  auto bar = []() __attribute__((always_inline)) {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  auto lgkm0 = []() __attribute__((always_inline)) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  auto vm6 = []() __attribute__((always_inline)) { asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); };
  auto vm0 = []() __attribute__((always_inline)) { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); };

  if (nt > 0) {
    // prologue: tile 0 whole into buffer 0; tile 1's Alo, Bhi, Ahi into buffer 1
#pragma unroll
    for (int q = 0; q < 4; ++q) stage(q, 0, 0);
    if (nt > 1) {
      stage(0, 1, 1);
      stage(3, 1, 1);
      stage(1, 1, 1);
      vm6();
    } else {
      vm0();
    }
    bar();
    if (stag && wr == 1) bar();  // stagger: waves 4-7 run one barrier behind
    constexpr int b0 = 0, b1 = 1;
    for (int it = 0; it < nt; it += 2) {
      const bool n1 = it + 1 < nt, n2 = dma_on && it + 2 < nt, n3 = dma_on && it + 3 < nt;
      // ph1: (a-lo, b-lo) of tile it; Blo of tile it + 1 -> buffer 1
      read_a(b0, 0);
      read_b(b0, 0);
      if (dma_on && n1) stage(2, it + 1, 1);
      lgkm0();
      bar();
      mma(0, 0);
      bar();
      // ph2: (a-lo, b-hi); Alo(it + 2) -> buffer 0
      read_b(b0, 1);
      if (n2) stage(0, it + 2, 0);
      lgkm0();
      bar();
      mma(0, 1);
      bar();
      // ph3: (a-hi, b-hi); Bhi(it + 2)
      read_a(b0, 1);
      if (n2) stage(3, it + 2, 0);
      lgkm0();
      bar();
      mma(1, 1);
      bar();
      // ph4: (a-hi, b-lo re-read); Ahi(it + 2); retire tile it + 1
      read_b(b0, 0);
      if (n2) {
        stage(1, it + 2, 0);
        vm6();
      } else {
        vm0();
      }
      lgkm0();
      bar();
      mma(1, 0);
      bar();
      if (!n1) break;
      // ph5..ph8: tile it + 1 from buffer 1; Blo(it + 2) -> buffer 0, then tile it + 3 -> buffer 1
      read_a(b1, 0);
      read_b(b1, 0);
      if (n2) stage(2, it + 2, 0);
      lgkm0();
      bar();
      mma(0, 0);
      bar();
      read_b(b1, 1);
      if (n3) stage(0, it + 3, 1);
      lgkm0();
      bar();
      mma(0, 1);
      bar();
      read_a(b1, 1);
      if (n3) stage(3, it + 3, 1);
      lgkm0();
      bar();
      mma(1, 1);
      bar();
      read_b(b1, 0);
      if (n3) {
        stage(1, it + 3, 1);
        vm6();
      } else {
        vm0();
      }
      lgkm0();
      bar();
      mma(1, 0);
      bar();
    }
    if (stag && wr == 0) bar();  // balance the stagger
  }
  // ---- epilogue.  Block (i, j) of the wave: i = 2 h + i' -> tile rows
  // 128 h + 64 wr + 32 i', j -> tile cols 128 j + 32 wc; lane holds rows
  // (lane & 31), columns 8 g + 4 (lane >> 5) + e in acc[i][j][4 g + e].
  // Written for a low register peak: every finished 4-value group leaves
  // for LDS (bf16) or memory (fp32) at once, and the split-K reducer rebuilds
  // one block at a time from the slabs.  The lane id is re-derived (opaque to
  // the compiler) so no lane value of the prologue stays live across the loop.
  int ln;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
  const int tid2 = wave * 64 + ln, hh = ln >> 5;
  auto row_of = [&](int i) __attribute__((always_inline)) { return m0 + 128 * (i >> 1) + 64 * wr + 32 * (i & 1) + (ln & 31); };
  auto col_of = [&](int j, int g) __attribute__((always_inline)) { return n0 + 128 * j + 32 * wc + 8 * g + 4 * hh; };
  constexpr int LROW = 256 * 2 + 16;  // bf16 staging image [256][256] + 16 B row pad
  const int64_t mn = int64_t(p.M) * p.N;
  float* slabs = p.counters ? p.ws : reinterpret_cast<float*>(p.c);
  if (EPI == 1 && p.splits > 1) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int m = row_of(i), n = col_of(j, g);
          if (m < p.M && n < p.N)
            *reinterpret_cast<f32x4*>(slabs + split * mn + int64_t(m) * p.N + n) =
                f32x4{acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]};
        }
    if (!p.counters) return;
    // in-launch reduction by the last slice to arrive (agent-scope release
    // before the ticket, acquire after it; counter reset for the next launch)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = reinterpret_cast<int*>(smem);
    if (tid2 == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const int old = __hip_atomic_fetch_add(p.counters + t, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      flag[0] = old == p.splits - 1;
    }
    __syncthreads();
    if (!flag[0]) return;
    if (tid2 == 0) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(p.counters + t, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();  // LDS free (main loop / flag) for the bf16 staging image
  auto finish = [&](int i, int j, int g, float v0, float v1, float v2, float v3) __attribute__((always_inline)) {
    const int m = row_of(i), n = col_of(j, g);
    if (m >= p.M || n >= p.N) return;
    float v[4] = {v0, v1, v2, v3};
    const int64_t off = int64_t(m) * p.ldc + n;
    if constexpr (EPI != 0) {
    if (p.bias) {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        v[e] += p.bias_bf16 ? bf16_to_f32(reinterpret_cast<const uint16_t*>(p.bias)[n + e])
                            : reinterpret_cast<const float*>(p.bias)[n + e];
    }
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
    }
    if (!p.c_bf16) {
      *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(p.c) + off) = f32x4{v[0], v[1], v[2], v[3]};
    } else {
      const int r = m - m0, c = n - n0;
      *reinterpret_cast<uint2*>(smem + r * LROW + c * 2) = uint2{pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3])};
    }
  };
  if (EPI == 1 && p.splits > 1) {  // the reducer: one 4-value group of all slices at a time (acc is in its own slab)
    for (int i = 0; i < FM; ++i)
      for (int j = 0; j < FN; ++j)
        for (int g = 0; g < 4; ++g) {
          const int m = row_of(i), n = col_of(j, g);
          f32x4 sum = {0.f, 0.f, 0.f, 0.f};
          if (m < p.M && n < p.N)
            for (int s2 = 0; s2 < p.splits; ++s2) sum += *reinterpret_cast<const f32x4*>(slabs + s2 * mn + int64_t(m) * p.N + n);
          finish(i, j, g, sum[0], sum[1], sum[2], sum[3]);
        }
  } else {  // fully unrolled: acc is only ever indexed by constants (else it lands in scratch)
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g)
          finish(i, j, g, acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]);
  }
  if (!p.c_bf16 || (probe & 4)) return;
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 256 * 32 / 512; ++q) {  // 256 rows x 32 16-byte chunks
    const int chunk = q * 512 + tid2, r = chunk >> 5, c = chunk & 31;
    const int m = m0 + r, n = n0 + c * 8;
    if (m < p.M && n < p.N)
      *reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(p.c) + int64_t(m) * p.ldc + n) =
          *reinterpret_cast<const uint4*>(smem + r * LROW + c * 16);
  }
}

template <bool KA, bool KB>
static void launch_pp(const GemmParams& p, hipStream_t s) {
  const int tm = (p.M + 255) / 256, tn = (p.N + 255) / 256;
  const int grid = tm * tn * (p.splits > 1 ? p.splits : 1);
  switch (epilogue_kind(p)) {
    case 0:
      hipLaunchKernelGGL((gemm_pp_kernel<PPSrc<KA>, PPSrc<KB>, KA, KB, 0>), dim3(grid), dim3(512), 0, s, p, tm, tn);
      break;
    case 2:
      hipLaunchKernelGGL((gemm_pp_kernel<PPSrc<KA>, PPSrc<KB>, KA, KB, 2>), dim3(grid), dim3(512), 0, s, p, tm, tn);
      break;
    default:
      hipLaunchKernelGGL((gemm_pp_kernel<PPSrc<KA>, PPSrc<KB>, KA, KB, 1>), dim3(grid), dim3(512), 0, s, p, tm, tn);
  }
}

}  // namespace p2gemm

namespace p2 {

using p2gemm::BK;

bool gemm_pp_supported(const GemmParams& p) {
  // 32-bit element offsets within each operand
  // byte ranges of the buffer descriptors are 32-bit; a k-major operand's
  // K tail is not range-checked (k past K lies inside the next row)
  const int64_t na = p.a_kmajor ? int64_t(p.M) * p.lda : int64_t(p.K) * p.lda;
  const int64_t nb = p.b_kmajor ? int64_t(p.N) * p.ldb : int64_t(p.K) * p.ldb;
  const bool ktail_ok = (!p.a_kmajor && !p.b_kmajor) || p.K % BK == 0;
  return 2 * na < (int64_t(1) << 31) && 2 * nb < (int64_t(1) << 31) && p.M >= 8 && p.N >= 8 && ktail_ok;
}

void gemm_bf16_pp(const GemmParams& p, hipStream_t s) {
  using namespace p2gemm;
  if (p.a_kmajor && p.b_kmajor)
    launch_pp<true, true>(p, s);
  else if (p.a_kmajor)
    launch_pp<true, false>(p, s);
  else if (p.b_kmajor)
    launch_pp<false, true>(p, s);
  else
    launch_pp<false, false>(p, s);
}

}  // namespace p2
