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
#include <type_traits>

#include "gemm_core.h"

namespace p2gemm {

using PPCfg = Tile256;  // 256 x 256, 8 waves as 2 x 4, FM = 4, FN = 2
constexpr int PP_M16 = 1 << 16;  // variant bit: 16x16x32 MFMA form
constexpr int PP_SK = 1 << 17;   // variant bit: stream-K schedule (GemmParams::splits = grid size)

// Stream-K: the T = tiles x KT K-tile iterations of the product are cut into G
// equal contiguous ranges, one per workgroup (w covers [sk_begin(w), sk_begin(w + 1))),
// in tile-major order, so every CU runs the same number of MFMA K-tiles whatever
// the tile count (75 tiles of 256 x 256 on 256 CUs: 14 K-tiles each instead of
// 48 on 75 CUs).  A workgroup's range is at most two partial tiles (its first
// and its last) around whole ones.
P2_DEVICE int sk_begin(int w, int total, int G) { return int(int64_t(w) * total / G); }
P2_DEVICE int sk_owner(int i, int total, int G) { return int((int64_t(i + 1) * G - 1) / total); }
// XCD of remapped workgroup id b (the inverse of gemm_core.h's xcd_remap)
P2_DEVICE int xcd_of(int b, int nwg) {
  const int q = nwg / 8, r = nwg % 8;
  return b < r * (q + 1) ? b / (q + 1) : r + (b - r * (q + 1)) / max(q, 1);
}

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
  d.z = __builtin_amdgcn_readfirstlane(int(uint32_t(bytes)));  // > 0: only K-tiles inside the operand are staged
  d.w = 0x00020000;  // gfx9 raw-buffer dword 3 (dword loads, no swizzle)
  return d;
}

// One operand's DMA sources for this thread: both 128-row halves, the thread's
// two chunks (i = 2 grp + c of gemm_core.h's 256-thread chunk geometry).  The
// K-tile at k0 is one wave-uniform buffer descriptor (base = operand + k0 x
// kstep, range = the bytes from there to the operand's end), and every chunk's
// row / column / lane offset a VGPR relative to it, so a piece's DMA costs two
// scalar ops for the descriptor and the m0 hand-off per load (a descriptor per
// chunk cost ~14 scalar ops each, on the read side of every phase).  Rows past
// M / N of a k-major operand and k rows past K of an m/n-major one fall past
// the range and read zeros; m/n-major columns past the operand are clamped
// onto its last chunk (their outputs are never stored).
template <bool KMAJ>
struct PPSrc {
  const char* g;
  int64_t total;        // operand bytes
  int64_t kstep;        // bytes per unit of k0 (2 for k-major, 2 ld for m/n-major)
  uint32_t voff[2][2];  // [half][chunk] per-lane byte offset from the K-tile's base

  P2_DEVICE void init(const uint16_t* g_, int64_t ld, int nrows, int K, int r0, int grp, int gt) {
    g = reinterpret_cast<const char*>(g_);
    total = KMAJ ? int64_t(nrows) * ld * 2 : int64_t(K) * ld * 2;
    kstep = KMAJ ? 2 : ld * 2;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int i = 2 * grp + c;
#pragma unroll
      for (int h = 0; h < 2; ++h)
        voff[h][c] = KMAJ ? uint32_t((int64_t(r0 + 128 * h + 32 * i + (gt >> 3)) * ld + kmaj_k(gt)) * 2)
                          : uint32_t((int64_t(16 * i + (gt >> 4)) * ld + min(r0 + 128 * h + mnmaj_col(gt), nrows - 8)) * 2);
    }
  }
  P2_DEVICE i32x4 desc(int k0) const {
    const int64_t ub = int64_t(k0) * kstep;
    return buf_desc(g + ub, total - ub);
  }
  // chunk c of half h of the K-tile whose descriptor is d into LDS `dst`
  P2_DEVICE void dma(const i32x4& d, int h, int c, char* dst) const { dma_buf16(d, voff[h][c], dst); }
};

// Per-lane byte offset, within an m/n-major piece ([64 k][128] bf16, 256-B
// rows), of transpose read t (0, 1) of the fragment at column rb for
// k-substep 0.  32x32x16 operand (gemm_core.h frag<false>): 32 columns, lane
// group g takes columns 16 (g & 1) and k rows 8 (g >> 1) + 4 t + [0, 4);
// k-substep ks adds 16 rows = 4096 B.  16x16x32 operand (M16): 16 columns,
// group g takes k rows 8 g + 4 t + [0, 4); ks adds 32 rows = 8192 B.  Both are
// conflict-free on the swz_mn image (a 32-lane half reads two 4-row blocks 8
// rows apart in the same columns, or 4 rows of 32 columns).
template <bool M16>
P2_DEVICE uint32_t mn_base(int rb, int t, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int col = M16 ? rb + 4 * p : rb + 16 * (g & 1) + 4 * p;
  const int row = (M16 ? 8 * g : 8 * (g >> 1)) + 4 * t + q;
  return row * 256 + (((col >> 3) ^ swz_mn(row)) << 4) + (col & 7) * 2;
}

P2_DEVICE f32x4 mfma16(uint4 a, uint4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c,
                                                  0, 0, 0);
}

// M16: the same schedule on v_mfma_f32_16x16x32_bf16 (variant bit 16): equal
// MFMA cycles per FLOP, but the chip holds a higher clock under the 16x16 form
// (MI355X_MICROARCH.md, DVFS item 7: 1.12-1.15x FLOP/s in LDS-fed loops).  Per
// phase a wave runs 4 x 2 blocks of 16 x 16 over 2 k-substeps of 32 (16 MFMAs
// of 16 cycles) from the same 8 + 4 fragment registers; accumulators are
// [8][4] f32x4 instead of [4][2] f32x16 (same 128 registers).
//
// EPI (epilogue_kind): 0 = plain product (no split-K, bias, GELU, residual),
// 2 = bias only, 1 = every epilogue feature behind runtime flags.  The plain instance's epilogue is a few hundred
// instructions instead of ~60 KB of unrolled bias / GELU / split-K code: run once
// per tile, straight-line, that code is fetched cold from L2 by every workgroup,
// and on the short-K ViT products the fetch stalls cost more than the stores
// (scripts/gemm_anatomy.py: 12.5 us for a launch with the K loop switched off).
template <class SA, class SB, bool KA, bool KB, int EPI, bool M16, bool SK>
__global__ __launch_bounds__(512) void gemm_pp_kernel(GemmParams p, int tiles_m, int tiles_n) {
  __shared__ __attribute__((aligned(16))) char smem[smem_bytes<PPCfg, 2>()];
  constexpr int FM = PPCfg::FM, FN = PPCfg::FN, STG = PPCfg::STAGE;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;  // waves 0-3: wr = 0 (one per SIMD), 4-7: wr = 1
  const int grp = __builtin_amdgcn_readfirstlane(tid >> 8), gt = tid & 255;  // staging group (wave-uniform)
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tiles = tiles_m * tiles_n;
  // timing probes (variant bits): 12 no DMA after the prologue, 13 no stagger,
  // 14 no C stores, 15 no K loop
  const int probe = (p.variant >> 12) & 15;
  const bool dma_on = !(probe & 1), stag = !(probe & 2);
  // stream-K range of this workgroup (consecutive ids share an XCD, so the
  // workgroups of one tile mostly do too)
  const int KT = (p.K + BK - 1) / BK, total = tiles * KT, G = gridDim.x;
  int it = SK ? sk_begin(bid, total, G) : 0;
  const int it_end = SK ? sk_begin(bid + 1, total, G) : 0;
  int t = 0, split = 0, m0 = 0, n0 = 0, kb = 0, ke = 0, nt = 0;
  bool partial = false;

  SA sa;
  SB sb;

  // accumulator blocks [NI][NJ], NG groups of 4 values each (see row_of / col_of)
  constexpr int NI = M16 ? 8 : FM, NJ = M16 ? 4 : FN, NG = M16 ? 1 : 4;
  // fragments per phase: NA A row blocks, NB B column blocks, NKS k-substeps
  constexpr int NA = M16 ? 4 : 2, NB = M16 ? 2 : 1, NKS = M16 ? 2 : 4;
  constexpr int RBLK = M16 ? 16 : 32;             // rows per fragment block
  constexpr int TR_KS = M16 ? 8192 : 4096;        // mn-major: bytes per k-substep
  using AccT = std::conditional_t<M16, f32x4, f32x16>;
  AccT acc[NI][NJ];

  // LDS: piece q (0 Alo, 1 Ahi, 2 Blo, 3 Bhi) of buffer b at (2 q + b) x 16 KB,
  // so every fragment read below is one per-lane base VGPR + an immediate
  // offset below 64 KB (A pieces in the first 64 KB, B pieces in the second)
  auto stage = [&](int q, int tile, int buf) __attribute__((always_inline)) {
    const int k0 = kb + tile * BK;
    char* dst = smem + (2 * q + buf) * TILE;
    const i32x4 d = q < 2 ? sa.desc(k0) : sb.desc(k0);
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      char* l = dst + ((2 * grp + c) * 256 + (wave & 3) * 64) * 16;  // lane L writes l + 16 L
      if (q < 2)
        sa.dma(d, q, c, l);
      else
        sb.dma(d, q - 2, c, l);
    }
  };
  // per-lane LDS base addresses (bytes from smem) of the fragment reads:
  //   k-major: [k-substep], mn-major (two transpose reads per fragment): [row block][t]
  //   k-major row reads: lane row r = RBLK-row block + (lane % RBLK), 16-B chunk
  //   (32x32x16) 2 ks + lane / 32 or (16x16x32) 4 ks + lane / 16 of its 128-B row
  const int lr = lane % RBLK, lc = lane / RBLK;
  auto kbase = [&](int row0, int ks) __attribute__((always_inline)) {
    const int c = M16 ? (4 * ks) | lc : (2 * ks) | lc;
    return uint32_t((row0 + lr) * 128 + ((c ^ ((lr >> 1) & 7)) << 4));
  };
  // k-major: one base per k-substep; mn-major: one per (block, transpose read)
  constexpr int NVA = KA ? NKS : 2 * NA, NVB = KB ? NKS : 2 * NB;
  uint32_t va[NVA], vb[NVB];
  if constexpr (KA) {
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) va[ks] = kbase(64 * wr, ks);
  } else {
#pragma unroll
    for (int u = 0; u < 2 * NA; ++u) va[u] = mn_base<M16>(64 * wr + RBLK * (u >> 1), u & 1, lane);
  }
  if constexpr (KB) {
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) vb[ks] = 4 * TILE + kbase(32 * wc, ks);
  } else {
#pragma unroll
    for (int u = 0; u < 2 * NB; ++u) vb[u] = 4 * TILE + mn_base<M16>(32 * wc + RBLK * (u >> 1), u & 1, lane);
  }
  // fragment (block i, k-substep ks) of piece `half` in buffer `buf`
  auto frag_pp = [&](const uint32_t* v, bool kmaj, int half, int buf, int i, int ks) __attribute__((always_inline)) {
    const int cst = (2 * half + buf) * TILE;
    if (kmaj) return *reinterpret_cast<const uint4*>(smem + v[ks] + cst + i * RBLK * 128);
    uint4 out;
    const s16x4 x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4*)(smem + v[2 * i] + cst + ks * TR_KS));
    const s16x4 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4*)(smem + v[2 * i + 1] + cst + ks * TR_KS));
    const uint2 u0 = __builtin_bit_cast(uint2, x0), u1 = __builtin_bit_cast(uint2, x1);
    out.x = u0.x;
    out.y = u0.y;
    out.z = u1.x;
    out.w = u1.y;
    return out;
  };
  uint4 fa[NA][NKS], fb[NB][NKS];  // [block][k-substep]
  auto read_a = [&](int buf, int h) __attribute__((always_inline)) {
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
      for (int i = 0; i < NA; ++i) fa[i][ks] = frag_pp(va, KA, h, buf, i, ks);
  };
  auto read_b = [&](int buf, int h) __attribute__((always_inline)) {
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
      for (int j = 0; j < NB; ++j) fb[j][ks] = frag_pp(vb, KB, h, buf, j, ks);
  };
  auto mma = [&](int h, int g) __attribute__((always_inline)) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
      for (int i = 0; i < NA; ++i)
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          if constexpr (M16)
            acc[NA * h + i][NB * g + j] = mfma16(fb[j][ks], fa[i][ks], acc[NA * h + i][NB * g + j]);
          else
            acc[NA * h + i][g] = mfma(fb[0][ks], fa[i][ks], acc[NA * h + i][g]);
        }
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

  for (;;) {  // one pass per tile segment (a single pass unless SK)
  if constexpr (SK) {
    if (it >= it_end) break;
    t = it / KT;
    const int k0i = it - t * KT, k1i = min(KT, k0i + (it_end - it));
    it += k1i - k0i;
    m0 = (t / tiles_n) * 256;  // tile-major: the workgroups of one XCD walk a few A row panels
    n0 = (t % tiles_n) * 256;
    kb = k0i * BK;
    ke = min(p.K, k1i * BK);
    partial = k0i != 0 || k1i != KT;
    nt = !(probe & 8) ? k1i - k0i : 0;
  } else {
    split = bid / tiles;
    t = bid % tiles;
    int tm, tn;
    {  // grouped tile order (8 tile rows per column step), as gemm_body
      constexpr int GROUP_M = 8;
      const int per_group = GROUP_M * tiles_n, g0 = (t / per_group) * GROUP_M;
      const int gsize = min(tiles_m - g0, GROUP_M), r = t % per_group;
      tm = g0 + r % gsize;
      tn = r / gsize;
    }
    m0 = tm * 256;
    n0 = tn * 256;
    int kper = (p.K + p.splits - 1) / p.splits;
    kper = (kper + BK - 1) / BK * BK;
    kb = split * kper;
    ke = min(p.K, kb + kper);
    nt = (ke > kb && !(probe & 8)) ? (ke - kb + BK - 1) / BK : 0;
  }
  sa.init(p.a, p.lda, p.M, p.K, m0, grp, gt);
  sb.init(p.b, p.ldb, p.N, p.K, n0, grp, gt);
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int e = 0; e < 4 * NG; ++e) acc[i][j][e] = 0.f;

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
  // ---- epilogue.  32x32x16 block (i, j) of the wave: i = 2 h + i' -> tile
  // rows 128 h + 64 wr + 32 i', j -> tile cols 128 j + 32 wc; lane holds rows
  // (lane & 31), columns 8 g + 4 (lane >> 5) + e in acc[i][j][4 g + e].
  // 16x16x32 block (i, j): i = 4 h + i' -> rows 128 h + 64 wr + 16 i', j =
  // 2 g + j' -> cols 128 g + 32 wc + 16 j'; lane holds row (lane & 15),
  // columns 4 (lane >> 4) + e in acc[i][j][e].
  // Every finished 4-value group leaves for LDS (bf16) or memory (fp32) at
  // once.  The lane id is re-derived (opaque to the compiler) so no lane value
  // of the prologue stays live across the loop.
  int ln;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
  const int tid2 = wave * 64 + ln, hh = ln >> 5;
  auto row_of = [&](int i) __attribute__((always_inline)) {
    return M16 ? m0 + 128 * (i >> 2) + 64 * wr + 16 * (i & 3) + (ln & 15) : m0 + 128 * (i >> 1) + 64 * wr + 32 * (i & 1) + (ln & 31);
  };
  auto col_of = [&](int j, int g) __attribute__((always_inline)) {
    return M16 ? n0 + 128 * (j >> 1) + 32 * wc + 16 * (j & 1) + 4 * (ln >> 4) : n0 + 128 * j + 32 * wc + 8 * g + 4 * hh;
  };
  constexpr int LROW = 256 * 2 + 16;  // bf16 staging image [256][256] + 16 B row pad
  if (!SK && EPI == 1 && p.splits > 1) {
    if (!p.counters) {  // row-major fp32 slabs, summed by a separate launch (ops.gemm slab_sum)
      const int64_t mn = int64_t(p.M) * p.N;
      float* slabs = reinterpret_cast<float*>(p.c);
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int g = 0; g < NG; ++g) {
            const int m = row_of(i), n = col_of(j, g);
            if (m < p.M && n < p.N)
              *reinterpret_cast<f32x4*>(slabs + split * mn + int64_t(m) * p.N + n) =
                  f32x4{acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]};
          }
      return;
    }
    // In-launch reduction, gemm_core.h's protocol: every K-slice writes its
    // fp32 partial tile fragment-native (wave w, group q, lane l at float
    // ((w QN + q) 64 + l) 4 of the tile's 256 KB slab: 1 KB per wave store)
    // with sc1 (write-through) stores, drains them, takes one relaxed
    // agent-scope ticket; the last slice to arrive sums every slice's slab
    // (sc1 loads, its own included: its accumulators are dead by then, which
    // keeps the reduction out of the 128 accumulator registers) and runs the
    // epilogue on the sums.  The
    // hardware assumption this rests on is spelled out in gemm_core.h and pinned
    // by tests/test_gpu_gemm.py::test_in_launch_splitk_reused_workspace.
    constexpr int QN = NI * NJ * NG, TILEF = 256 * 256;
    const int tiles = tiles_m * tiles_n;
    const uint32_t lane_off = uint32_t(((wave * QN) * 64 + ln) * 16);
    auto tile_rsrc = [&](int s2) __attribute__((always_inline)) {
      return __builtin_amdgcn_make_buffer_rsrc(p.ws + (int64_t(s2) * tiles + t) * TILEF, 0, TILEF * 4, 0x00020000);
    };
    {
      const auto rs = tile_rsrc(split);
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int g = 0; g < NG; ++g) {
            const int q = (i * NJ + j) * NG + g;
            const f32x4 v = {acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]};
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rs, lane_off + q * 1024, 0, 16);
          }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = reinterpret_cast<int*>(smem);
    if (tid2 == 0) {
      const int old = __hip_atomic_fetch_add(p.counters + t, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      flag[0] = old == p.splits - 1;
      if (old == p.splits - 1) __hip_atomic_store(p.counters + t, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!flag[0]) return;
  }
  bool emit = true;
  if constexpr (SK) {
    if (partial) {
      // Stream-K fix-up of a tile cut between workgroups c0..c1 (consecutive
      // ids).  Partials are fragment-native 256 KB slabs (as the split-K
      // reduction above: sc1 stores / loads, one relaxed agent-scope ticket per
      // tile, the same hardware assumption), slab 2 w + (t is w's first tile ?
      // 0 : 1) of workgroup w.  The tile's head (k = 0) belongs to c0, which
      // runs it as the LAST segment of its range while c0 + 1..c1 ran their
      // parts of the tile first, so c0 usually finds every other partial
      // published: it then writes nothing and adds them to its registers.
      // Otherwise the last workgroup to arrive reduces.  Either way the sum is
      // formed in the order c0, c0 + 1, .., c1 (bitwise the same whoever
      // reduces): c0 adds the others to its own accumulators; any other
      // reducer publishes its own slab and re-reads them all from c0 on.
      constexpr int QN = NI * NJ * NG, TILEF = 256 * 256, GB = 16;
      const int c0 = sk_owner(t * KT, total, G), c1 = sk_owner(t * KT + KT - 1, total, G);
      const uint32_t lane_off = uint32_t(((wave * QN) * 64 + ln) * 16);
      auto slab_rs = [&](int w) __attribute__((always_inline)) {
        const int slot = sk_begin(w, total, G) / KT == t ? 0 : 1;
        return __builtin_amdgcn_make_buffer_rsrc(p.ws + int64_t(2 * w + slot) * TILEF, 0, TILEF * 4, 0x00020000);
      };
      // variant bits 18 / 19: timing probes (no partial stores / no fix-up loads);
      // bit 20: a tile whose workgroups all sit on one XCD is published with
      // plain stores (kept in that XCD's L2, which serves the sc1 loads)
      const int skm = (p.variant >> 18) & 7;
      const bool local_st = (skm & 4) && xcd_of(c0, G) == xcd_of(c1, G);
      auto publish = [&]() __attribute__((always_inline)) {
        if (skm & 1) return;
        const auto rs = slab_rs(bid);
        if (local_st) {
#pragma unroll
          for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j)
#pragma unroll
              for (int g = 0; g < NG; ++g) {
                const int q = (i * NJ + j) * NG + g;
                const f32x4 v = {acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]};
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rs, lane_off + q * 1024, 0, 0);
              }
        } else {
#pragma unroll
          for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j)
#pragma unroll
              for (int g = 0; g < NG; ++g) {
                const int q = (i * NJ + j) * NG + g;
                const f32x4 v = {acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]};
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rs, lane_off + q * 1024, 0, 16);
              }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      };
      int* flag = reinterpret_cast<int*>(smem);
      __syncthreads();  // every wave past the K loop's last LDS access
      if (tid2 == 0)
        flag[0] = __hip_atomic_load(p.counters + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == c1 - c0;
      __syncthreads();
      bool last = flag[0] != 0;
      bool published = false;
      if (!last) {
        publish();
        published = true;
        __syncthreads();
        if (tid2 == 0) flag[1] = __hip_atomic_fetch_add(p.counters + t, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == c1 - c0;
        __syncthreads();
        last = flag[1] != 0;
      }
      emit = last;
      if (last) {
        if (tid2 == 0) __hip_atomic_store(p.counters + t, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int cfirst = c0 + 1;
        if (bid != c0) {  // not the head owner: start the ordered sum from c0's slab
          if (!published) publish();
#pragma unroll
          for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j)
#pragma unroll
              for (int e = 0; e < 4 * NG; ++e) acc[i][j][e] = 0.f;
          cfirst = c0;
        }
        for (int w = cfirst; w <= (skm & 2 ? cfirst - 1 : c1); ++w) {
          const auto rs = slab_rs(w);
#pragma unroll
          for (int b0 = 0; b0 < QN; b0 += GB) {  // GB groups (64 registers) in flight per round trip
            f32x4 v[GB];
#pragma unroll
            for (int q = 0; q < GB; ++q)
              v[q] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, lane_off + (b0 + q) * 1024, 0, 16));
#pragma unroll
            for (int q = 0; q < GB; ++q) {
              const int qq = b0 + q, i = qq / (NJ * NG), j = (qq / NG) % NJ, g = qq % NG;
#pragma unroll
              for (int e = 0; e < 4; ++e) acc[i][j][4 * g + e] += v[q][e];
            }
          }
        }
      }
    }
  }
  if (emit) {
  __syncthreads();  // LDS free (main loop / flag) for the bf16 staging image
  // bias of 4 consecutive columns: one 16-byte (fp32) / 8-byte (bf16) load
  auto bias4 = [&](int n) __attribute__((always_inline)) {
    if (!p.bias) return f32x4{0.f, 0.f, 0.f, 0.f};
    if (p.bias_bf16) {
      const uint2 b2 = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(p.bias) + n);
      return f32x4{__uint_as_float(b2.x << 16), __uint_as_float(b2.x & 0xffff0000u), __uint_as_float(b2.y << 16),
                   __uint_as_float(b2.y & 0xffff0000u)};
    }
    return *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(p.bias) + n);
  };
  // the bias-only epilogue loads the lane's bias columns once, before the stores
  // (the full epilogue's GELU / residual registers leave no room: it loads per group)
  f32x4 bv[NJ][NG];
  if constexpr (EPI == 2) {
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int g = 0; g < NG; ++g) bv[j][g] = bias4(min(col_of(j, g), p.N - 4));
  }
  auto finish = [&](int i, int j, int g, float v0, float v1, float v2, float v3) __attribute__((always_inline)) {
    const int m = row_of(i), n = col_of(j, g);
    if (m >= p.M || n >= p.N) return;
    float v[4] = {v0, v1, v2, v3};
    const int64_t off = int64_t(m) * p.ldc + n;
    if constexpr (EPI != 0) {
      const f32x4 b = EPI == 2 ? bv[j][g] : bias4(n);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] += b[e];
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
  if (!SK && EPI == 1 && p.splits > 1) {
    // 8 groups of a slice in flight per load round, 4 batches
    constexpr int QN = NI * NJ * NG, TILEF = 256 * 256, GB = 8;
    const int tiles = tiles_m * tiles_n;
    const uint32_t lane_off = uint32_t(((wave * QN) * 64 + ln) * 16);
#pragma unroll
    for (int b0 = 0; b0 < QN; b0 += GB) {
      f32x4 sum[GB];
#pragma unroll
      for (int q = 0; q < GB; ++q) sum[q] = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int s2 = 0; s2 < p.splits; ++s2) {
        const auto rs = __builtin_amdgcn_make_buffer_rsrc(p.ws + (int64_t(s2) * tiles + t) * TILEF, 0, TILEF * 4, 0x00020000);
        f32x4 v[GB];
#pragma unroll
        for (int q = 0; q < GB; ++q)
          v[q] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, lane_off + (b0 + q) * 1024, 0, 16));
#pragma unroll
        for (int q = 0; q < GB; ++q) sum[q] += v[q];
      }
#pragma unroll
      for (int q = 0; q < GB; ++q) {
        const int qq = b0 + q;
        finish(qq / (NJ * NG), (qq / NG) % NJ, qq % NG, sum[q][0], sum[q][1], sum[q][2], sum[q][3]);
      }
    }
  } else {  // fully unrolled: acc is only ever indexed by constants (else it lands in scratch)
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int g = 0; g < NG; ++g)
          finish(i, j, g, acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]);
  }
  if (p.c_bf16 && !(probe & 4)) {
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
  }  // emit
  if constexpr (!SK) break;
  __syncthreads();  // the staging image / flags are the next segment's DMA target
  }  // segment loop
}

// ---- 256 x 128 output tile (variant bit 21 with bit 11) ---------------------------
// The N = 768 Linear products (ViT-B proj / fc2 / patch forward, qkv / fc1 input
// gradients, M = 6304 tokens) have 75 tiles of 256 x 256 for 256 CUs; cutting K
// to fill the chip (split-K / stream-K above) moves 256 KB fp32 partials per
// workgroup, ~15-18 us of chip-wide traffic per product (scripts/sk_anatomy.py).
// A 256 x 128 tile gives 150 whole tiles instead, each CU running the full K
// with no partials.  Same ping-pong scheme as gemm_pp_kernel, 8 waves as 2 x 4,
// each wave 128 x 32 (four 32 x 32 blocks): three operand pieces per K-tile
// (0 Alo, 1 Ahi, 2 B; 16 KB each, two buffers = 96 KB), two phases per K-tile
// -- ph1 (a-lo, b), ph2 (a-hi, b: the B fragments stay in registers) -- and,
// over a pair of K-tiles (j in buffer 0, j + 1 in buffer 1), the DMA schedule
//   ph1 Ahi(j+1)->b1   ph2 Alo,B(j+2)->b0   ph3 Ahi(j+2)->b0   ph4 Alo,B(j+3)->b1
// (a piece is restaged one phase after its last read), so every phase retires
// exactly the piece(s) the next phase reads with one s_waitcnt vmcnt(6).
template <class SA, class SB, bool KA, bool KB, int EPI, bool M16>
__global__ __launch_bounds__(512) void gemm_pp128_kernel(GemmParams p, int tiles_m, int tiles_n) {
  constexpr int LROW = 128 * 2 + 16;  // bf16 staging image [256][128] + 16 B row pad
  constexpr int SMEM = 6 * TILE > 256 * LROW ? 6 * TILE : 256 * LROW;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int grp = __builtin_amdgcn_readfirstlane(tid >> 8), gt = tid & 255;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int t = bid;
  int tm, tn;
  {  // grouped tile order (8 tile rows per column step)
    constexpr int GROUP_M = 8;
    const int per_group = GROUP_M * tiles_n, g0 = (t / per_group) * GROUP_M;
    const int gsize = min(tiles_m - g0, GROUP_M), r = t % per_group;
    tm = g0 + r % gsize;
    tn = r / gsize;
  }
  const int m0 = tm * 256, n0 = tn * 128;
  const int probe = (p.variant >> 12) & 15;  // bit 14: no C stores, 15: no K loop (timing only)
  const int nt = !(probe & 8) ? (p.K + BK - 1) / BK : 0;
  SA sa;
  SB sb;
  sa.init(p.a, p.lda, p.M, p.K, m0, grp, gt);
  sb.init(p.b, p.ldb, p.N, p.K, n0, grp, gt);

  // 32x32x16 form: 4 row blocks of 32 x 1 column block of 32 (f32x16 each), per phase
  // 2 A blocks x 4 k-substeps of 16; M16 (16x16x32, variant bit 16; the chip holds a
  // higher clock under it): 8 row blocks of 16 x 2 column blocks of 16 (f32x4 each),
  // per phase 4 A blocks x 2 B blocks x 2 k-substeps of 32 -- same registers
  constexpr int NI = M16 ? 8 : 4, NJ = M16 ? 2 : 1, NA = M16 ? 4 : 2, NB = M16 ? 2 : 1, NKS = M16 ? 2 : 4;
  constexpr int RBLK = M16 ? 16 : 32, TR_KS = M16 ? 8192 : 4096;
  using AccT = std::conditional_t<M16, f32x4, f32x16>;
  AccT acc[NI][NJ];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int e = 0; e < (M16 ? 4 : 16); ++e) acc[i][j][e] = 0.f;

  // LDS piece q (0 Alo, 1 Ahi, 2 B) of buffer b at (2 q + b) x 16 KB
  auto stage = [&](int q, int tile, int buf) __attribute__((always_inline)) {
    const int k0 = tile * BK;
    char* dst = smem + (2 * q + buf) * TILE;
    const i32x4 d = q < 2 ? sa.desc(k0) : sb.desc(k0);
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      char* l = dst + ((2 * grp + c) * 256 + (wave & 3) * 64) * 16;
      if (q < 2)
        sa.dma(d, q, c, l);
      else
        sb.dma(d, 0, c, l);
    }
  };
  const int lr = lane % RBLK, lc = lane / RBLK;
  auto kbase = [&](int row0, int ks) __attribute__((always_inline)) {
    const int c = M16 ? (4 * ks) | lc : (2 * ks) | lc;
    return uint32_t((row0 + lr) * 128 + ((c ^ ((lr >> 1) & 7)) << 4));
  };
  constexpr int NVA = KA ? NKS : 2 * NA, NVB = KB ? NKS : 2 * NB;
  uint32_t va[NVA], vb[NVB];
  if constexpr (KA) {
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) va[ks] = kbase(64 * wr, ks);
  } else {
#pragma unroll
    for (int u = 0; u < 2 * NA; ++u) va[u] = mn_base<M16>(64 * wr + RBLK * (u >> 1), u & 1, lane);
  }
  if constexpr (KB) {
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) vb[ks] = 4 * TILE + kbase(32 * wc, ks);
  } else {
#pragma unroll
    for (int u = 0; u < 2 * NB; ++u) vb[u] = 4 * TILE + mn_base<M16>(32 * wc + RBLK * (u >> 1), u & 1, lane);
  }
  auto frag_pp = [&](const uint32_t* v, bool kmaj, int cst, int i, int ks) __attribute__((always_inline)) {
    if (kmaj) return *reinterpret_cast<const uint4*>(smem + v[ks] + cst + i * RBLK * 128);
    uint4 out;
    const s16x4 x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4*)(smem + v[2 * i] + cst + ks * TR_KS));
    const s16x4 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4*)(smem + v[2 * i + 1] + cst + ks * TR_KS));
    const uint2 u0 = __builtin_bit_cast(uint2, x0), u1 = __builtin_bit_cast(uint2, x1);
    out.x = u0.x;
    out.y = u0.y;
    out.z = u1.x;
    out.w = u1.y;
    return out;
  };
  uint4 fa[NA][NKS], fb[NB][NKS];
  auto read_a = [&](int buf, int h) __attribute__((always_inline)) {
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
      for (int i = 0; i < NA; ++i) fa[i][ks] = frag_pp(va, KA, (2 * h + buf) * TILE, i, ks);
  };
  auto read_b = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
      for (int j = 0; j < NB; ++j) fb[j][ks] = frag_pp(vb, KB, buf * TILE, j, ks);
  };
  auto mma = [&](int h) __attribute__((always_inline)) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
      for (int i = 0; i < NA; ++i)
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          if constexpr (M16)
            acc[NA * h + i][j] = mfma16(fb[j][ks], fa[i][ks], acc[NA * h + i][j]);
          else
            acc[NA * h + i][0] = mfma(fb[0][ks], fa[i][ks], acc[NA * h + i][0]);
        }
    __builtin_amdgcn_s_setprio(0);
  };
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
  // a phase's wait: vmcnt(6) retires exactly the piece(s) the next phase reads when
  // this phase staged; at the tail (nothing staged) everything is drained
  auto vwait = [&](bool staged) __attribute__((always_inline)) {
    if (staged)
      vm6();
    else
      vm0();
  };

  if (nt > 0) {
    stage(0, 0, 0);
    stage(2, 0, 0);
    stage(1, 0, 0);
    if (nt > 1) {
      stage(0, 1, 1);
      stage(2, 1, 1);
    }
    vwait(nt > 1);
    bar();
    if (wr == 1) bar();  // stagger: waves 4-7 run one barrier behind
    for (int j = 0; j < nt; j += 2) {
      const bool n1 = j + 1 < nt, n2 = j + 2 < nt, n3 = j + 3 < nt;
      // ph1: (a-lo, b) of tile j; Ahi(j + 1) -> b1; retire Ahi(j)
      read_a(0, 0);
      read_b(0);
      if (n1) stage(1, j + 1, 1);
      vwait(n1);
      lgkm0();
      bar();
      mma(0);
      bar();
      // ph2: (a-hi, b held); Alo, B (j + 2) -> b0; retire Alo, B (j + 1)
      read_a(0, 1);
      if (n2) {
        stage(0, j + 2, 0);
        stage(2, j + 2, 0);
      }
      vwait(n2);
      lgkm0();
      bar();
      mma(1);
      bar();
      if (!n1) break;
      // ph3: (a-lo, b) of tile j + 1; Ahi(j + 2) -> b0; retire Ahi(j + 1)
      read_a(1, 0);
      read_b(1);
      if (n2) stage(1, j + 2, 0);
      vwait(n2);
      lgkm0();
      bar();
      mma(0);
      bar();
      // ph4: (a-hi, b held); Alo, B (j + 3) -> b1; retire Alo, B (j + 2)
      read_a(1, 1);
      if (n3) {
        stage(0, j + 3, 1);
        stage(2, j + 3, 1);
      }
      vwait(n3);
      lgkm0();
      bar();
      mma(1);
      bar();
    }
    if (wr == 0) bar();  // balance the stagger
  }
  // ---- epilogue.  32x32x16: block i -> tile rows 128 (i >> 1) + 64 wr + 32 (i & 1) +
  // (lane & 31), cols 32 wc + 8 g + 4 (lane >> 5) + e in acc[i][0][4 g + e].  16x16x32:
  // block (i, j) -> rows 128 (i >> 2) + 64 wr + 16 (i & 3) + (lane & 15), cols 32 wc +
  // 16 j + 4 (lane >> 4) + e in acc[i][j][e]
  int ln;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
  const int tid2 = wave * 64 + ln, hh = ln >> 5;
  auto row_of = [&](int i) __attribute__((always_inline)) {
    return M16 ? m0 + 128 * (i >> 2) + 64 * wr + 16 * (i & 3) + (ln & 15) : m0 + 128 * (i >> 1) + 64 * wr + 32 * (i & 1) + (ln & 31);
  };
  // column group q: (32x32x16) g = q of the lane's 4 groups, (16x16x32) j = q of its 2 blocks
  constexpr int NQ = M16 ? 2 : 4;
  auto col_of = [&](int q) __attribute__((always_inline)) {
    return M16 ? n0 + 32 * wc + 16 * q + 4 * (ln >> 4) : n0 + 32 * wc + 8 * q + 4 * hh;
  };
  auto accv = [&](int i, int q, int e) __attribute__((always_inline)) {
    return M16 ? acc[i][q][e] : acc[i][0][4 * q + e];
  };
  __syncthreads();  // LDS free for the bf16 staging image
  auto bias4 = [&](int n) __attribute__((always_inline)) {
    if (!p.bias) return f32x4{0.f, 0.f, 0.f, 0.f};
    if (p.bias_bf16) {
      const uint2 b2 = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(p.bias) + n);
      return f32x4{__uint_as_float(b2.x << 16), __uint_as_float(b2.x & 0xffff0000u), __uint_as_float(b2.y << 16),
                   __uint_as_float(b2.y & 0xffff0000u)};
    }
    return *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(p.bias) + n);
  };
  f32x4 bv[NQ];
  if constexpr (EPI != 0) {
#pragma unroll
    for (int g = 0; g < NQ; ++g) bv[g] = bias4(min(col_of(g), p.N - 4));
  }
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int g = 0; g < NQ; ++g) {
      const int m = row_of(i), n = col_of(g);
      if (m >= p.M || n >= p.N) continue;
      float v[4] = {accv(i, g, 0), accv(i, g, 1), accv(i, g, 2), accv(i, g, 3)};
      const int64_t off = int64_t(m) * p.ldc + n;
      if constexpr (EPI != 0) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += bv[g][e];
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
      if (!p.c_bf16)
        *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(p.c) + off) = f32x4{v[0], v[1], v[2], v[3]};
      else
        *reinterpret_cast<uint2*>(smem + (m - m0) * LROW + (n - n0) * 2) = uint2{pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3])};
    }
  if (!p.c_bf16 || (probe & 4)) return;
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 256 * 16 / 512; ++q) {  // 256 rows x 16 16-byte chunks
    const int chunk = q * 512 + tid2, r = chunk >> 4, c = chunk & 15;
    const int m = m0 + r, n = n0 + c * 8;
    if (m < p.M && n < p.N)
      *reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(p.c) + int64_t(m) * p.ldc + n) =
          *reinterpret_cast<const uint4*>(smem + r * LROW + c * 16);
  }
}

template <bool KA, bool KB, bool M16>
static void launch_pp128_m(const GemmParams& p, hipStream_t s) {
  const int tm = (p.M + 255) / 256, tn = (p.N + 127) / 128;
  switch (epilogue_kind(p)) {
    case 0:
      hipLaunchKernelGGL((gemm_pp128_kernel<PPSrc<KA>, PPSrc<KB>, KA, KB, 0, M16>), dim3(tm * tn), dim3(512), 0, s, p, tm, tn);
      break;
    case 2:
      hipLaunchKernelGGL((gemm_pp128_kernel<PPSrc<KA>, PPSrc<KB>, KA, KB, 2, M16>), dim3(tm * tn), dim3(512), 0, s, p, tm, tn);
      break;
    default:
      hipLaunchKernelGGL((gemm_pp128_kernel<PPSrc<KA>, PPSrc<KB>, KA, KB, 1, M16>), dim3(tm * tn), dim3(512), 0, s, p, tm, tn);
  }
}

template <bool KA, bool KB>
static void launch_pp128(const GemmParams& p, hipStream_t s) {
  if (p.variant & PP_M16)
    launch_pp128_m<KA, KB, true>(p, s);
  else
    launch_pp128_m<KA, KB, false>(p, s);
}

template <bool KA, bool KB, bool M16, bool SK>
static void launch_pp_m(const GemmParams& p, hipStream_t s) {
  const int tm = (p.M + 255) / 256, tn = (p.N + 255) / 256;
  // stream-K: `splits` is the grid size; its epilogue kind is that of the unsplit product
  const int grid = SK ? p.splits : tm * tn * (p.splits > 1 ? p.splits : 1);
  GemmParams q = p;
  if (SK) q.splits = 1;
  switch (epilogue_kind(q)) {
    case 0:
      hipLaunchKernelGGL((gemm_pp_kernel<PPSrc<KA>, PPSrc<KB>, KA, KB, 0, M16, SK>), dim3(grid), dim3(512), 0, s, p, tm, tn);
      break;
    case 2:
      hipLaunchKernelGGL((gemm_pp_kernel<PPSrc<KA>, PPSrc<KB>, KA, KB, 2, M16, SK>), dim3(grid), dim3(512), 0, s, p, tm, tn);
      break;
    default:
      hipLaunchKernelGGL((gemm_pp_kernel<PPSrc<KA>, PPSrc<KB>, KA, KB, 1, M16, SK>), dim3(grid), dim3(512), 0, s, p, tm, tn);
  }
}

constexpr int PP_N128 = 1 << 21;  // variant bit: the 256 x 128 tile (gemm_pp128_kernel)

template <bool KA, bool KB>
static void launch_pp(const GemmParams& p, hipStream_t s) {
  if (p.variant & PP_N128) {
    launch_pp128<KA, KB>(p, s);
    return;
  }
  const bool sk = p.variant & PP_SK;
  if (p.variant & PP_M16)
    sk ? launch_pp_m<KA, KB, true, true>(p, s) : launch_pp_m<KA, KB, true, false>(p, s);
  else
    sk ? launch_pp_m<KA, KB, false, true>(p, s) : launch_pp_m<KA, KB, false, false>(p, s);
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
