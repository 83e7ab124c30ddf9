// Fused multi-head self-attention for short sequences (ViT: 197 tokens, head
// dim 64) on MI355X (gfx950, wave64, v_mfma_f32_32x32x16_bf16).
//
// Operates directly on the QKV projection output [B, T, 3, H, 64] (bf16) and
// writes O as [B, T, H, 64] -- the layouts the surrounding GEMMs produce and
// consume -- so neither the head split/permute before attention nor the
// transpose after it is materialised.  The backward writes dQ/dK/dV straight
// into one [B, T, 3, H, 64] gradient, which is the QKV GEMM's input gradient.
//
// MFMA lane maps (32x32x16 bf16): lane l (r = l & 31, h = l >> 5) supplies
// A[row r][k = 8h + j] and B[k = 8h + j][col r] (j = 0..7); accumulator
// register i holds C[row (i&3) + 8(i>>2) + 4h][col r].  An accumulator X is
// reused as the next MFMA's operand without data movement when the next
// product sums over X's rows: registers 8s..8s+7 (packed to bf16) are the
// k-step-s fragment, whose element j is X row 16s + 8(j>>2) + 4h + (j&3); the
// other operand is then read from a TRANSPOSED LDS image ([d][token], rows of
// kSP elements) as two 8-byte reads at tokens 16s + 4h and 16s + 8 + 4h.
// kSP = 260 makes the 32 rows a half-wave reads land on 32 distinct bank pairs.
//
// forward (per wave: 32 queries; online softmax over 32-key tiles)
//   S^T = K Q^T          A = K rows (global), B = Q rows (registers)
//   O^T += V^T P^T       A = V^T (LDS image), B = P^T (the S^T accumulator)
//   keys live in registers and queries on lanes, so the row max / row sum is
//   a register reduction plus one lane^32 exchange.
// backward, two passes (no atomics: every output element has one owner)
//   dK/dV (per wave: 32 keys, loop over query tiles)
//     S  = Q K^T, dP = dO V^T        A = Q / dO rows (global), B = K / V rows (registers)
//     dV += P^T dO, dK += dS^T Q     A = P / dS (accumulators), B = dO^T / Q^T (LDS images)
//   dQ (per wave: 32 queries, loop over key tiles)
//     S^T = K Q^T, dP^T = V dO^T     A = K / V rows (global), B = Q / dO rows (registers)
//     dQ^T += K^T dS^T               A = K^T (LDS image), B = dS^T (accumulator)
//   with P = exp(S - lse) from the forward's log-sum-exp and
//   dS = P * (dP - rowsum(dO * O)).
#include "attention.h"
#include "common.h"
#include <stdlib.h>

namespace p2attn {
using namespace p2;

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

// The kernels are VALU-bound at these sizes (PMC: ~2.6 K VALU instructions per
// wave vs 49 MFMAs in the forward), so conversions use the hardware
// instructions: a plain float->__bf16 conversion lowers to v_cvt_pk_bf16_f32
// (round-to-nearest-even, 1 instruction per 2 values instead of the ~12 of the
// bit-level path in common.h), and exp2 is the raw v_exp_f32.
P2_DEVICE uint32_t cvt_pk(float a, float b) {
  const bf16x2_t v = {static_cast<__bf16>(a), static_cast<__bf16>(b)};
  return __builtin_bit_cast(uint32_t, v);
}
P2_DEVICE uint16_t cvt1(float a) { return __builtin_bit_cast(uint16_t, static_cast<__bf16>(a)); }
P2_DEVICE float ex2(float x) { return __builtin_amdgcn_exp2f(x); }

constexpr int kD = 64;
constexpr int kSP = 260;  // LDS image row length (elements): 520 B rows -> conflict-free 8-B reads
// W waves per block, a block per 32 W tokens of a (batch, head).  W = 8 covers
// ViT's 197 tokens in one block (2 x 12 x 32 = 384 blocks = 1.5 per CU, so half
// the CUs run two); W = 4 splits them (768 blocks = 3 per CU, the K/V or Q
// images staged twice).  Chosen per launch (attention_waves()).
constexpr float kLog2e = 1.4426950408889634f;

P2_DEVICE f32x16 mfma(uint4 a, uint4 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c,
                                                 0, 0, 0);
}
P2_DEVICE int acc_row(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }
P2_DEVICE f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}
P2_DEVICE uint4 ld16(const uint16_t* p) { return *reinterpret_cast<const uint4*>(p); }
P2_DEVICE uint4 ld16_if(bool ok, const uint16_t* p) { return ok ? ld16(p) : make_uint4(0u, 0u, 0u, 0u); }
// Main-loop operand rows are clamped into [0, T) instead of predicated (no
// exec-mask branch per load): a padded key's scores are masked to -inf / its
// P forced to 0, and a padded query's lse is +inf (P = 0) or its output is
// simply not stored, so the duplicated row never reaches a result.
P2_DEVICE int clampT(int row, int T) { return row < T ? row : T - 1; }
// k-step s fragment of an accumulator (registers 8s .. 8s+7) as a bf16 operand
P2_DEVICE uint4 pack_frag(const f32x16& x, int s) {
  return make_uint4(cvt_pk(x[8 * s + 0], x[8 * s + 1]), cvt_pk(x[8 * s + 2], x[8 * s + 3]),
                    cvt_pk(x[8 * s + 4], x[8 * s + 5]), cvt_pk(x[8 * s + 6], x[8 * s + 7]));
}
// the matching operand from a transposed LDS image: row `row`, tokens t0..t0+3 and t0+8..t0+11
P2_DEVICE uint4 lds_frag(const uint16_t* img, int row, int t0) {
  const uint2 lo = *reinterpret_cast<const uint2*>(img + row * kSP + t0);
  const uint2 hi = *reinterpret_cast<const uint2*>(img + row * kSP + t0 + 8);
  return make_uint4(lo.x, lo.y, hi.x, hi.y);
}

// Transposed LDS image img[d][t] = src[t][d] for t < T, zero for T <= t < Tp
// (Tp <= kMaxT, even).  A work item is a token pair x 8 head dims: two 16-B
// global loads, then 8 dword LDS writes of (src[t][d], src[t+1][d]) --
// consecutive lanes take consecutive token pairs, so the writes of a wave
// hit distinct banks.  All of a thread's loads are issued before any write.
template <int kThreads>
P2_DEVICE void stage_transposed(uint16_t* img, const uint16_t* src, int64_t rs, int T, int Tp) {
  constexpr int kItems = (kMaxT / 2) * 8 / kThreads;  // per thread, upper bound
  const int half = Tp >> 1;
  uint4 a[kItems], b[kItems];
#pragma unroll
  for (int u = 0; u < kItems; ++u) {
    const int i = threadIdx.x + u * kThreads;
    const int tp = i % half, c = (i / half) * 8, t = 2 * tp;
    const bool ok = i < half * 8;
    a[u] = ld16_if(ok && t < T, src + t * rs + c);
    b[u] = ld16_if(ok && t + 1 < T, src + (t + 1) * rs + c);
  }
#pragma unroll
  for (int u = 0; u < kItems; ++u) {
    const int i = threadIdx.x + u * kThreads;
    if (i < half * 8) {
      const int tp = i % half, c = (i / half) * 8;
      const uint32_t x[4] = {a[u].x, a[u].y, a[u].z, a[u].w}, y[4] = {b[u].x, b[u].y, b[u].z, b[u].w};
      uint32_t* row = reinterpret_cast<uint32_t*>(img + c * kSP) + tp;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        row[(2 * j) * (kSP / 2)] = (x[j] & 0xffffu) | (y[j] << 16);
        row[(2 * j + 1) * (kSP / 2)] = (x[j] >> 16) | (y[j] & 0xffff0000u);
      }
    }
  }
}

// Row-major LDS image img[t][0..63] = src[min(t, T - 1)][0..63] for t < Tp, rows
// kRS elements apart (144 B: the 16-B fragment reads of 16 lanes at rows t0..t0+15
// land on distinct bank quads).  The main loops read their row-operand fragments
// (K in the forward, Q / dO in dK/dV, K / V in dQ) from here instead of from
// global memory -- they used to prefetch one 32-token tile ahead from L2, so every
// tile waited out most of a load round trip (~10 tiles of ~0.4 us of compute each).
// Clamped rows reproduce the loops' clampT addressing, so results are bitwise equal.
constexpr int kRS = 72;
template <int kThreads>
P2_DEVICE void stage_rows(uint16_t* img, const uint16_t* src, int64_t rs, int T, int Tp) {
  constexpr int kItems = (kMaxT * 8 + kThreads - 1) / kThreads;
  uint4 v[kItems];
#pragma unroll
  for (int u = 0; u < kItems; ++u) {
    const int i = threadIdx.x + u * kThreads, t = i >> 3, c = (i & 7) * 8;
    v[u] = ld16_if(t < Tp, src + clampT(t, T) * rs + c);
  }
#pragma unroll
  for (int u = 0; u < kItems; ++u) {
    const int i = threadIdx.x + u * kThreads, t = i >> 3, c = (i & 7) * 8;
    if (t < Tp) *reinterpret_cast<uint4*>(img + t * kRS + c) = v[u];
  }
}
P2_DEVICE uint4 row_frag(const uint16_t* img, int t, int c) { return *reinterpret_cast<const uint4*>(img + t * kRS + c); }

// rowsum(dO * O) over the 64 head dims of token t
P2_DEVICE float dot64(const uint16_t* a, const uint16_t* b) {
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < kD; c += 8) {
    const uint4 x = ld16(a + c), y = ld16(b + c);
    const uint32_t xa[4] = {x.x, x.y, x.z, x.w}, ya[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      s = fmaf(__uint_as_float(xa[j] << 16), __uint_as_float(ya[j] << 16), s);
      s = fmaf(__uint_as_float(xa[j] & 0xffff0000u), __uint_as_float(ya[j] & 0xffff0000u), s);
    }
  }
  return s;
}

// ---------------------------------------------------------------------------
// forward.  Grid (T / 128, H, B), 4 waves: wave w owns queries [32 (4 x + w), +32).  lse2 = log2-domain log-sum-exp of the scaled scores.
// ---------------------------------------------------------------------------
template <int kWaves, bool kRows>
__global__ __launch_bounds__(64 * kWaves) void attn_fwd_kernel(const uint16_t* __restrict__ qkv, uint16_t* __restrict__ o,
                                                       float* __restrict__ lse2, AttnShape sh) {
  __shared__ __attribute__((aligned(16))) uint16_t vt[kD * kSP];
  __shared__ __attribute__((aligned(16))) uint16_t kr[kRows ? kMaxT * kRS : 8];  // K rows (kRows)
  const int b = blockIdx.z, hd = blockIdx.y, T = sh.T;
  const int64_t rs = sh.qkv_row;
  const uint16_t* Q = qkv + b * sh.qkv_batch + hd * kD;
  const uint16_t* K = Q + sh.C;
  const uint16_t* V = Q + 2 * sh.C;
  const int nkt = (T + 31) >> 5;
  stage_transposed<64 * kWaves>(vt, V, rs, T, nkt * 32);
  if constexpr (kRows) stage_rows<64 * kWaves>(kr, K, rs, T, nkt * 32);
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int q0 = (blockIdx.x * kWaves + wave) * 32;
  if (q0 >= T) return;  // no barrier below
  const bool qv = q0 + r < T;
  uint4 qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) qf[s] = ld16(Q + clampT(q0 + r, T) * rs + 16 * s + 8 * h);
  f32x16 o0 = zero16(), o1 = zero16();
  float m = -INFINITY, l = 0.f;
  const float sl2 = sh.scale * kLog2e;
  uint4 kn[4];
  if constexpr (!kRows) {
#pragma unroll
    for (int s = 0; s < 4; ++s) kn[s] = ld16(K + clampT(r, T) * rs + 16 * s + 8 * h);
  }
  for (int kt = 0; kt < nkt; ++kt) {
    uint4 kf[4];
    if constexpr (kRows) {
#pragma unroll
      for (int s = 0; s < 4; ++s) kf[s] = row_frag(kr, kt * 32 + r, 16 * s + 8 * h);
    } else {
#pragma unroll
      for (int s = 0; s < 4; ++s) kf[s] = kn[s];
      const int nkey = (kt + 1) * 32 + r;  // prefetch the next key tile
#pragma unroll
      for (int s = 0; s < 4; ++s) kn[s] = ld16(K + clampT(nkey, T) * rs + 16 * s + 8 * h);
    }
    f32x16 st = zero16();
#pragma unroll
    for (int s = 0; s < 4; ++s) st = mfma(kf[s], qf[s], st);
    // raw scores; the scale is folded into the exponent (scale > 0 keeps the max)
    float tmax = -INFINITY;
    if (kt * 32 + 32 <= T) {  // wave-uniform: only the last tile needs the key mask
#pragma unroll
      for (int i = 0; i < 16; ++i) tmax = fmaxf(tmax, st[i]);
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        if (kt * 32 + acc_row(i, h) >= T) st[i] = -INFINITY;
        tmax = fmaxf(tmax, st[i]);
      }
    }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    // Lazy rescale: the running max m only moves (and O, l are rescaled) when some
    // query's tile max exceeds it by more than 2^8 in the exponent -- in practice on
    // the first tile only.  Otherwise P = 2^(s - m) <= 256 against a stale m, which
    // leaves O / l and lse2 = m + log2 l exact (both are invariant to the reference
    // m) and saves the 32 rescale multiplies + one exp2 per lane and tile.
    if (__any(tmax * sl2 > m + 8.f)) {  // wave-uniform; always true on tile 0 (m = -inf)
      const float mn = fmaxf(m, tmax * sl2);  // finite: key tile 0 always holds key 0
      const float alpha = ex2(m - mn);
      l *= alpha;
      m = mn;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        o0[i] *= alpha;
        o1[i] *= alpha;
      }
    }
    float ps = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float p = ex2(fmaf(st[i], sl2, -m));
      st[i] = p;
      ps += p;
    }
    l += ps;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const uint4 pb = pack_frag(st, s);
      const int t0 = kt * 32 + 16 * s + 4 * h;
      o0 = mfma(lds_frag(vt, r, t0), pb, o0);
      o1 = mfma(lds_frag(vt, 32 + r, t0), pb, o1);
    }
  }
  l += __shfl_xor(l, 32, 64);
  if (!qv) return;
  const float inv = 1.f / l;
  uint16_t* orow = o + b * sh.o_batch + (q0 + r) * sh.o_row + hd * kD;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int d = 8 * g + 4 * h;
    *reinterpret_cast<uint2*>(orow + d) =
        make_uint2(cvt_pk(o0[4 * g] * inv, o0[4 * g + 1] * inv), cvt_pk(o0[4 * g + 2] * inv, o0[4 * g + 3] * inv));
    *reinterpret_cast<uint2*>(orow + 32 + d) =
        make_uint2(cvt_pk(o1[4 * g] * inv, o1[4 * g + 1] * inv), cvt_pk(o1[4 * g + 2] * inv, o1[4 * g + 3] * inv));
  }
  if (h == 0) lse2[(int64_t(b) * sh.H + hd) * T + q0 + r] = m + __log2f(l);
}

// ---------------------------------------------------------------------------
// backward pass 1: dK, dV.  Grid (T / 128, H, B), wave w owns keys [32 (4 x + w), +32)
// and loops over all query tiles (next tile's Q / dO rows prefetched).
// ---------------------------------------------------------------------------
template <int kWaves, bool kRows>
__global__ __launch_bounds__(64 * kWaves) void attn_bwd_dkdv_kernel(const uint16_t* __restrict__ qkv,
                                                            const uint16_t* __restrict__ o,
                                                            const uint16_t* __restrict__ dout,
                                                            const float* __restrict__ lse2,
                                                            uint16_t* __restrict__ dqkv, AttnShape sh) {
  __shared__ __attribute__((aligned(16))) uint16_t qtl[kD * kSP];   // Q^T
  __shared__ __attribute__((aligned(16))) uint16_t dotl[kD * kSP];  // dO^T
  __shared__ float s_lse[kMaxT], s_dvec[kMaxT];
  __shared__ __attribute__((aligned(16))) uint16_t qr[kRows ? kMaxT * kRS : 8];   // Q rows (kRows)
  __shared__ __attribute__((aligned(16))) uint16_t dr[kRows ? kMaxT * kRS : 8];   // dO rows (kRows)
  const int b = blockIdx.z, hd = blockIdx.y, T = sh.T;
  const int64_t rs = sh.qkv_row;
  const uint16_t* Q = qkv + b * sh.qkv_batch + hd * kD;
  const uint16_t* K = Q + sh.C;
  const uint16_t* V = Q + 2 * sh.C;
  const uint16_t* O = o + b * sh.o_batch + hd * kD;
  const uint16_t* DO = dout + b * sh.o_batch + hd * kD;
  const float* L = lse2 + (int64_t(b) * sh.H + hd) * T;
  const int nqt = (T + 31) >> 5, Tp = nqt * 32;
  stage_transposed<64 * kWaves>(qtl, Q, rs, T, Tp);
  stage_transposed<64 * kWaves>(dotl, DO, sh.o_row, T, Tp);
  if constexpr (kRows) {
    stage_rows<64 * kWaves>(qr, Q, rs, T, Tp);
    stage_rows<64 * kWaves>(dr, DO, sh.o_row, T, Tp);
  }
  for (int t = threadIdx.x; t < Tp; t += blockDim.x) {
    const bool ok = t < T;
    s_lse[t] = ok ? L[t] : INFINITY;  // padded queries: P = exp2(-inf) = 0
    s_dvec[t] = ok ? dot64(DO + t * sh.o_row, O + t * sh.o_row) : 0.f;
  }
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int k0 = (blockIdx.x * kWaves + wave) * 32;
  if (k0 >= T) return;
  const bool kv = k0 + r < T;
  uint4 kf[4], vf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    kf[s] = ld16(K + clampT(k0 + r, T) * rs + 16 * s + 8 * h);
    vf[s] = ld16(V + clampT(k0 + r, T) * rs + 16 * s + 8 * h);
  }
  f32x16 dv0 = zero16(), dv1 = zero16(), dk0 = zero16(), dk1 = zero16();
  const float sl2 = sh.scale * kLog2e;
  uint4 qn[4], dn[4];
  if constexpr (!kRows) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      qn[s] = ld16(Q + clampT(r, T) * rs + 16 * s + 8 * h);
      dn[s] = ld16(DO + clampT(r, T) * sh.o_row + 16 * s + 8 * h);
    }
  }
  for (int qt = 0; qt < nqt; ++qt) {
    uint4 qa[4], da[4];
    if constexpr (kRows) {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        qa[s] = row_frag(qr, qt * 32 + r, 16 * s + 8 * h);
        da[s] = row_frag(dr, qt * 32 + r, 16 * s + 8 * h);
      }
    } else {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        qa[s] = qn[s];
        da[s] = dn[s];
      }
      const int nq = (qt + 1) * 32 + r;  // prefetch the next query tile
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        qn[s] = ld16(Q + clampT(nq, T) * rs + 16 * s + 8 * h);
        dn[s] = ld16(DO + clampT(nq, T) * sh.o_row + 16 * s + 8 * h);
      }
    }
    f32x16 sacc = zero16(), dp = zero16();
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      sacc = mfma(qa[s], kf[s], sacc);
      dp = mfma(da[s], vf[s], dp);
    }
    // rows = queries qt*32 + acc_row(i, h), column = key k0 + r
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int row = qt * 32 + acc_row(i, h);
      const float p = kv ? ex2(fmaf(sacc[i], sl2, -s_lse[row])) : 0.f;
      sacc[i] = p;
      dp[i] = p * (dp[i] - s_dvec[row]);
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const uint4 pa = pack_frag(sacc, s), da = pack_frag(dp, s);
      const int t0 = qt * 32 + 16 * s + 4 * h;
      dv0 = mfma(pa, lds_frag(dotl, r, t0), dv0);
      dv1 = mfma(pa, lds_frag(dotl, 32 + r, t0), dv1);
      dk0 = mfma(da, lds_frag(qtl, r, t0), dk0);
      dk1 = mfma(da, lds_frag(qtl, 32 + r, t0), dk1);
    }
  }
  // rows = keys k0 + acc_row(i, h), column = head dim r (tile 0) / 32 + r (tile 1)
  uint16_t* dK = dqkv + b * sh.qkv_batch + hd * kD + sh.C;
  uint16_t* dV = dK + sh.C;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int key = k0 + acc_row(i, h);
    if (key < T) {
      dK[key * rs + r] = cvt1(dk0[i] * sh.scale);
      dK[key * rs + 32 + r] = cvt1(dk1[i] * sh.scale);
      dV[key * rs + r] = cvt1(dv0[i]);
      dV[key * rs + 32 + r] = cvt1(dv1[i]);
    }
  }
}

// ---------------------------------------------------------------------------
// backward pass 2: dQ.  Grid (T / 128, H, B), wave w owns queries [32 (4 x + w), +32)
// and loops over all key tiles (next tile's K / V rows prefetched).
// ---------------------------------------------------------------------------
template <int kWaves, bool kRows>
__global__ __launch_bounds__(64 * kWaves) void attn_bwd_dq_kernel(const uint16_t* __restrict__ qkv,
                                                          const uint16_t* __restrict__ o,
                                                          const uint16_t* __restrict__ dout,
                                                          const float* __restrict__ lse2, uint16_t* __restrict__ dqkv,
                                                          AttnShape sh) {
  __shared__ __attribute__((aligned(16))) uint16_t ktl[kD * kSP];  // K^T
  __shared__ __attribute__((aligned(16))) uint16_t kr[kRows ? kMaxT * kRS : 8];  // K rows (kRows)
  __shared__ __attribute__((aligned(16))) uint16_t vr[kRows ? kMaxT * kRS : 8];  // V rows (kRows)
  const int b = blockIdx.z, hd = blockIdx.y, T = sh.T;
  const int64_t rs = sh.qkv_row;
  const uint16_t* Q = qkv + b * sh.qkv_batch + hd * kD;
  const uint16_t* K = Q + sh.C;
  const uint16_t* V = Q + 2 * sh.C;
  const uint16_t* O = o + b * sh.o_batch + hd * kD;
  const uint16_t* DO = dout + b * sh.o_batch + hd * kD;
  const int nkt = (T + 31) >> 5;
  stage_transposed<64 * kWaves>(ktl, K, rs, T, nkt * 32);
  if constexpr (kRows) {
    stage_rows<64 * kWaves>(kr, K, rs, T, nkt * 32);
    stage_rows<64 * kWaves>(vr, V, rs, T, nkt * 32);
  }
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int q0 = (blockIdx.x * kWaves + wave) * 32;
  if (q0 >= T) return;
  const int qq = q0 + r;
  const bool qv = qq < T;
  uint4 qf[4], df[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    qf[s] = ld16(Q + clampT(qq, T) * rs + 16 * s + 8 * h);
    df[s] = ld16(DO + clampT(qq, T) * sh.o_row + 16 * s + 8 * h);
  }
  const float lq = qv ? lse2[(int64_t(b) * sh.H + hd) * T + qq] : INFINITY;
  float dvec = 0.f;
  if (qv) {  // each lane half sums 32 of the 64 head dims
    const uint16_t* a = DO + qq * sh.o_row + 32 * h;
    const uint16_t* c = O + qq * sh.o_row + 32 * h;
#pragma unroll
    for (int u = 0; u < 32; u += 8) {
      const uint4 x = ld16(a + u), y = ld16(c + u);
      const uint32_t xa[4] = {x.x, x.y, x.z, x.w}, ya[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        dvec = fmaf(__uint_as_float(xa[j] << 16), __uint_as_float(ya[j] << 16), dvec);
        dvec = fmaf(__uint_as_float(xa[j] & 0xffff0000u), __uint_as_float(ya[j] & 0xffff0000u), dvec);
      }
    }
  }
  dvec += __shfl_xor(dvec, 32, 64);
  f32x16 dq0 = zero16(), dq1 = zero16();
  const float sl2 = sh.scale * kLog2e;
  uint4 kn[4], vn[4];
  if constexpr (!kRows) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      kn[s] = ld16(K + clampT(r, T) * rs + 16 * s + 8 * h);
      vn[s] = ld16(V + clampT(r, T) * rs + 16 * s + 8 * h);
    }
  }
  for (int kt = 0; kt < nkt; ++kt) {
    uint4 ka[4], va[4];
    if constexpr (kRows) {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        ka[s] = row_frag(kr, kt * 32 + r, 16 * s + 8 * h);
        va[s] = row_frag(vr, kt * 32 + r, 16 * s + 8 * h);
      }
    } else {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        ka[s] = kn[s];
        va[s] = vn[s];
      }
      const int nk = (kt + 1) * 32 + r;  // prefetch the next key tile
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        kn[s] = ld16(K + clampT(nk, T) * rs + 16 * s + 8 * h);
        vn[s] = ld16(V + clampT(nk, T) * rs + 16 * s + 8 * h);
      }
    }
    f32x16 st = zero16(), dpt = zero16();
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      st = mfma(ka[s], qf[s], st);
      dpt = mfma(va[s], df[s], dpt);
    }
    // rows = keys kt*32 + acc_row(i, h), column = query qq
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float p = (kt * 32 + acc_row(i, h) < T) ? ex2(fmaf(st[i], sl2, -lq)) : 0.f;
      st[i] = p * (dpt[i] - dvec);
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const uint4 db = pack_frag(st, s);
      const int t0 = kt * 32 + 16 * s + 4 * h;
      dq0 = mfma(lds_frag(ktl, r, t0), db, dq0);
      dq1 = mfma(lds_frag(ktl, 32 + r, t0), db, dq1);
    }
  }
  if (!qv) return;
  uint16_t* drow = dqkv + b * sh.qkv_batch + qq * rs + hd * kD;
  const float sc = sh.scale;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int d = 8 * g + 4 * h;
    *reinterpret_cast<uint2*>(drow + d) = make_uint2(cvt_pk(dq0[4 * g] * sc, dq0[4 * g + 1] * sc),
                                                     cvt_pk(dq0[4 * g + 2] * sc, dq0[4 * g + 3] * sc));
    *reinterpret_cast<uint2*>(drow + 32 + d) = make_uint2(cvt_pk(dq1[4 * g] * sc, dq1[4 * g + 1] * sc),
                                                          cvt_pk(dq1[4 * g + 2] * sc, dq1[4 * g + 3] * sc));
  }
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
template <int W>
static dim3 grid_of(const AttnShape& sh) { return dim3((sh.T + 32 * W - 1) / (32 * W), sh.H, sh.B); }

// 8-wave blocks unless P2PFL_ATTN_WAVES=4 (A/B switch, read once; measured at
// the ViT shape: fwd 21.8 vs 23.7 us, fwd+bwd 118 vs 121 us -- the kernels are
// VALU-bound, the 1.5-blocks-per-CU imbalance costs less than staging twice)
static int attention_waves() {
  static const int w = [] {
    const char* e = getenv("P2PFL_ATTN_WAVES");
    return (e && atoi(e) == 4) ? 4 : 8;
  }();
  return w;
}
// row operands staged in LDS (default) or streamed from L2 one tile ahead
// (P2PFL_ATTN_LDS_ROWS=0, the round-5 kernels)
static bool attention_rows() {
  static const bool on = [] {
    const char* e = getenv("P2PFL_ATTN_LDS_ROWS");
    return !(e && e[0] == '0');
  }();
  return on;
}

template <int W, bool R>
static void fwd_w(const uint16_t* qkv, uint16_t* o, float* lse2, const AttnShape& sh, hipStream_t s) {
  hipLaunchKernelGGL((attn_fwd_kernel<W, R>), grid_of<W>(sh), dim3(64 * W), 0, s, qkv, o, lse2, sh);
}
template <int W, bool R>
static void bwd_w(const uint16_t* qkv, const uint16_t* o, const uint16_t* dout, const float* lse2, uint16_t* dqkv,
                  const AttnShape& sh, hipStream_t s) {
  hipLaunchKernelGGL((attn_bwd_dkdv_kernel<W, R>), grid_of<W>(sh), dim3(64 * W), 0, s, qkv, o, dout, lse2, dqkv, sh);
  hipLaunchKernelGGL((attn_bwd_dq_kernel<W, R>), grid_of<W>(sh), dim3(64 * W), 0, s, qkv, o, dout, lse2, dqkv, sh);
}

void attention_fwd(const uint16_t* qkv, uint16_t* o, float* lse2, const AttnShape& sh, hipStream_t s) {
  const bool r = attention_rows();
  if (attention_waves() == 8)
    r ? fwd_w<8, true>(qkv, o, lse2, sh, s) : fwd_w<8, false>(qkv, o, lse2, sh, s);
  else
    r ? fwd_w<4, true>(qkv, o, lse2, sh, s) : fwd_w<4, false>(qkv, o, lse2, sh, s);
}

void attention_bwd(const uint16_t* qkv, const uint16_t* o, const uint16_t* dout, const float* lse2, uint16_t* dqkv,
                   const AttnShape& sh, hipStream_t s) {
  const bool r = attention_rows();
  if (attention_waves() == 8)
    r ? bwd_w<8, true>(qkv, o, dout, lse2, dqkv, sh, s) : bwd_w<8, false>(qkv, o, dout, lse2, dqkv, sh, s);
  else
    r ? bwd_w<4, true>(qkv, o, dout, lse2, dqkv, sh, s) : bwd_w<4, false>(qkv, o, dout, lse2, dqkv, sh, s);
}

}  // namespace p2attn
