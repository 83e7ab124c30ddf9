// Implicit-GEMM convolutions for the ResNet family (gfx950), NHWC bf16.
//
// All three products of a convolution run on the MFMA GEMM core of
// gemm_core.h; only the operand LOADERS differ, so no im2col matrix is ever
// materialised and no tensor is transposed in memory:
//
//   forward   Y[m = (n, oh, ow)][o]        = sum_{k = (ky, kx, c)} X~(m, k) W[o][k]
//   dgrad    dX[m = (n, ih, iw)][c]        = sum_{k = (ky, kx, o)} dY~(m, k) W[o][ky][kx][c]
//   wgrad    dW[o][(ky, kx, c)]            = sum_{k = (n, oh, ow)} dY[k][o] X~(k, (ky, kx, c))
//
// X~ / dY~ are gathers: every 16-byte chunk of an operand tile is 8
// consecutive channels of one pixel, located by the loader; padding taps,
// stride holes and tails resolve to the shared zero page.  Per K-tile the
// forward/dgrad gathers need a single (ky, kx) (C resp. O % 64 == 0), so the
// tap decode is a wave-uniform scalar computation and a lane only adds its
// precomputed pixel offset.  The weight gradient decodes output pixels per
// chunk with multiply-high division.
//
// Layouts match the learner's channels-last weight shadows (arena.py):
// weights are (O, kh, kw, C), so dW is written straight into the gradient
// layout the multi-tensor optimizer consumes.
//
// The reference trains convolutions through torch.nn.Conv2d
// (/root/reference/p2pfl/learning/pytorch/mnist_examples/models/cnn.py:55-62);
// the ResNet targets are BASELINE.json configs 3 and 5.
#include "conv.h"
#include <cstdlib>

#include "gemm_core.h"

namespace p2gemm {

struct FastDiv {  // n / d for 0 <= n < 2^31 as (umulhi(n, mul) + n) >> shift
  uint32_t d, mul, shift;
};
inline FastDiv make_fastdiv(uint32_t d) {
  uint32_t l = 0;
  while ((uint64_t(1) << l) < d) ++l;
  const uint64_t mul = ((uint64_t(1) << 32) * ((uint64_t(1) << l) - d)) / d + 1;
  return FastDiv{d, uint32_t(mul), l};
}
P2_DEVICE int fdiv(int n, const FastDiv& f) { return int((__umulhi(uint32_t(n), f.mul) + uint32_t(n)) >> f.shift); }

constexpr int kOff = -(1 << 28);  // pixel coordinate that fails every bounds check

// ---- forward: A = im2col(X), k-major, k = (ky, kx, c) ------------------------------
struct ConvFwdA {
  static constexpr bool KMAJ = true;
  const uint16_t* x;
  FastDiv ohw, ow, cdiv, kwdiv;  // cdiv / kwdiv: the per-K-tile tap decode by multiply-high
  int M, H, W, C, stride, pad, dil, kw;
  struct St {
    int64_t base[4];  // element offset of X[n][ih0][iw0][kk]
    int ih0[4], iw0[4];
    int kk;
  };
  P2_DEVICE St prep(int r0, int tid) const {
    St st;
    st.kk = kmaj_k(tid);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = r0 + kmaj_row(i, tid);
      const int n = fdiv(m, ohw), r = m - n * int(ohw.d);
      const int oh = fdiv(r, ow), owi = r - oh * int(ow.d);
      st.ih0[i] = m < M ? oh * stride - pad : kOff;
      st.iw0[i] = owi * stride - pad;
      st.base[i] = ((int64_t(n) * H + st.ih0[i]) * W + st.iw0[i]) * C + st.kk;
    }
    return st;
  }
  P2_DEVICE const void* src(const St& st, int i, int k0, int) const {
    // wave-uniform tap decode: scalar multiply-high, not two ~40-instruction
    // scalar divisions per chunk (they were most of the K loop's scalar work)
    const int tap = fdiv(k0, cdiv), cb = k0 - tap * C;
    const int ky = fdiv(tap, kwdiv), kx = tap - ky * kw;
    const int ih = st.ih0[i] + ky * dil, iw = st.iw0[i] + kx * dil;
    const bool ok = unsigned(ih) < unsigned(H) && unsigned(iw) < unsigned(W);
    return ok ? static_cast<const void*>(x + st.base[i] + (int64_t(ky * dil) * W + kx * dil) * C + cb)
              : zero_chunk();
  }
};

// ---- dgrad: A = transposed-conv gather of dY, k-major, k = (ky, kx, o) -------------
struct ConvDgradA {
  static constexpr bool KMAJ = true;
  const uint16_t* dy;
  FastDiv hw, w, odiv, kwdiv;
  int M, OH, OW, O, stride, pad, dil, kw;
  struct St {
    int64_t nbase[4];  // element offset of dY[n][0][0][kk]
    int thp[4], twp[4];  // ih + pad, iw + pad
    int kk;
  };
  P2_DEVICE St prep(int r0, int tid) const {
    St st;
    st.kk = kmaj_k(tid);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = r0 + kmaj_row(i, tid);
      const int n = fdiv(m, hw), r = m - n * int(hw.d);
      const int ih = fdiv(r, w), iw = r - ih * int(w.d);
      st.thp[i] = m < M ? ih + pad : kOff;
      st.twp[i] = iw + pad;
      st.nbase[i] = int64_t(n) * OH * OW * O + st.kk;
    }
    return st;
  }
  P2_DEVICE const void* src(const St& st, int i, int k0, int) const {
    const int tap = fdiv(k0, odiv), ob = k0 - tap * O;  // wave-uniform, multiply-high
    const int ky = fdiv(tap, kwdiv), kx = tap - ky * kw;
    int oh = st.thp[i] - ky * dil, ow = st.twp[i] - kx * dil;
    bool ok = oh >= 0 && ow >= 0;
    if (stride == 2) {
      ok = ok && !((oh | ow) & 1);
      oh >>= 1;
      ow >>= 1;
    }
    ok = ok && oh < OH && ow < OW;
    return ok ? static_cast<const void*>(dy + st.nbase[i] + (int64_t(oh) * OW + ow) * O + ob)
              : zero_chunk();
  }
};

// ---- dgrad: B = W[o][ky][kx][c] read c-contiguous, mn-major, k = (ky, kx, o) -------
struct ConvDgradB {
  static constexpr bool KMAJ = false;
  const uint16_t* w;
  FastDiv odiv;
  int C, O, T;  // T = kh * kw
  struct St {
    const uint16_t* col;
    int kr;
  };
  P2_DEVICE St prep(int r0, int tid) const {
    const int c = r0 + mnmaj_col(tid);
    return St{c < C ? w + c : nullptr, tid >> 4};
  }
  P2_DEVICE const void* src(const St& st, int i, int k0, int) const {
    const int tap = fdiv(k0, odiv), ob = k0 - tap * O;  // wave-uniform
    const int o = ob + 16 * i + st.kr;
    return st.col ? static_cast<const void*>(st.col + (int64_t(o) * T + tap) * C) : zero_chunk();
  }
};

// ---- dgrad, stride 2: one output phase per tile ------------------------------
// A stride-2 input gradient receives, at pixel (ih, iw), only the taps with
// ky = (ih + pad) mod 2 (mod 2) and kx likewise: for a 3x3 kernel 4, 2, 2 or 1
// of the 9 taps, 2.25 on average.  The plain gather above runs all 9 for every
// pixel (the holes read the zero page), 4x the MFMA work and K-tiles needed.
// Here the rows of the product are the dX pixels grouped by phase q = (a, b),
// a = (ih + pad) & 1, b = (iw + pad) & 1 -- row m of phase q (Mq rows each,
// a multiple of 128, so a tile never straddles two phases) is pixel
// (n, 2 ih2 + ((a - pad) & 1), 2 iw2 + ((b - pad) & 1)) -- and k = (tap of the
// phase, o) runs over ceil(kh/2) x ceil(kw/2) taps (fewer for odd phases: the
// surplus reads the zero page; the slowest phase sets the launch's time
// anyway).  The result is phase-major; phase_interleave_kernel puts it into
// dX.  H and W are even (the host falls back to ConvDgradA otherwise).
P2_DEVICE void s2_tap(int t, int a, int b, int kh, int kw, int& ky, int& kx, bool& valid) {
  const int nkx = (kw - b + 1) >> 1, nky = (kh - a + 1) >> 1;  // taps of this phase per axis
  if (nkx == 0) {  // kw == 1, odd column phase: no taps (never launched, see conv_dgrad_s2)
    ky = kx = 0;
    valid = false;
    return;
  }
  const int ty = nkx == 1 ? t : (nkx == 2 ? (t >> 1) : t / nkx);
  const int tx = t - ty * nkx;
  ky = a + 2 * ty;
  kx = b + 2 * tx;
  valid = ty < nky;
}

struct ConvDgradS2A {
  static constexpr bool KMAJ = true;
  const uint16_t* dy;
  FastDiv hw2, w2, odiv;
  int Mq, W2, OH, OW, O, pad, kh, kw;
  struct St {
    int64_t nbase[4];    // element offset of dY[n][0][0][kk]
    int thp[4], twp[4];  // ih + pad, iw + pad
    int kk, a, b;
  };
  P2_DEVICE St prep(int r0, int tid) const {
    St st;
    st.kk = kmaj_k(tid);
    const int q = min(r0 / Mq, 3);  // tile-uniform (Mq % 128 == 0)
    st.a = q >> 1;
    st.b = q & 1;
    const int ihoff = (st.a - pad) & 1, iwoff = (st.b - pad) & 1;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = r0 + kmaj_row(i, tid), loc = m - q * Mq;
      const int n = fdiv(loc, hw2), r = loc - n * int(hw2.d);
      const int ih2 = fdiv(r, w2), iw2 = r - ih2 * W2;
      st.thp[i] = m < 4 * Mq ? 2 * ih2 + ihoff + pad : kOff;
      st.twp[i] = 2 * iw2 + iwoff + pad;
      st.nbase[i] = int64_t(n) * OH * OW * O + st.kk;
    }
    return st;
  }
  P2_DEVICE const void* src(const St& st, int i, int k0, int) const {
    const int t = fdiv(k0, odiv), ob = k0 - t * O;  // wave-uniform
    int ky, kx;
    bool ok;
    s2_tap(t, st.a, st.b, kh, kw, ky, kx, ok);
    const int dh = st.thp[i] - ky, dw = st.twp[i] - kx;  // even by construction
    ok = ok && dh >= 0 && dw >= 0 && (dh >> 1) < OH && (dw >> 1) < OW;
    return ok ? static_cast<const void*>(dy + st.nbase[i] + (int64_t(dh >> 1) * OW + (dw >> 1)) * O + ob)
              : zero_chunk();
  }
};

// B = W[o][ky][kx][c] at the taps of the tile's phase (bound by tile_bound)
struct ConvDgradS2B {
  static constexpr bool KMAJ = false;
  const uint16_t* w;
  FastDiv odiv;
  int C, O, Mq, kh, kw, a, b;
  struct St {
    const uint16_t* col;
    int kr;
  };
  P2_DEVICE St prep(int r0, int tid) const {
    const int c = r0 + mnmaj_col(tid);
    return St{c < C ? w + c : nullptr, tid >> 4};
  }
  P2_DEVICE const void* src(const St& st, int i, int k0, int) const {
    const int t = fdiv(k0, odiv), ob = k0 - t * O;  // wave-uniform
    int ky, kx;
    bool ok;
    s2_tap(t, a, b, kh, kw, ky, kx, ok);
    const int o = ob + 16 * i + st.kr;
    return (ok && st.col) ? static_cast<const void*>(st.col + (int64_t(o) * kh * kw + ky * kw + kx) * C) : zero_chunk();
  }
};
P2_DEVICE ConvDgradS2B tile_bound(const ConvDgradS2B& l, int m0) {
  ConvDgradS2B t = l;
  const int q = min(m0 / l.Mq, 3);
  t.a = q >> 1;
  t.b = q & 1;
  return t;
}

// dX[n][ih][iw][:] <- phase-major row of (ih, iw): one thread per 16-byte chunk.
// Phases q >= nq were not computed (no taps: a 1x1 kernel) and are zero.
__global__ __launch_bounds__(256) void phase_interleave_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                               int64_t nchunks, int cpr, FastDiv cprd, FastDiv hw2,
                                                               FastDiv w2, int Mq, int nq, int H, int W, int pad) {
  const int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (i >= nchunks) return;
  const int m = fdiv(int(i), cprd), c = int(i) - m * cpr;  // phase-major row, chunk within the row
  const int q = m / Mq, loc = m - q * Mq;
  const int n = fdiv(loc, hw2), r = loc - n * int(hw2.d), ih2 = fdiv(r, w2), iw2 = r - ih2 * int(w2.d);
  const int ih = 2 * ih2 + (((q >> 1) - pad) & 1), iw = 2 * iw2 + (((q & 1) - pad) & 1);
  dst[((int64_t(n) * H + ih) * W + iw) * cpr + c] = q < nq ? src[i] : make_uint4(0, 0, 0, 0);
}

// ---- wgrad: B = im2col(X) read c-contiguous, mn-major, cols = (ky, kx, c), k = pixel
struct ConvWgradB {
  static constexpr bool KMAJ = false;
  const uint16_t* x;
  FastDiv ohw, ow, c_div;
  int M, H, W, C, stride, pad, dil, kw, ncols;
  struct St {
    int kyd, kxd, c, kr;
  };
  P2_DEVICE St prep(int r0, int tid) const {
    const int col = r0 + mnmaj_col(tid);
    const int tap = fdiv(col, c_div), c = col - tap * C;
    const int ky = tap / kw, kx = tap - ky * kw;
    return St{col < ncols ? ky * dil - pad : kOff, kx * dil - pad, c, tid >> 4};
  }
  P2_DEVICE const void* src(const St& st, int i, int k0, int) const {
    const int m = k0 + 16 * i + st.kr;
    const int n = fdiv(m, ohw), r = m - n * int(ohw.d);
    const int oh = fdiv(r, ow), owi = r - oh * int(ow.d);
    const int ih = oh * stride + st.kyd, iw = owi * stride + st.kxd;
    const bool ok = m < M && unsigned(ih) < unsigned(H) && unsigned(iw) < unsigned(W);
    return ok ? static_cast<const void*>(x + ((int64_t(n) * H + ih) * W + iw) * C + st.c)
              : zero_chunk();
  }
};

// EPI (gemm_core.h epilogue_kind): 0 = plain bf16 / fp32 store -- the common
// convolution launch, whose compact epilogue avoids fetching the ~60 KB of
// unrolled split-K / bias / GELU / residual / BatchNorm code every workgroup
// otherwise pulls cold from L2 once (the GEMM measurement: a launch with no K
// loop 12.9 -> 8.6 us, profiles/r5_vit_gemm_sweep.md); 1 = every feature.
template <int NBUF, class LA, class LB, int BN, int EPI>
__global__ __launch_bounds__(NT, NBUF == 1 ? 3 : (NBUF == 2 ? 2 : 1)) void conv_kernel(GemmParams p, LA la, LB lb, int tiles_m, int tiles_n) {
  __shared__ __attribute__((aligned(16))) char smem[smem_bytes<Tile128, NBUF>()];
  gemm_body<Tile128, NBUF, LA, LB, BN, EPI>(p, la, lb, tiles_m, tiles_n, smem);
}

// 64 x 64 output tiles (variant bit 14, kConvT64): four 32 x 32 waves; a k-major
// operand stages only its 64 rows (8 KB per half), so the forward's 4-stage ring is
// 64 KB -- two workgroups per CU -- and a 16x16 / 8x8 / 4x4 stage fills the chip
// with tiles instead of split-K slices (no slab reduce launch).  No BatchNorm
// statistics epilogue (BN = 0 only).
template <int NBUF, class LA, class LB, int EPI>
__global__ __launch_bounds__(NT, NBUF >= 3 ? 2 : 4) void conv64_kernel(GemmParams p, LA la, LB lb, int tiles_m, int tiles_n) {
  __shared__ __attribute__((aligned(16))) char smem[smem_bytes_l<Tile64, NBUF, LA, LB>()];
  gemm_body<Tile64, NBUF, LA, LB, 0, EPI>(p, la, lb, tiles_m, tiles_n, smem);
}

template <class LA, class LB, int EPI>
static void launch_e64(const GemmParams& p, const LA& la, const LB& lb, int grid, int tm, int tn, hipStream_t s) {
  if (p.variant & 4096)
    hipLaunchKernelGGL((conv64_kernel<4, LA, LB, EPI>), dim3(grid), dim3(NT), 0, s, p, la, lb, tm, tn);
  else if (p.variant & 8)
    hipLaunchKernelGGL((conv64_kernel<1, LA, LB, EPI>), dim3(grid), dim3(NT), 0, s, p, la, lb, tm, tn);
  else
    hipLaunchKernelGGL((conv64_kernel<2, LA, LB, EPI>), dim3(grid), dim3(NT), 0, s, p, la, lb, tm, tn);
}

template <class LA, class LB, int BN, int EPI>
static void launch_e(const GemmParams& p, const LA& la, const LB& lb, int grid, int tm, int tn, hipStream_t s) {
  if (p.variant & 4096)  // 4-stage ring, one workgroup per CU: short-K / small-grid shapes
    hipLaunchKernelGGL((conv_kernel<4, LA, LB, BN, EPI>), dim3(grid), dim3(NT), 0, s, p, la, lb, tm, tn);
  else if (p.variant & 8)
    hipLaunchKernelGGL((conv_kernel<1, LA, LB, BN, EPI>), dim3(grid), dim3(NT), 0, s, p, la, lb, tm, tn);
  else
    hipLaunchKernelGGL((conv_kernel<2, LA, LB, BN, EPI>), dim3(grid), dim3(NT), 0, s, p, la, lb, tm, tn);
}

template <class LA, class LB, int BN>
static void launch_t(const GemmParams& p, const LA& la, const LB& lb, hipStream_t s) {
  int tm, tn;
  if constexpr (BN == 0) {
    if (p.variant & kConvT64) {
      const int grid = gemm_grid<Tile64>(p, tm, tn);
      if (epilogue_kind(p) == 0)
        launch_e64<LA, LB, 0>(p, la, lb, grid, tm, tn, s);
      else
        launch_e64<LA, LB, 1>(p, la, lb, grid, tm, tn, s);
      return;
    }
  }
  const int grid = gemm_grid<Tile128>(p, tm, tn);
  if (BN == 0 && epilogue_kind(p) == 0)
    launch_e<LA, LB, BN, 0>(p, la, lb, grid, tm, tn, s);
  else
    launch_e<LA, LB, BN, 1>(p, la, lb, grid, tm, tn, s);
}

// the BatchNorm-statistics instantiation only where a launch asks for it; BNK: the
// statistics direction this product can carry (1 forward, 2 input gradient, 0 none)
template <int BNK, class LA, class LB>
static void launch(const GemmParams& p0, const LA& la, const LB& lb, hipStream_t s) {
  static const int bn_mode = [] {
    const char* e = getenv("P2_BN_EPI_MODE");
    return e ? atoi(e) : 0;
  }();
  GemmParams p = p0;
  p.bn.mode = bn_mode;
  if constexpr (BNK != 0) {
    if (p.bn.part) {
      launch_t<LA, LB, BNK>(p, la, lb, s);
      return;
    }
  }
  launch_t<LA, LB, 0>(p, la, lb, s);
}

static GemmParams base_params(int M, int N, int K, void* c, int64_t ldc, int c_bf16, const p2::SplitK& k,
                              int variant) {
  const int splits = k.splits;
  GemmParams p{};
  p.ws = k.ws;
  p.counters = splits > 1 ? k.counters : nullptr;
  p.M = M;
  p.N = N;
  p.K = K;
  p.c = c;
  p.ldc = ldc;
  p.c_bf16 = c_bf16;
  p.splits = splits < 1 ? 1 : splits;
  p.variant = variant;
  return p;
}

// One float4 column per thread, slices summed 8 loads at a time (independent
// loads in flight); 64-thread blocks so even a small gradient spreads over the CUs.
__global__ __launch_bounds__(64) void slab_sum_kernel(const float* __restrict__ slabs, int splits, int64_t n4,
                                                       void* out, int out_bf16) {
  const int64_t i = blockIdx.x * int64_t(64) + threadIdx.x;
  if (i >= n4) return;
  const f32x4* src = reinterpret_cast<const f32x4*>(slabs) + i;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  int s = 0;
  for (; s + 8 <= splits; s += 8) {
    f32x4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = src[(s + u) * n4];
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += v[u];
  }
  for (; s < splits; ++s) acc += src[s * n4];
  if (out_bf16)
    reinterpret_cast<uint2*>(out)[i] = uint2{pack_bf16x2(acc[0], acc[1]), pack_bf16x2(acc[2], acc[3])};
  else
    reinterpret_cast<f32x4*>(out)[i] = acc;
}

}  // namespace p2gemm

namespace p2 {

void conv_fwd(const ConvShape& s, const uint16_t* x, const uint16_t* w, void* y, const SplitK& k, int variant,
              hipStream_t st, const BnEpi* bn) {
  using namespace p2gemm;
  const int M = s.N * s.OH * s.OW, K = s.kh * s.kw * s.C;
  GemmParams p = base_params(M, s.O, K, y, s.O, k.splits <= 1 || k.counters, k, variant);
  if (bn) p.bn = *bn;
  const ConvFwdA la{x,   make_fastdiv(s.OH * s.OW), make_fastdiv(s.OW), make_fastdiv(s.C), make_fastdiv(s.kw), M, s.H, s.W,
                    s.C, s.stride, s.pad, s.dil, s.kw};
  launch<1>(p, la, PlainK{w, K, s.O, K}, st);
}

void conv_dgrad(const ConvShape& s, const uint16_t* dy, const uint16_t* w, void* dx, const SplitK& k, int variant,
                hipStream_t st, const BnEpi* bn) {
  using namespace p2gemm;
  const int M = s.N * s.H * s.W, K = s.kh * s.kw * s.O;
  GemmParams p = base_params(M, s.C, K, dx, s.C, k.splits <= 1 || k.counters, k, variant);
  if (bn) p.bn = *bn;
  const ConvDgradA la{dy,  make_fastdiv(s.H * s.W), make_fastdiv(s.W), make_fastdiv(s.O), make_fastdiv(s.kw), M, s.OH, s.OW,
                      s.O, s.stride, s.pad, s.dil, s.kw};
  launch<2>(p, la, ConvDgradB{w, make_fastdiv(s.O), s.C, s.O, s.kh * s.kw}, st);
}

// phases with taps: all four, or only (0, 0) for a 1x1 kernel (pad 0; with pad p
// the tap-less phases are the ones with (ih + p) odd -- still phases 1..3)
int s2_phases(const ConvShape& s) { return (s.kh == 1 && s.kw == 1) ? 1 : 4; }

bool conv_dgrad_s2_ok(const ConvShape& s) {
  const int64_t Mq = int64_t(s.N) * (s.H / 2) * (s.W / 2);
  return s.stride == 2 && s.dil == 1 && s.H % 2 == 0 && s.W % 2 == 0 && Mq % 128 == 0 && 4 * Mq < (int64_t(1) << 31);
}

void conv_dgrad_s2(const ConvShape& s, const uint16_t* dy, const uint16_t* w, void* dx_phases, const SplitK& k, int variant,
                   hipStream_t st) {
  using namespace p2gemm;
  const int H2 = s.H / 2, W2 = s.W / 2, Mq = s.N * H2 * W2;
  const int K = ((s.kh + 1) / 2) * ((s.kw + 1) / 2) * s.O;
  GemmParams p = base_params(s2_phases(s) * Mq, s.C, K, dx_phases, s.C, k.splits <= 1 || k.counters, k, variant);
  const ConvDgradS2A la{dy, make_fastdiv(H2 * W2), make_fastdiv(W2), make_fastdiv(s.O), Mq, W2, s.OH, s.OW, s.O,
                        s.pad, s.kh, s.kw};
  const ConvDgradS2B lb{w, make_fastdiv(s.O), s.C, s.O, Mq, s.kh, s.kw, 0, 0};
  launch<0>(p, la, lb, st);
}

void phase_interleave(const ConvShape& s, const uint16_t* src, uint16_t* dx, hipStream_t st) {
  using namespace p2gemm;
  const int H2 = s.H / 2, W2 = s.W / 2, Mq = s.N * H2 * W2, cpr = s.C / 8;
  const int64_t nchunks = int64_t(4) * Mq * cpr;
  hipLaunchKernelGGL(phase_interleave_kernel, dim3(int((nchunks + 255) / 256)), dim3(256), 0, st,
                     reinterpret_cast<const uint4*>(src), reinterpret_cast<uint4*>(dx), nchunks, cpr, make_fastdiv(cpr),
                     make_fastdiv(H2 * W2), make_fastdiv(W2), Mq, s2_phases(s), s.H, s.W, s.pad);
}

void conv_wgrad(const ConvShape& s, const uint16_t* dy, const uint16_t* x, void* out, int out_bf16, const SplitK& k,
                int variant, hipStream_t st) {
  using namespace p2gemm;
  const int npix = s.N * s.OH * s.OW, ncols = s.kh * s.kw * s.C;
  const GemmParams p =
      base_params(s.O, ncols, npix, out, ncols, (k.splits > 1 && !k.counters) ? 0 : out_bf16, k, variant);
  const ConvWgradB lb{x,   make_fastdiv(s.OH * s.OW), make_fastdiv(s.OW), make_fastdiv(s.C), npix, s.H, s.W, s.C,
                      s.stride, s.pad, s.dil, s.kw, ncols};
  launch<0>(p, PlainMN{dy, s.O, s.O, npix}, lb, st);
}

void slab_sum(const float* slabs, int splits, int64_t n, void* out, int out_bf16, hipStream_t st) {
  const int64_t n4 = n / 4;
  hipLaunchKernelGGL(p2gemm::slab_sum_kernel, dim3(int((n4 + 63) / 64)), dim3(64), 0, st, slabs, splits, n4, out,
                     out_bf16);
}

}  // namespace p2
