// Direct convolution for inputs with few channels (the 3-channel ResNet stem),
// gfx950.  The implicit-GEMM kernels of conv.hip stage 8 consecutive channels
// of a pixel per 16-byte chunk, which a 3-channel image does not have; the
// stem is tiny (K = kh * kw * C = 27 for the CIFAR 3x3 stem, 147 for 7x7), so
// it gets two dedicated kernels instead of MIOpen:
//
//   forward  y[n][oh][ow][o] = sum_k x~(p, k) w[o][k]     (fp32 FMA, weights in LDS)
//   wgrad    dw[o][k]        = sum_p dy[p][o] x~(p, k)    (MFMA 32x32x16 bf16 over
//                                                          16-pixel k-steps, fixed-
//                                                          order partials + reduce)
//
// x is read in whatever layout and dtype the batch has (fp32 / bf16 / uint8,
// NCHW or channels-last, through element strides) and rounded to bf16 -- the
// value autocast would hand the convolution -- so the model needs neither a
// channels-last copy nor a dtype cast of the input; a uint8 batch folds the
// 1/255 normalisation in.  No dgrad: the stem's input is data.
//
// Reference op: the first convolution of the reference CNN,
// /root/reference/p2pfl/learning/pytorch/mnist_examples/models/cnn.py:55-60
// (1 input channel: the same small-K problem).
#include "conv.h"
#include "gemm_core.h"

namespace p2stem {
using namespace p2;

struct StemArgs {
  int N, H, W, C, O, OH, OW, kh, kw, stride, pad;
  int64_t sn, sc, sh, sw;  // element strides of x
  float xscale;
};

template <typename TX>
P2_DEVICE float load_x(const TX* x, int64_t off, float scale);
template <>
P2_DEVICE float load_x<float>(const float* x, int64_t off, float scale) {
  return bf16_to_f32(f32_to_bf16(x[off] * scale));
}
template <>
P2_DEVICE float load_x<uint16_t>(const uint16_t* x, int64_t off, float scale) {
  return bf16_to_f32(f32_to_bf16(bf16_to_f32(x[off]) * scale));
}
template <>
P2_DEVICE float load_x<uint8_t>(const uint8_t* x, int64_t off, float scale) {
  return bf16_to_f32(f32_to_bf16(float(x[off]) * scale));
}

constexpr int kMaxK = 160;       // kh * kw * C (7 x 7 x 3 = 147)
constexpr int kLdsW = 40 * 1024;  // fp32 weight image [K][O]

// ---- forward: thread = one output pixel x 16 output channels --------------------
template <typename TX>
__global__ __launch_bounds__(256) void stem_fwd_kernel(const TX* __restrict__ x, const uint16_t* __restrict__ w,
                                                       uint16_t* __restrict__ y, StemArgs a) {
  __shared__ __attribute__((aligned(16))) float wl[kLdsW / 4];
  const int K = a.kh * a.kw * a.C, OB = a.O / 16;
  // weights (O, kh, kw, C) bf16 -> LDS [k][o] fp32
  for (int i = threadIdx.x; i < a.O * K; i += 256) {
    const int o = i / K, k = i - o * K;
    wl[k * a.O + o] = bf16_to_f32(w[i]);
  }
  __syncthreads();
  const int P = a.N * a.OH * a.OW;
  const int ppb = 256 / OB;
  const int p = blockIdx.x * ppb + int(threadIdx.x) / OB, ob = int(threadIdx.x) % OB;
  if (int(threadIdx.x) >= ppb * OB || p >= P) return;
  const int n = p / (a.OH * a.OW), r = p - n * (a.OH * a.OW);
  const int oh = r / a.OW, ow = r - oh * a.OW;
  const int ih0 = oh * a.stride - a.pad, iw0 = ow * a.stride - a.pad;
  float acc[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) acc[j] = 0.f;
  const TX* xn = x + int64_t(n) * a.sn;
  int k = 0;
  for (int ky = 0; ky < a.kh; ++ky) {
    const int ih = ih0 + ky;
    for (int kx = 0; kx < a.kw; ++kx) {
      const int iw = iw0 + kx;
      const bool ok = unsigned(ih) < unsigned(a.H) && unsigned(iw) < unsigned(a.W);
      for (int c = 0; c < a.C; ++c, ++k) {
        const float xv = ok ? load_x<TX>(xn, c * a.sc + ih * a.sh + iw * a.sw, a.xscale) : 0.f;
        const f32x4* wr = reinterpret_cast<const f32x4*>(wl + k * a.O + ob * 16);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f32x4 wv = wr[q];
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[4 * q + e] = fmaf(xv, wv[e], acc[4 * q + e]);
        }
      }
    }
  }
  uint4* dst = reinterpret_cast<uint4*>(y + int64_t(p) * a.O + ob * 16);
  dst[0] = uint4{pack_bf16x2(acc[0], acc[1]), pack_bf16x2(acc[2], acc[3]), pack_bf16x2(acc[4], acc[5]),
                 pack_bf16x2(acc[6], acc[7])};
  dst[1] = uint4{pack_bf16x2(acc[8], acc[9]), pack_bf16x2(acc[10], acc[11]), pack_bf16x2(acc[12], acc[13]),
                 pack_bf16x2(acc[14], acc[15])};
}

// ---- weight gradient -----------------------------------------------------------------
// D[kidx][o] = sum_p X~[p][kidx] dy[p][o] with v_mfma_f32_32x32x16_bf16: A = X~^T
// (rows kidx, 32 per block, KB blocks), B = dy (cols o, 32 per block, OBK blocks), k
// = 16 pixels.  Lane l supplies A[kidx = 32 rb + (l & 31)][p0 + 8 (l >> 5) + j] and
// B[p0 + 8 (l >> 5) + j][o = 32 cb + (l & 31)], j = 0..7, and holds D[32 rb + 8 (v / 4)
// + 4 (l >> 5) + v % 4][32 cb + (l & 31)] in element v of acc[rb][cb].  Each wave
// reduces a pixel range; the workgroup's 4 waves add into one LDS image in fixed wave
// order and the workgroup writes its [O][K] partial; stem_wgrad_reduce sums the
// partials over workgroups in fixed order (bitwise reproducible).
constexpr int kPixPerWave = 64;

template <typename TX, int KB, int OBK>
__global__ __launch_bounds__(256) void stem_wgrad_kernel(const TX* __restrict__ x, const uint16_t* __restrict__ dy,
                                                         float* __restrict__ part, StemArgs a) {
  __shared__ __attribute__((aligned(16))) float red[KB * 32 * OBK * 32];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, l32 = lane & 31;
  const int K = a.kh * a.kw * a.C, P = a.N * a.OH * a.OW, OHW = a.OH * a.OW;
  // this lane's A rows: kidx = 32 rb + l32 -> (ky, kx, c)
  int dky[KB], dkx[KB], dc[KB];
#pragma unroll
  for (int rb = 0; rb < KB; ++rb) {
    const int kidx = 32 * rb + l32;
    const int c = kidx % a.C, t = kidx / a.C;
    dky[rb] = kidx < K ? t / a.kw : (1 << 28);
    dkx[rb] = t % a.kw;
    dc[rb] = c;
  }
  f32x16 acc[KB][OBK];
#pragma unroll
  for (int rb = 0; rb < KB; ++rb)
#pragma unroll
    for (int cb = 0; cb < OBK; ++cb)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[rb][cb][e] = 0.f;
  const int pw0 = (blockIdx.x * 4 + wave) * kPixPerWave;
#pragma unroll 2
  for (int s = 0; s < kPixPerWave / 16; ++s) {
    const int p0 = pw0 + 16 * s + 8 * h;
    // decode the lane's 8 pixels (consecutive)
    int pn[8], poh[8], pow_[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int p = p0 + j;
      const int n = p / OHW, r = p - n * OHW;
      pn[j] = p < P ? n : -1;
      poh[j] = r / a.OW;
      pow_[j] = r - poh[j] * a.OW;
    }
    uint16_t bv[OBK][8];
#pragma unroll
    for (int cb = 0; cb < OBK; ++cb)
#pragma unroll
      for (int j = 0; j < 8; ++j) bv[cb][j] = pn[j] >= 0 ? dy[int64_t(p0 + j) * a.O + 32 * cb + l32] : uint16_t(0);
    uint16_t av[KB][8];
#pragma unroll
    for (int rb = 0; rb < KB; ++rb)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int ih = poh[j] * a.stride - a.pad + dky[rb], iw = pow_[j] * a.stride - a.pad + dkx[rb];
        const bool ok = pn[j] >= 0 && unsigned(ih) < unsigned(a.H) && unsigned(iw) < unsigned(a.W);
        av[rb][j] = ok ? f32_to_bf16(load_x<TX>(x, int64_t(pn[j]) * a.sn + dc[rb] * a.sc + ih * a.sh + iw * a.sw,
                                                a.xscale))
                       : uint16_t(0);
      }
#pragma unroll
    for (int rb = 0; rb < KB; ++rb) {
      uint4 fa;
      fa.x = av[rb][0] | (uint32_t(av[rb][1]) << 16);
      fa.y = av[rb][2] | (uint32_t(av[rb][3]) << 16);
      fa.z = av[rb][4] | (uint32_t(av[rb][5]) << 16);
      fa.w = av[rb][6] | (uint32_t(av[rb][7]) << 16);
#pragma unroll
      for (int cb = 0; cb < OBK; ++cb) {
        uint4 fb;
        fb.x = bv[cb][0] | (uint32_t(bv[cb][1]) << 16);
        fb.y = bv[cb][2] | (uint32_t(bv[cb][3]) << 16);
        fb.z = bv[cb][4] | (uint32_t(bv[cb][5]) << 16);
        fb.w = bv[cb][6] | (uint32_t(bv[cb][7]) << 16);
        acc[rb][cb] = p2gemm::mfma(fa, fb, acc[rb][cb]);
      }
    }
  }
  // fixed-order sum of the 4 waves in LDS: red[kidx][o]
  constexpr int OW_ = OBK * 32;
  for (int wv = 0; wv < 4; ++wv) {
    if (wave == wv) {
#pragma unroll
      for (int rb = 0; rb < KB; ++rb)
#pragma unroll
        for (int cb = 0; cb < OBK; ++cb)
#pragma unroll
          for (int v = 0; v < 16; ++v) {
            const int kidx = 32 * rb + 8 * (v / 4) + 4 * h + (v % 4), o = 32 * cb + l32;
            float* d = red + kidx * OW_ + o;
            *d = wv == 0 ? acc[rb][cb][v] : *d + acc[rb][cb][v];
          }
    }
    __syncthreads();
  }
  // partial [O][K] of this workgroup
  float* out = part + int64_t(blockIdx.x) * a.O * K;
  for (int i = threadIdx.x; i < a.O * K; i += 256) {
    const int o = i / K, k = i - o * K;
    out[i] = red[k * OW_ + o];
  }
}

// dw[i] = sum_b part[b][i], i < n: 32 outputs x 8 partial-row phases per workgroup
__global__ __launch_bounds__(256) void stem_wgrad_reduce(const float* __restrict__ part, int nparts, int n,
                                                         void* __restrict__ dw, int out_bf16) {
  __shared__ float red[8][32];
  const int col = threadIdx.x & 31, ph = threadIdx.x >> 5;
  const int i = blockIdx.x * 32 + col;
  float s = 0.f;
  if (i < n)
    for (int b = ph; b < nparts; b += 8) s += part[int64_t(b) * n + i];
  red[ph][col] = s;
  __syncthreads();
  if (ph == 0 && i < n) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) t += red[q][col];
    if (out_bf16)
      reinterpret_cast<uint16_t*>(dw)[i] = f32_to_bf16(t);
    else
      reinterpret_cast<float*>(dw)[i] = t;
  }
}

template <typename TX, int KB>
void launch_wgrad_kb(const TX* x, const uint16_t* dy, float* part, const StemArgs& a, int nwg, hipStream_t st) {
  if (a.O == 32)
    hipLaunchKernelGGL((stem_wgrad_kernel<TX, KB, 1>), dim3(nwg), dim3(256), 0, st, x, dy, part, a);
  else
    hipLaunchKernelGGL((stem_wgrad_kernel<TX, KB, 2>), dim3(nwg), dim3(256), 0, st, x, dy, part, a);
}

template <typename TX>
void launch_wgrad(const TX* x, const uint16_t* dy, float* part, const StemArgs& a, int nwg, hipStream_t st) {
  const int K = a.kh * a.kw * a.C;
  if (K <= 32)
    launch_wgrad_kb<TX, 1>(x, dy, part, a, nwg, st);
  else if (K <= 64)
    launch_wgrad_kb<TX, 2>(x, dy, part, a, nwg, st);
  else if (K <= 96)
    launch_wgrad_kb<TX, 3>(x, dy, part, a, nwg, st);
  else if (K <= 128)
    launch_wgrad_kb<TX, 4>(x, dy, part, a, nwg, st);
  else
    launch_wgrad_kb<TX, 5>(x, dy, part, a, nwg, st);
}

}  // namespace p2stem

namespace p2 {

int stem_wgrad_parts(int N, int OH, int OW) {
  const int P = N * OH * OW;
  return (P + 4 * p2stem::kPixPerWave - 1) / (4 * p2stem::kPixPerWave);
}

void stem_fwd(const StemShape& s, const void* x, int xtype, const uint16_t* w, uint16_t* y, hipStream_t st) {
  using namespace p2stem;
  const StemArgs a{s.N, s.H, s.W, s.C, s.O, s.OH, s.OW, s.kh, s.kw, s.stride, s.pad, s.sn, s.sc, s.sh, s.sw, s.xscale};
  const int P = s.N * s.OH * s.OW, ppb = 256 / (s.O / 16);
  const int grid = (P + ppb - 1) / ppb;
  if (xtype == 0)
    hipLaunchKernelGGL(stem_fwd_kernel<float>, dim3(grid), dim3(256), 0, st, static_cast<const float*>(x), w, y, a);
  else if (xtype == 1)
    hipLaunchKernelGGL(stem_fwd_kernel<uint16_t>, dim3(grid), dim3(256), 0, st, static_cast<const uint16_t*>(x), w, y, a);
  else
    hipLaunchKernelGGL(stem_fwd_kernel<uint8_t>, dim3(grid), dim3(256), 0, st, static_cast<const uint8_t*>(x), w, y, a);
}

void stem_wgrad(const StemShape& s, const void* x, int xtype, const uint16_t* dy, float* part, void* dw, int out_bf16,
                hipStream_t st) {
  using namespace p2stem;
  const StemArgs a{s.N, s.H, s.W, s.C, s.O, s.OH, s.OW, s.kh, s.kw, s.stride, s.pad, s.sn, s.sc, s.sh, s.sw, s.xscale};
  const int nwg = stem_wgrad_parts(s.N, s.OH, s.OW);
  if (xtype == 0)
    launch_wgrad(static_cast<const float*>(x), dy, part, a, nwg, st);
  else if (xtype == 1)
    launch_wgrad(static_cast<const uint16_t*>(x), dy, part, a, nwg, st);
  else
    launch_wgrad(static_cast<const uint8_t*>(x), dy, part, a, nwg, st);
  const int n = s.O * s.kh * s.kw * s.C;
  hipLaunchKernelGGL(stem_wgrad_reduce, dim3((n + 31) / 32), dim3(256), 0, st, part, nwg, n, dw, out_bf16);
}

}  // namespace p2
