// Fused MNIST-CNN training step -- backward kernels with fused Adam epilogues.
// Layouts: see cnn_fwd.hip.  Extra buffers:
//   dH    bf16 [mrows][2048]     dLoss/dH (ReLU mask applied), rows >= B are zero
//   dHt   bf16 [2048][mrows]     the same, transposed (A operand of dW1)
//   slabs2 f32 [S2][mrows][3136] split-K partials of dA1 = dH x W1
//   W2q   bf16 [32][25][64]      conv2 weight, (ic, tap, oc) -- B operand of the transposed conv
//   wslab1 f32 [B][832]          per-image conv1 weight/bias gradients
//   wslab2 f32 [B][51264]        per-image conv2 weight/bias gradients
// Adam's step counter lives in device memory (step_begin increments it), so
// the whole step can be captured once in a HIP graph and replayed.
#include "cnn.h"
#include "common.h"

namespace p2cnn {
using namespace p2;

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
P2_DEVICE f32x16 mfma32b(uint4 a, uint4 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c,
                                                  0, 0, 0);
}
P2_DEVICE int acc_row_b(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

struct AdamScal {
  float step_size, inv_sqrt_bc2;
};
P2_DEVICE AdamScal adam_scal(const AdamCfg& c, const int* t) {
  const float tt = float(*t);
  AdamScal s;
  s.step_size = c.lr / (1.f - powf(c.beta1, tt));
  s.inv_sqrt_bc2 = 1.f / sqrtf(1.f - powf(c.beta2, tt));
  return s;
}
// torch.optim.Adam semantics (L2 weight decay added to the gradient).
P2_DEVICE float adam_apply(float* __restrict__ p, float* __restrict__ m, float* __restrict__ v, int64_t e, float g,
                           const AdamCfg& c, const AdamScal& s) {
  float pv = p[e];
  if (c.weight_decay != 0.f) g = fmaf(c.weight_decay, pv, g);
  const float mv = fmaf(c.beta1, m[e], (1.f - c.beta1) * g);
  const float vv = fmaf(c.beta2, v[e], (1.f - c.beta2) * g * g);
  pv -= s.step_size * (mv / (sqrtf(vv) * s.inv_sqrt_bc2 + c.eps));
  p[e] = pv;
  m[e] = mv;
  v[e] = vv;
  return pv;
}

// ---------------------------------------------------------------------------
// 6. FC2 weight/bias gradient + Adam: dW2[c][k] = sum_b dlogits[b][c] H[b][k].
//    20,490 parameters, one thread each, Adam applied in place.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void fc2_wgrad_adam_kernel(const float* __restrict__ dlogits,
                                                             const uint16_t* __restrict__ H, int B,
                                                             float* __restrict__ p, float* __restrict__ m,
                                                             float* __restrict__ v, float* __restrict__ gdump,
                                                             Offsets off, const int* __restrict__ adam_t, AdamCfg cfg) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  const int nW = kCls * kHid;
  if (e >= nW + kCls) return;
  float g = 0.f;
  int64_t pi;
  if (e < nW) {
    const int c = e / kHid, k = e % kHid;
    for (int b = 0; b < B; ++b) g = fmaf(dlogits[b * kCls + c], bf16_to_f32(H[size_t(b) * kHid + k]), g);
    pi = off.l2w + e;
  } else {
    const int c = e - nW;
    for (int b = 0; b < B; ++b) g += dlogits[b * kCls + c];
    pi = off.l2b + c;
  }
  if (gdump) gdump[pi] = g;
  const AdamScal s = adam_scal(cfg, adam_t);
  adam_apply(p, m, v, pi, g, cfg, s);
}

void fc2_wgrad_adam(const float* dlogits, const uint16_t* H, int B, float* params, float* m, float* v, float* gdump,
                    Offsets off, const int* adam_t, AdamCfg cfg, hipStream_t s) {
  const int n = kCls * kHid + kCls;
  hipLaunchKernelGGL(fc2_wgrad_adam_kernel, dim3((n + 255) / 256), dim3(256), 0, s, dlogits, H, B, params, m, v,
                     gdump, off, adam_t, cfg);
}

// ---------------------------------------------------------------------------
// 8. FC1 weight gradient on MFMA with Adam fused into the epilogue.
//    dW1[n][k] = sum_b dHt[n][b] * A1t[k][b]  (K = batch, mrows/16 k-steps).
//    Grid (25, 64): block = 32 rows of n x 128 columns of k (one 32x32 tile
//    per wave).  The gradient tile never leaves registers: each lane updates
//    W1/m/v for its 16 elements (two coalesced 128-B rows per register), writes
//    the bf16 shadow, and stages the bf16 tile in LDS so the transposed shadow
//    W1^T is written as 64-B row segments.
// ---------------------------------------------------------------------------
template <int KS>
__global__ __launch_bounds__(256) void fc1_wgrad_adam_kernel(const uint16_t* __restrict__ dHt,
                                                             const uint16_t* __restrict__ a1t, int mrows,
                                                             float* __restrict__ p, float* __restrict__ m,
                                                             float* __restrict__ v, float* __restrict__ gdump,
                                                             uint16_t* __restrict__ w1bf,
                                                             uint16_t* __restrict__ w1tbf, Offsets off,
                                                             const int* __restrict__ adam_t, AdamCfg cfg) {
  __shared__ __attribute__((aligned(16))) uint16_t tr[128][40];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const int n0 = blockIdx.y * 32;
  const int k0 = (blockIdx.x * 4 + wave) * 32;
  const bool valid = k0 < kFeat;
  f32x16 acc = {};
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const uint4 a = *reinterpret_cast<const uint4*>(dHt + size_t(n0 + r) * mrows + ks * 16 + 8 * h);
    const uint4 b = valid ? *reinterpret_cast<const uint4*>(a1t + size_t(k0 + r) * mrows + ks * 16 + 8 * h)
                          : make_uint4(0, 0, 0, 0);
    acc = mfma32b(a, b, acc);
  }
  const AdamScal s = adam_scal(cfg, adam_t);
  float* pw = p + off.l1w;
  float* mw = m + off.l1w;
  float* vw = v + off.l1w;
  if (valid) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int nl = acc_row_b(i, h);
      const int64_t e = int64_t(n0 + nl) * kFeat + k0 + r;
      if (gdump) gdump[off.l1w + e] = acc[i];
      const float pn = adam_apply(pw, mw, vw, e, acc[i], cfg, s);
      const uint16_t hb = f32_to_bf16(pn);
      w1bf[e] = hb;
      tr[wave * 32 + r][nl] = hb;
    }
  }
  __syncthreads();
  for (int j = tid; j < 128 * 4; j += 256) {
    const int kl = j >> 2, q = j & 3;
    const int k = blockIdx.x * 128 + kl;
    if (k < kFeat)
      *reinterpret_cast<uint4*>(w1tbf + size_t(k) * kHid + n0 + q * 8) = *reinterpret_cast<const uint4*>(&tr[kl][q * 8]);
  }
  if (blockIdx.x == 0 && wave == 0 && lane < 32) {
    const int n = n0 + lane;
    float g = 0.f;
    for (int b = 0; b < mrows; ++b) g += bf16_to_f32(dHt[size_t(n) * mrows + b]);
    if (gdump) gdump[off.l1b + n] = g;
    adam_apply(p, m, v, off.l1b + n, g, cfg, s);
  }
}

void fc1_wgrad_adam(const uint16_t* dHt, const uint16_t* a1t, int mrows, float* params, float* m, float* v,
                    float* gdump, uint16_t* w1bf, uint16_t* w1tbf, Offsets off, const int* adam_t, AdamCfg cfg,
                    hipStream_t s) {
  const dim3 grid((kFeat / 32 + 3) / 4, kHid / 32);
  if (mrows == 32)
    hipLaunchKernelGGL(fc1_wgrad_adam_kernel<2>, grid, dim3(256), 0, s, dHt, a1t, mrows, params, m, v, gdump, w1bf,
                       w1tbf, off, adam_t, cfg);
  else
    hipLaunchKernelGGL(fc1_wgrad_adam_kernel<4>, grid, dim3(256), 0, s, dHt, a1t, mrows, params, m, v, gdump, w1bf,
                       w1tbf, off, adam_t, cfg);
}

// ---------------------------------------------------------------------------
// shared: dC2 = maxpool2/ReLU backward of dA1 (sum of the split-K slabs),
// routed to the argmax position of each 2x2 window.
// ---------------------------------------------------------------------------
P2_DEVICE float dA1_value(const float* __restrict__ slabs2, int S2, int mrows, int b, int feat) {
  float g = 0.f;
  for (int s = 0; s < S2; ++s) g += slabs2[(size_t(s) * mrows + b) * kFeat + feat];
  return g;
}

// ---------------------------------------------------------------------------
// 9. conv2 weight gradient on MFMA, per image and tap group.
//    Grid (4, B), 8 waves.  C[oc][ic] for tap t = sum_pos dC2[oc][pos] *
//    P1pad[pos + tap][ic]; M = 64 oc (2 tiles), N = 32 ic per tap, K = 196
//    positions (14 k-steps).  A fragments are 16-B LDS reads of the [oc][pos]
//    dC2 image; B fragments gather 8 positions of one channel from the HWC
//    image (a position->pixel offset table in LDS keeps the address math out
//    of the loop).  Output: per-image slab in PyTorch [oc][ic][ky][kx] order.
// ---------------------------------------------------------------------------
constexpr int kICP2 = 40;
constexpr int kWgImg = 18 * 18 * kICP2 * 2;  // 25920
constexpr int kWgDc2 = 64 * 224 * 2;         // 28672
constexpr int kWgTab = 224 * 4;              // 896
constexpr int kWgLds = kWgImg + kWgDc2 + kWgTab;

__global__ __launch_bounds__(512) void conv2_wgrad_kernel(const float* __restrict__ slabs2, int S2, int mrows,
                                                          const uint8_t* __restrict__ am2,
                                                          const uint16_t* __restrict__ p1,
                                                          float* __restrict__ wslab) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint16_t* simg = reinterpret_cast<uint16_t*>(smem);
  uint16_t* dc2 = reinterpret_cast<uint16_t*>(smem + kWgImg);
  int* tab = reinterpret_cast<int*>(smem + kWgImg + kWgDc2);
  const int b = blockIdx.y, grp = blockIdx.x, tid = threadIdx.x;
  const uint4 z4 = make_uint4(0, 0, 0, 0);
  for (int i = tid; i < kWgImg / 16; i += 512) reinterpret_cast<uint4*>(simg)[i] = z4;
  for (int i = tid; i < kWgDc2 / 16; i += 512) reinterpret_cast<uint4*>(dc2)[i] = z4;
  for (int i = tid; i < 224; i += 512) {
    const int pc = i < 196 ? i : 195;
    tab[i] = ((pc / 14) * 18 + (pc % 14)) * kICP2;
  }
  __syncthreads();
  for (int i = tid; i < 196 * 4; i += 512) {
    const int pix = i >> 2, q = i & 3, y = pix / 14, x = pix % 14;
    *reinterpret_cast<uint4*>(simg + ((y + 2) * 18 + (x + 2)) * kICP2 + q * 8) =
        reinterpret_cast<const uint4*>(p1 + (size_t(b) * 196 + pix) * kC1)[q];
  }
  for (int i = tid; i < kC2 * 49; i += 512) {
    const int oc = i / 49, pp = i % 49;
    const int feat = oc * 49 + pp;
    const uint8_t a = am2[size_t(b) * kFeat + feat];
    if (a < 4) {
      const float g = dA1_value(slabs2, S2, mrows, b, feat);
      const int pos = (2 * (pp / 7) + (a >> 1)) * 14 + 2 * (pp % 7) + (a & 1);
      dc2[oc * 224 + pos] = f32_to_bf16(g);
    }
  }
  if (grp == 0 && tid < kC2) {  // conv2 bias gradient (fp32, unrounded)
    float gb = 0.f;
    for (int pp = 0; pp < 49; ++pp) {
      const int feat = tid * 49 + pp;
      if (am2[size_t(b) * kFeat + feat] < 4) gb += dA1_value(slabs2, S2, mrows, b, feat);
    }
    wslab[size_t(b) * kSlab2 + kC2 * kC1 * kTaps + tid] = gb;
  }
  __syncthreads();
  const int wave = tid >> 6, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const int mt = wave & 1, tw = wave >> 1;
  for (int tj = tw; tj < 7; tj += 4) {
    const int t = grp + 4 * tj;
    if (t >= kTaps) break;
    const int tap_off = ((t / 5) * 18 + (t % 5)) * kICP2 + r;
    f32x16 acc = {};
#pragma unroll 2
    for (int ks = 0; ks < 14; ++ks) {
      const uint4 a = *reinterpret_cast<const uint4*>(dc2 + (mt * 32 + r) * 224 + ks * 16 + 8 * h);
      uint16_t bv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) bv[j] = simg[tab[ks * 16 + 8 * h + j] + tap_off];
      uint4 bq;
      bq.x = uint32_t(bv[0]) | (uint32_t(bv[1]) << 16);
      bq.y = uint32_t(bv[2]) | (uint32_t(bv[3]) << 16);
      bq.z = uint32_t(bv[4]) | (uint32_t(bv[5]) << 16);
      bq.w = uint32_t(bv[6]) | (uint32_t(bv[7]) << 16);
      acc = mfma32b(a, bq, acc);
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int oc = mt * 32 + acc_row_b(i, h);
      wslab[size_t(b) * kSlab2 + (oc * kC1 + r) * kTaps + t] = acc[i];
    }
  }
}

void conv2_wgrad(const float* slabs2, int S2, int mrows, const uint8_t* am2, const uint16_t* p1, float* wslab, int B,
                 hipStream_t s) {
  hipLaunchKernelGGL(conv2_wgrad_kernel, dim3(4, B), dim3(512), kWgLds, s, slabs2, S2, mrows, am2, p1, wslab);
}

// ---------------------------------------------------------------------------
// 10. conv2 input gradient (transposed conv on MFMA) with pool1/ReLU backward
//     and the conv1 weight gradient fused into the epilogue.  Grid B, 7 waves
//     (one 32-position tile each).  C[pos][ic] = sum_{tap,oc}
//     dC2pad[pos - tap][oc] * W2[oc][ic][tap]: K = 25 x 64 (100 k-steps), A from
//     the padded HWC dC2 image, B from the (ic, tap, oc) weight copy, both
//     16-B LDS reads.  The resulting dP1 never leaves registers: each lane owns
//     one channel, routes its values through the pool1 argmax and accumulates
//     that channel's 25 conv1 weight gradients + bias gradient against the
//     input image in LDS; lanes and waves are then reduced through LDS.
// ---------------------------------------------------------------------------
constexpr int kW2qRow = kTaps * kC2 + 8;            // 1608 elements per ic (pad breaks bank aliasing)
constexpr int kDgW = kC1 * kW2qRow * 2;             // 102912
constexpr int kOCP = 72;                            // dC2 pixel stride (144 B)
constexpr int kDgDc2 = 18 * 18 * kOCP * 2;          // 46656
constexpr int kDgX = 32 * 32 * 4;                   // 4096
constexpr int kDgLds = kDgW + kDgDc2 + kDgX;        // 153664

__global__ __launch_bounds__(448) void conv2_dgrad_kernel(const float* __restrict__ slabs2, int S2, int mrows,
                                                          const uint8_t* __restrict__ am2,
                                                          const uint8_t* __restrict__ am1,
                                                          const uint16_t* __restrict__ w2q,
                                                          const uint8_t* __restrict__ xds,
                                                          const int64_t* __restrict__ idx,
                                                          float* __restrict__ wslab1) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint16_t* sw = reinterpret_cast<uint16_t*>(smem);
  uint16_t* dch = reinterpret_cast<uint16_t*>(smem + kDgW);
  float* ximg = reinterpret_cast<float*>(smem + kDgW + kDgDc2);
  const int b = blockIdx.x, tid = threadIdx.x;
  const uint4 z4 = make_uint4(0, 0, 0, 0);
  for (int i = tid; i < kDgDc2 / 16; i += 448) reinterpret_cast<uint4*>(dch)[i] = z4;
  for (int i = tid; i < kC1 * (kTaps * kC2 / 8); i += 448) {
    const int ic = i / (kTaps * kC2 / 8), q = i % (kTaps * kC2 / 8);
    *reinterpret_cast<uint4*>(sw + ic * kW2qRow + q * 8) =
        reinterpret_cast<const uint4*>(w2q + size_t(ic) * kTaps * kC2)[q];
  }
  const int64_t row = idx ? idx[b] : b;
  const uint8_t* src = xds + row * (kImg * kImg);
  for (int i = tid; i < 32 * 32; i += 448) {
    const int yy = i >> 5, xx = i & 31, sy = yy - 2, sx = xx - 2;
    ximg[i] = (sy >= 0 && sy < kImg && sx >= 0 && sx < kImg) ? float(src[sy * kImg + sx]) * (1.f / 255.f) : 0.f;
  }
  __syncthreads();
  for (int i = tid; i < kC2 * 49; i += 448) {
    const int oc = i % kC2, pp = i / kC2;  // oc fastest: neighbouring threads write neighbouring LDS halves
    const int feat = oc * 49 + pp;
    const uint8_t a = am2[size_t(b) * kFeat + feat];
    if (a < 4) {
      const float g = dA1_value(slabs2, S2, mrows, b, feat);
      const int y = 2 * (pp / 7) + (a >> 1), x = 2 * (pp % 7) + (a & 1);
      dch[((y + 2) * 18 + (x + 2)) * kOCP + oc] = f32_to_bf16(g);
    }
  }
  __syncthreads();

  const int wave = tid >> 6, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const int m = wave * 32 + r;
  const int mc = m < 196 ? m : 195;
  const int y = mc / 14, x = mc % 14;
  f32x16 acc = {};
#pragma unroll 4
  for (int s = 0; s < 100; ++s) {
    const int t = s >> 2, ky = t / 5, kx = t % 5, oc0 = (s & 3) * 16 + 8 * h;
    const uint4 a = *reinterpret_cast<const uint4*>(dch + ((y + 4 - ky) * 18 + (x + 4 - kx)) * kOCP + oc0);
    const uint4 bb = *reinterpret_cast<const uint4*>(sw + r * kW2qRow + t * kC2 + oc0);
    acc = mfma32b(a, bb, acc);
  }
  // epilogue: pool1/ReLU backward + conv1 weight gradient for channel c = r
  float dw[kTaps + 1];
#pragma unroll
  for (int t = 0; t < kTaps + 1; ++t) dw[t] = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int pos = wave * 32 + acc_row_b(i, h);
    if (pos < 196) {
      const uint8_t a = am1[(size_t(b) * 196 + pos) * kC1 + r];
      if (a < 4) {
        const float g = acc[i];
        const int yy = 2 * (pos / 14) + (a >> 1), xx = 2 * (pos % 14) + (a & 1);
#pragma unroll
        for (int ky = 0; ky < 5; ++ky)
#pragma unroll
          for (int kx = 0; kx < 5; ++kx) dw[ky * 5 + kx] = fmaf(g, ximg[(yy + ky) * 32 + xx + kx], dw[ky * 5 + kx]);
        dw[kTaps] += g;
      }
    }
  }
#pragma unroll
  for (int t = 0; t < kTaps + 1; ++t) dw[t] += __shfl_xor(dw[t], 32, 64);
  __syncthreads();  // weights no longer needed: reuse their LDS for the wave reduction
  float* red = reinterpret_cast<float*>(smem);  // [7][32][26]
  if (h == 0)
#pragma unroll
    for (int t = 0; t < kTaps + 1; ++t) red[(wave * kC1 + r) * (kTaps + 1) + t] = dw[t];
  __syncthreads();
  for (int e = tid; e < kC1 * (kTaps + 1); e += 448) {
    float sum = 0.f;
#pragma unroll
    for (int w = 0; w < 7; ++w) sum += red[w * kC1 * (kTaps + 1) + e];
    const int c = e / (kTaps + 1), t = e % (kTaps + 1);
    const int o = t < kTaps ? c * kTaps + t : kC1 * kTaps + c;
    wslab1[size_t(b) * kSlab1 + o] = sum;
  }
}

void conv2_dgrad_conv1_wgrad(const float* slabs2, int S2, int mrows, const uint8_t* am2, const uint8_t* am1,
                             const uint16_t* w2q, const uint8_t* x, const int64_t* idx, float* wslab1, int B,
                             hipStream_t s) {
  hipLaunchKernelGGL(conv2_dgrad_kernel, dim3(B), dim3(448), kDgLds, s, slabs2, S2, mrows, am2, am1, w2q, x, idx,
                     wslab1);
}

// ---------------------------------------------------------------------------
// 11. Conv parameters: reduce the per-image gradient slabs, Adam, and repack
//     the conv2 bf16 shadows (W2r for the forward, W2q for the transposed conv).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void conv_adam_kernel(const float* __restrict__ ws1, const float* __restrict__ ws2,
                                                        int B, float* __restrict__ p, float* __restrict__ m,
                                                        float* __restrict__ v, float* __restrict__ gdump,
                                                        uint16_t* __restrict__ w2r, uint16_t* __restrict__ w2q,
                                                        Offsets off, const int* __restrict__ adam_t, AdamCfg cfg,
                                                        int64_t end) {
  const int64_t e = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (e >= end) return;
  const float* slab;
  int stride, j;
  bool is_c2w = false;
  if (e >= off.c1w && e < off.c1w + kC1 * kTaps) {
    slab = ws1; stride = kSlab1; j = int(e - off.c1w);
  } else if (e >= off.c1b && e < off.c1b + kC1) {
    slab = ws1; stride = kSlab1; j = kC1 * kTaps + int(e - off.c1b);
  } else if (e >= off.c2w && e < off.c2w + kC2 * kC1 * kTaps) {
    slab = ws2; stride = kSlab2; j = int(e - off.c2w); is_c2w = true;
  } else if (e >= off.c2b && e < off.c2b + kC2) {
    slab = ws2; stride = kSlab2; j = kC2 * kC1 * kTaps + int(e - off.c2b);
  } else {
    return;  // arena padding
  }
  float g = 0.f;
  for (int b = 0; b < B; ++b) g += slab[size_t(b) * stride + j];
  if (gdump) gdump[e] = g;
  const AdamScal s = adam_scal(cfg, adam_t);
  const float pn = adam_apply(p, m, v, e, g, cfg, s);
  if (is_c2w) {
    const int oc = j / (kC1 * kTaps), rem = j % (kC1 * kTaps), ic = rem / kTaps, t = rem % kTaps;
    const uint16_t hb = f32_to_bf16(pn);
    w2r[(oc * kTaps + t) * kC1 + ic] = hb;
    w2q[(ic * kTaps + t) * kC2 + oc] = hb;
  }
}

void conv_adam(const float* wslab1, const float* wslab2, int B, float* params, float* m, float* v, float* gdump,
               uint16_t* w2r, uint16_t* w2q, Offsets off, const int* adam_t, AdamCfg cfg, hipStream_t s) {
  const int64_t end = off.c2b + kC2;
  hipLaunchKernelGGL(conv_adam_kernel, dim3(int((end + 255) / 256)), dim3(256), 0, s, wslab1, wslab2, B, params, m, v,
                     gdump, w2r, w2q, off, adam_t, cfg, end);
}

void init_fwd_attributes();

// Raise the dynamic-LDS limit of the kernels that stage > 64 KB.  Called once
// (from the bindings) before any HIP-graph capture.
void init_attributes() {
  init_fwd_attributes();
  P2_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(conv2_wgrad_kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, kWgLds));
  P2_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(conv2_dgrad_kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, kDgLds));
}

}  // namespace p2cnn
