// Fused MNIST-CNN training step -- backward kernels with fused Adam epilogues.
// Layouts: see cnn_fwd.hip.  Backward buffers:
//   dH     bf16 [mrows][2048]      dLoss/dH (ReLU mask applied), rows >= B are zero
//   dC2m   bf16 [mrows][64][224]   dC2 map, positions laid out 14 rows x 16 cols
//   dCh    bf16 [mrows][324][64]   dC2 as padded HWC image (18x18 pixels)
//   gB     f32  [mrows][3136]      alive-masked dA1 (conv2 bias gradient terms)
//   W2q    bf16 [32][25][64]       conv2 weight, (ic, tap, oc) -- transposed-conv B operand
//   wslab1 f32  [B][832]           per-image conv1 weight/bias gradients
//   wslab2 f32  [B][51264]         per-image conv2 weight/bias gradients
// Every reduction has a fixed order (no float atomics), so a step is bitwise
// reproducible -- required because Adam amplifies last-bit differences in
// near-zero gradients.  Adam's step count is (*adam_t + t_off): a device base
// plus an offset baked into each launch, so a whole epoch is one HIP graph.
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
P2_DEVICE uint4 pack8(const uint16_t (&v)[8]) {
  uint4 q;
  q.x = uint32_t(v[0]) | (uint32_t(v[1]) << 16);
  q.y = uint32_t(v[2]) | (uint32_t(v[3]) << 16);
  q.z = uint32_t(v[4]) | (uint32_t(v[5]) << 16);
  q.w = uint32_t(v[6]) | (uint32_t(v[7]) << 16);
  return q;
}

struct AdamScal {
  float step_size, inv_sqrt_bc2;
};
P2_DEVICE AdamScal adam_scal(const AdamCfg& c, const int* t, int t_off) {
  const float tt = float(*t + t_off);
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
// 5. FC2 weight/bias gradient + Adam: dW2[c][k] = sum_b dlogits[b][c] H[b][k].
//    20,490 parameters, one thread each, Adam applied in place.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void fc2_wgrad_adam_kernel(const float* __restrict__ dlogits,
                                                             const uint16_t* __restrict__ H, int B,
                                                             float* __restrict__ p, float* __restrict__ m,
                                                             float* __restrict__ v, float* __restrict__ gdump,
                                                             Offsets off, const int* __restrict__ adam_t, int t_off,
                                                             AdamCfg cfg) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  const int nW = kCls * kHid;
  if (e >= nW + kCls) return;
  float g = 0.f;
  int64_t pi;
  if (e < nW) {
    const int c = e / kHid, k = e % kHid;
#pragma unroll 8
    for (int b = 0; b < B; ++b) g = fmaf(dlogits[b * kCls + c], bf16_to_f32(H[size_t(b) * kHid + k]), g);
    pi = off.l2w + e;
  } else {
    const int c = e - nW;
    for (int b = 0; b < B; ++b) g += dlogits[b * kCls + c];
    pi = off.l2b + c;
  }
  if (gdump) gdump[pi] = g;
  const AdamScal s = adam_scal(cfg, adam_t, t_off);
  adam_apply(p, m, v, pi, g, cfg, s);
}

void fc2_wgrad_adam(const float* dlogits, const uint16_t* H, int B, float* params, float* m, float* v, float* gdump,
                    Offsets off, const int* adam_t, int t_off, AdamCfg cfg, hipStream_t s) {
  const int n = kCls * kHid + kCls;
  hipLaunchKernelGGL(fc2_wgrad_adam_kernel, dim3((n + 255) / 256), dim3(256), 0, s, dlogits, H, B, params, m, v,
                     gdump, off, adam_t, t_off, cfg);
}

// ---------------------------------------------------------------------------
// 6. dA1 = dH x W1 on MFMA, pool2/ReLU backward fused into the epilogue.
//    Grid 98 (32 features each), 8 waves splitting K = 2048 in 64-wide groups
//    (same streaming scheme and k permutation as gemm_skinny), reduced in LDS
//    in fixed wave order.  Each output (b, feature) is routed to the argmax of
//    its 2x2 pooling window and all four window positions are written, in
//    both dC2 layouts.
// ---------------------------------------------------------------------------
template <int MT>
__global__ __launch_bounds__(512) void gemm_da1_route_kernel(const uint16_t* __restrict__ dH,
                                                             const uint16_t* __restrict__ w1t,
                                                             const uint8_t* __restrict__ am2, int B,
                                                             uint16_t* __restrict__ dc2m, uint16_t* __restrict__ dch,
                                                             float* __restrict__ gb) {
  __shared__ float red[8 * MT * 1024];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const int n0 = blockIdx.x * 32;
  constexpr int K = kHid, NG = K / 64;
  f32x16 acc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x16{};
  const uint16_t* brow = w1t + size_t(n0 + r) * K + 32 * h;
#pragma unroll
  for (int g = wave; g < NG; g += 8) {
    const int k0 = g * 64;
    uint4 bq[4], aq[MT][4];
#pragma unroll
    for (int q = 0; q < 4; ++q) bq[q] = ld_nt16(brow + k0 + q * 8);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        aq[mt][q] = reinterpret_cast<const uint4*>(dH + size_t(mt * 32 + r) * K + 32 * h + k0)[q];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) acc[mt] = mfma32b(aq[mt][q], bq[q], acc[mt]);
  }
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int i = 0; i < 16; ++i) red[((wave * MT + mt) * 16 + i) * 64 + lane] = acc[mt][i];
  __syncthreads();
  for (int e = tid; e < MT * 1024; e += 512) {
    float g = 0.f;
#pragma unroll
    for (int w = 0; w < 8; ++w) g += red[w * MT * 1024 + e];
    const int mt = e >> 10, i = (e >> 6) & 15, ln = e & 63;
    const int b = mt * 32 + acc_row_b(i, ln >> 5), feat = n0 + (ln & 31);
    if (b >= B) continue;
    const uint8_t a = am2[size_t(b) * kFeat + feat];
    const int oc = feat / 49, pp = feat % 49, py = pp / 7, px = pp % 7;
    gb[size_t(b) * kFeat + feat] = a < 4 ? g : 0.f;
    const uint16_t gv = f32_to_bf16(g);
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const int y = 2 * py + (d >> 1), x = 2 * px + (d & 1);
      const uint16_t v = (d == a) ? gv : uint16_t(0);
      dc2m[(size_t(b) * kC2 + oc) * 224 + y * 16 + x] = v;
      dch[(size_t(b) * 324 + (y + 2) * 18 + (x + 2)) * kC2 + oc] = v;
    }
  }
}

void gemm_da1_route(const uint16_t* dH, const uint16_t* w1t, const uint8_t* am2, int mrows, int B, uint16_t* dc2m,
                    uint16_t* dch, float* gb, hipStream_t s) {
  if (mrows == 32)
    hipLaunchKernelGGL(gemm_da1_route_kernel<1>, dim3(kFeat / 32), dim3(512), 0, s, dH, w1t, am2, B, dc2m, dch, gb);
  else
    hipLaunchKernelGGL(gemm_da1_route_kernel<2>, dim3(kFeat / 32), dim3(512), 0, s, dH, w1t, am2, B, dc2m, dch, gb);
}

// ---------------------------------------------------------------------------
// 7. FC1 weight gradient on MFMA with Adam fused into the epilogue.
//    dW1[n][k] = sum_b dH[b][n] * A1[b][k]  (K = batch).  Grid (25, 64):
//    block = 32 rows of n x 128 columns of k, one 32x32 tile per wave.  The
//    batch-major dH / A1 tiles are transposed through LDS (so no transposed
//    copies live in HBM); the gradient tile never leaves registers: each lane
//    updates W1/m/v for its 16 elements (coalesced 128-B rows), writes the
//    bf16 shadow, and stages the bf16 tile in LDS so W1^T is written as 64-B
//    row segments.
// ---------------------------------------------------------------------------
template <int MR>
__global__ __launch_bounds__(256) void fc1_wgrad_adam_kernel(const uint16_t* __restrict__ dH,
                                                             const uint16_t* __restrict__ a1,
                                                             float* __restrict__ p, float* __restrict__ m,
                                                             float* __restrict__ v, float* __restrict__ gdump,
                                                             uint16_t* __restrict__ w1bf,
                                                             uint16_t* __restrict__ w1tbf, Offsets off,
                                                             const int* __restrict__ adam_t, int t_off, AdamCfg cfg) {
  constexpr int P = MR + 8;  // padded batch pitch (16-B aligned rows, bank spread)
  __shared__ __attribute__((aligned(16))) uint16_t sdh[32][P];    // [n][b]
  __shared__ __attribute__((aligned(16))) uint16_t sa1[128][P];   // [k][b]
  __shared__ __attribute__((aligned(16))) uint16_t tr[128][40];   // bf16 W1 tile for the W1^T write
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const int n0 = blockIdx.y * 32;
  const int kb = blockIdx.x * 128;
  // stage and transpose: dH[b][n0..n0+31] -> sdh[n][b];  A1[b][kb..kb+127] -> sa1[k][b]
  for (int i = tid; i < MR * 4; i += 256) {
    const int b = i >> 2, q = i & 3;
    const uint4 u = reinterpret_cast<const uint4*>(dH + size_t(b) * kHid + n0)[q];
    const uint16_t* e = reinterpret_cast<const uint16_t*>(&u);
#pragma unroll
    for (int j = 0; j < 8; ++j) sdh[q * 8 + j][b] = e[j];
  }
  for (int i = tid; i < MR * 16; i += 256) {
    const int b = i >> 4, q = i & 15;
    const int k = kb + q * 8;
    uint4 u = make_uint4(0, 0, 0, 0);
    if (k < kFeat) u = reinterpret_cast<const uint4*>(a1 + size_t(b) * kFeat + k)[0];
    const uint16_t* e = reinterpret_cast<const uint16_t*>(&u);
#pragma unroll
    for (int j = 0; j < 8; ++j) sa1[q * 8 + j][b] = e[j];
  }
  __syncthreads();
  const int k0 = kb + wave * 32;
  const bool valid = k0 < kFeat;
  f32x16 acc = {};
#pragma unroll
  for (int ks = 0; ks < MR / 16; ++ks) {
    const uint4 a = *reinterpret_cast<const uint4*>(&sdh[r][ks * 16 + 8 * h]);
    const uint4 b = *reinterpret_cast<const uint4*>(&sa1[wave * 32 + r][ks * 16 + 8 * h]);
    acc = mfma32b(a, b, acc);
  }
  const AdamScal s = adam_scal(cfg, adam_t, t_off);
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
    const int k = kb + kl;
    if (k < kFeat)
      *reinterpret_cast<uint4*>(w1tbf + size_t(k) * kHid + n0 + q * 8) = *reinterpret_cast<const uint4*>(&tr[kl][q * 8]);
  }
  if (blockIdx.x == 0 && wave == 0 && lane < 32) {
    const int n = n0 + lane;
    float g = 0.f;
    for (int b = 0; b < MR; ++b) g += bf16_to_f32(sdh[lane][b]);
    if (gdump) gdump[off.l1b + n] = g;
    adam_apply(p, m, v, off.l1b + n, g, cfg, s);
  }
}

void fc1_wgrad_adam(const uint16_t* dH, const uint16_t* a1, int mrows, float* params, float* m, float* v,
                    float* gdump, uint16_t* w1bf, uint16_t* w1tbf, Offsets off, const int* adam_t, int t_off,
                    AdamCfg cfg, hipStream_t s) {
  const dim3 grid((kFeat + 127) / 128, kHid / 32);
  if (mrows == 32)
    hipLaunchKernelGGL(fc1_wgrad_adam_kernel<32>, grid, dim3(256), 0, s, dH, a1, params, m, v, gdump, w1bf, w1tbf,
                       off, adam_t, t_off, cfg);
  else
    hipLaunchKernelGGL(fc1_wgrad_adam_kernel<64>, grid, dim3(256), 0, s, dH, a1, params, m, v, gdump, w1bf, w1tbf,
                       off, adam_t, t_off, cfg);
}

// ---------------------------------------------------------------------------
// 8. conv2 weight gradient on MFMA, per image and tap group.
//    Grid (4, B), 8 waves.  For tap t: C[oc][ic] = sum_pos dC2[oc][pos] *
//    P1pad[ic][pos + tap]; M = 64 oc (2 tiles), N = 32 ic, K = positions laid
//    out 14 rows x 16 (one 16-wide MFMA k-step per image row).  The image is
//    kept as five kx-shifted channel-planar copies ([kx][ic][18 rows][16 cols]),
//    so every B fragment (8 consecutive positions of one channel) is ONE
//    aligned 16-B LDS read; A fragments are 16-B reads of the dC2 map.  The ic
//    pitch (296 elements = 148 dwords) puts a b128 lane group on disjoint
//    banks.  The conv2 bias gradient is a fixed-order wave reduction.
// ---------------------------------------------------------------------------
constexpr int kWgPitch = 18 * 16 + 8;                    // 296 elements per (kx, ic) plane
constexpr int kWgCopies = 5 * kC1 * kWgPitch * 2;        // 94720 B
constexpr int kWgDc2 = kC2 * 224 * 2;                    // 28672 B
constexpr int kWgHwc = 196 * kC1 * 2;                    // 12544 B staging of the HWC image
constexpr int kWgLds = kWgCopies + kWgDc2 + kWgHwc;      // 135936 B

__global__ __launch_bounds__(512) void conv2_wgrad_kernel(const uint16_t* __restrict__ dc2m,
                                                          const float* __restrict__ gb,
                                                          const uint16_t* __restrict__ p1,
                                                          float* __restrict__ wslab) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint16_t* cp = reinterpret_cast<uint16_t*>(smem);
  uint16_t* dc2 = reinterpret_cast<uint16_t*>(smem + kWgCopies);
  uint16_t* hwc = reinterpret_cast<uint16_t*>(smem + kWgCopies + kWgDc2);
  const int b = blockIdx.y, grp = blockIdx.x, tid = threadIdx.x;
  for (int i = tid; i < kWgDc2 / 16; i += 512)
    reinterpret_cast<uint4*>(dc2)[i] = reinterpret_cast<const uint4*>(dc2m + size_t(b) * kC2 * 224)[i];
  for (int i = tid; i < kWgHwc / 16; i += 512)
    reinterpret_cast<uint4*>(hwc)[i] = reinterpret_cast<const uint4*>(p1 + size_t(b) * 196 * kC1)[i];
  __syncthreads();
  // shifted planar copies: cp[kx][ic][yy][c] = P1pad[ic][yy][c + kx], P1pad = P1 zero-padded by 2
  for (int i = tid; i < 5 * kC1 * 18 * 2; i += 512) {
    const int half = i & 1, yy = (i >> 1) % 18, ic = (i / 36) % kC1, kx = i / (36 * kC1);
    uint16_t v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int y = yy - 2, x = half * 8 + j + kx - 2;
      v[j] = (y >= 0 && y < 14 && x >= 0 && x < 14) ? hwc[(y * 14 + x) * kC1 + ic] : uint16_t(0);
    }
    *reinterpret_cast<uint4*>(cp + (kx * kC1 + ic) * kWgPitch + yy * 16 + half * 8) = pack8(v);
  }
  __syncthreads();
  const int wave = tid >> 6, lane = tid & 63, r = lane & 31, h = lane >> 5;
  if (grp == 0) {  // conv2 bias gradient: 8 waves x 8 output channels, 49 terms each
    for (int oc = wave * 8; oc < wave * 8 + 8; ++oc) {
      const float v = wave_sum(lane < 49 ? gb[size_t(b) * kFeat + oc * 49 + lane] : 0.f);
      if (lane == 0) wslab[size_t(b) * kSlab2 + kC2 * kC1 * kTaps + oc] = v;
    }
  }
  const int mt = wave & 1, tw = wave >> 1;
  for (int tj = tw; tj < 7; tj += 4) {
    const int t = grp + 4 * tj;
    if (t >= kTaps) break;
    const int ky = t / 5, kx = t % 5;
    const uint16_t* brow = cp + (kx * kC1 + r) * kWgPitch + ky * 16 + 8 * h;
    const uint16_t* arow = dc2 + (mt * 32 + r) * 224 + 8 * h;
    f32x16 acc = {};
#pragma unroll 7
    for (int ks = 0; ks < 14; ++ks) {
      const uint4 a = *reinterpret_cast<const uint4*>(arow + ks * 16);
      const uint4 bq = *reinterpret_cast<const uint4*>(brow + ks * 16);
      acc = mfma32b(a, bq, acc);
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int oc = mt * 32 + acc_row_b(i, h);
      wslab[size_t(b) * kSlab2 + (oc * kC1 + r) * kTaps + t] = acc[i];
    }
  }
}

void conv2_wgrad(const uint16_t* dc2m, const float* gb, const uint16_t* p1, float* wslab, int B, hipStream_t s) {
  hipLaunchKernelGGL(conv2_wgrad_kernel, dim3(4, B), dim3(512), kWgLds, s, dc2m, gb, p1, wslab);
}

// ---------------------------------------------------------------------------
// 9. conv2 input gradient (transposed conv on MFMA) + pool1/ReLU backward +
//    conv1 weight gradient (second MFMA GEMM), one block per image, 7 waves.
//    Phase 1: C[pos][ic] = sum_{tap,oc} dC2pad[pos - tap][oc] * W2[oc][ic][tap]
//      (K = 25 x 64 = 100 k-steps; A from the padded HWC dC2 image, B from the
//      (ic, tap, oc) weight copy; both 16-B LDS reads, conflict-free pitches).
//    Phase 2: the dP1 tile is routed through the pool1 argmax into a dense dC1
//      map [32 ch][28 rows][32 cols] in LDS, then
//      dW1[c][tap] = sum_pos dC1[c][pos] * Xpad[pos + tap] runs as a 32x32
//      MFMA GEMM over 896 positions, with five kx-shifted bf16 copies of the
//      input image giving aligned 16-B B fragments.  Bias gradient and the
//      cross-wave sums are fixed-order LDS reductions (no float atomics).
// ---------------------------------------------------------------------------
constexpr int kW2qRow = kTaps * kC2 + 8;            // 1608 elements per ic (pad breaks bank aliasing)
constexpr int kDgW = kC1 * kW2qRow * 2;             // 102912
constexpr int kOCP = 72;                            // dC2 pixel stride (144 B)
constexpr int kDgDc2 = 18 * 18 * kOCP * 2;          // 46656
constexpr int kDgLds = kDgW + kDgDc2;               // 149568
constexpr int kDc1Pitch = 28 * 32 + 8;              // 904 elements per channel
constexpr int kDgDc1 = kC1 * kDc1Pitch * 2;         // 57856
constexpr int kXsPitch = 32 * 32;                   // per-kx copy [32 rows][32 cols]
constexpr int kDgXs = 5 * kXsPitch * 2;             // 10240
constexpr int kDgBias = 7 * kC1 * 4;                // 896
static_assert(kDgDc1 + kDgXs + kDgBias <= kDgW, "phase-2 LDS carve exceeds the weight region");

__global__ __launch_bounds__(448) void conv2_dgrad_kernel(const uint16_t* __restrict__ dchg,
                                                          const uint8_t* __restrict__ am1,
                                                          const uint16_t* __restrict__ w2q,
                                                          const uint8_t* __restrict__ xds,
                                                          const int64_t* __restrict__ idx,
                                                          float* __restrict__ wslab1) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint16_t* sw = reinterpret_cast<uint16_t*>(smem);
  uint16_t* dch = reinterpret_cast<uint16_t*>(smem + kDgW);
  const int b = blockIdx.x, tid = threadIdx.x;
  const uint4 z4 = make_uint4(0, 0, 0, 0);
  for (int i = tid; i < kC1 * (kTaps * kC2 / 8); i += 448) {
    const int ic = i / (kTaps * kC2 / 8), q = i % (kTaps * kC2 / 8);
    *reinterpret_cast<uint4*>(sw + ic * kW2qRow + q * 8) =
        reinterpret_cast<const uint4*>(w2q + size_t(ic) * kTaps * kC2)[q];
  }
  for (int i = tid; i < 324 * 8; i += 448) {  // padded HWC dC2 image, 64 ch per pixel (8 x 16 B)
    const int pix = i >> 3, q = i & 7;
    *reinterpret_cast<uint4*>(dch + pix * kOCP + q * 8) =
        reinterpret_cast<const uint4*>(dchg + (size_t(b) * 324 + pix) * kC2)[q];
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
  __syncthreads();  // weights and dC2 are dead: carve phase-2 buffers out of the weight region
  uint16_t* dc1 = reinterpret_cast<uint16_t*>(smem);
  uint16_t* xs = reinterpret_cast<uint16_t*>(smem + kDgDc1);
  float* bsum_w = reinterpret_cast<float*>(smem + kDgDc1 + kDgXs);  // [7 waves][32 ch]
  for (int i = tid; i < kDgDc1 / 16; i += 448) reinterpret_cast<uint4*>(dc1)[i] = z4;
  const int64_t row = idx ? idx[b] : b;
  const uint8_t* src = xds + row * (kImg * kImg);
  for (int i = tid; i < 5 * 32 * 4; i += 448) {  // xs[kx][yy][c] = Xpad[yy][c + kx], 8 columns per item
    const int q = i & 3, yy = (i >> 2) & 31, kx = i >> 7;
    uint16_t v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int sy = yy - 2, sx = q * 8 + j + kx - 2;
      v[j] = (sy >= 0 && sy < kImg && sx >= 0 && sx < kImg) ? f32_to_bf16(float(src[sy * kImg + sx]) * (1.f / 255.f))
                                                           : uint16_t(0);
    }
    *reinterpret_cast<uint4*>(xs + kx * kXsPitch + yy * 32 + q * 8) = pack8(v);
  }
  __syncthreads();
  float bsum = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int pos = wave * 32 + acc_row_b(i, h);
    if (pos < 196) {
      const uint8_t a = am1[(size_t(b) * 196 + pos) * kC1 + r];
      if (a < 4) {
        const int yy = 2 * (pos / 14) + (a >> 1), xx = 2 * (pos % 14) + (a & 1);
        dc1[r * kDc1Pitch + yy * 32 + xx] = f32_to_bf16(acc[i]);
        bsum += acc[i];
      }
    }
  }
  bsum += __shfl_xor(bsum, 32, 64);
  if (h == 0) bsum_w[wave * kC1 + r] = bsum;
  __syncthreads();
  // conv1 weight gradient: C[c][tap] over K = 28 rows x 32 cols of positions
  // (56 k-steps); waves split K, partial tiles reduced in fixed order.
  f32x16 wacc = {};
  const int t = r < kTaps ? r : kTaps - 1;  // lanes 25..31 compute a duplicate column, discarded
  const int ky = t / 5, kx = t % 5;
  for (int ks = wave; ks < 56; ks += 7) {
    const int yy = ks >> 1, x0 = (ks & 1) * 16 + 8 * h;
    const uint4 a = *reinterpret_cast<const uint4*>(dc1 + r * kDc1Pitch + yy * 32 + x0);
    const uint4 bq = *reinterpret_cast<const uint4*>(xs + kx * kXsPitch + (yy + ky) * 32 + x0);
    wacc = mfma32b(a, bq, wacc);
  }
  float* red = reinterpret_cast<float*>(smem + kDgW);  // [7 waves][16 regs][64 lanes] f32 = 28672 B
#pragma unroll
  for (int i = 0; i < 16; ++i) red[(wave * 16 + i) * 64 + lane] = wacc[i];
  __syncthreads();
  for (int e = tid; e < 16 * 64; e += 448) {
    float sum = 0.f;
#pragma unroll
    for (int w = 0; w < 7; ++w) sum += red[w * 1024 + e];
    const int i = e >> 6, ln = e & 63;
    const int c = acc_row_b(i, ln >> 5), tt = ln & 31;
    if (tt < kTaps) wslab1[size_t(b) * kSlab1 + c * kTaps + tt] = sum;
  }
  if (tid < kC1) {
    float sb = 0.f;
#pragma unroll
    for (int w = 0; w < 7; ++w) sb += bsum_w[w * kC1 + tid];
    wslab1[size_t(b) * kSlab1 + kC1 * kTaps + tid] = sb;
  }
}

void conv2_dgrad_conv1_wgrad(const uint16_t* dch, const uint8_t* am1, const uint16_t* w2q, const uint8_t* x,
                             const int64_t* idx, float* wslab1, int B, hipStream_t s) {
  hipLaunchKernelGGL(conv2_dgrad_kernel, dim3(B), dim3(448), kDgLds, s, dch, am1, w2q, x, idx, wslab1);
}

// ---------------------------------------------------------------------------
// 10. Conv parameters: reduce the per-image gradient slabs, Adam, and repack
//     the conv2 bf16 shadows (W2r for the forward, W2q for the transposed conv).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void conv_adam_kernel(const float* __restrict__ ws1, const float* __restrict__ ws2,
                                                        int B, float* __restrict__ p, float* __restrict__ m,
                                                        float* __restrict__ v, float* __restrict__ gdump,
                                                        uint16_t* __restrict__ w2r, uint16_t* __restrict__ w2q,
                                                        Offsets off, const int* __restrict__ adam_t, int t_off,
                                                        AdamCfg cfg, int64_t end) {
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
#pragma unroll 8
  for (int b = 0; b < B; ++b) g += slab[size_t(b) * stride + j];
  if (gdump) gdump[e] = g;
  const AdamScal s = adam_scal(cfg, adam_t, t_off);
  const float pn = adam_apply(p, m, v, e, g, cfg, s);
  if (is_c2w) {
    const int oc = j / (kC1 * kTaps), rem = j % (kC1 * kTaps), ic = rem / kTaps, t = rem % kTaps;
    const uint16_t hb = f32_to_bf16(pn);
    w2r[(oc * kTaps + t) * kC1 + ic] = hb;
    w2q[(ic * kTaps + t) * kC2 + oc] = hb;
  }
}

void conv_adam(const float* wslab1, const float* wslab2, int B, float* params, float* m, float* v, float* gdump,
               uint16_t* w2r, uint16_t* w2q, Offsets off, const int* adam_t, int t_off, AdamCfg cfg, hipStream_t s) {
  const int64_t end = off.c2b + kC2;
  hipLaunchKernelGGL(conv_adam_kernel, dim3(int((end + 255) / 256)), dim3(256), 0, s, wslab1, wslab2, B, params, m, v,
                     gdump, w2r, w2q, off, adam_t, t_off, cfg, end);
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
