// Fused MNIST-CNN training step -- forward kernels (see cnn.h for the pipeline).
//
// Layouts (all bf16 activations are raw uint16 bit patterns):
//   x    uint8  [N][28*28]           dataset, gathered by idx[b] (the /255 is folded in)
//   P1   bf16   [B][196][32]         pooled conv1 output, HWC (channels contiguous)
//   AM1  uint8  [B][196][32]         pool1 argmax (dy*2+dx) or 4 = dead (ReLU zero)
//   P1s  bf16   [B][5][32][18][16]   kx-shifted planar copies of zero-padded P1 (training
//                                    only): P1s[b][kx][ic][yy][c] = P1pad[ic][yy][c + kx],
//                                    the conv2-wgrad B operand as aligned 16-B rows
//   A1   bf16   [mrows][3136]        pooled conv2 output, PyTorch flatten order c*49+y*7+x
//   AM2  uint8  [B][3136]            pool2 argmax / dead
//   W2r  bf16   [64][25][32]         conv2 weight, (oc, tap, ic)   -- conv2_fwd B operand
//   W1bf bf16   [2048][3136]         FC1 weight (row-major = [N][K]) -- FC1 forward
//   W1T  bf16   [3136][2048]         FC1 weight transposed          -- dA1 = dH W1
// MFMA: v_mfma_f32_32x32x16_bf16.  Lane l (r = l & 31, h = l >> 5) supplies
// A[row r][k = 8h + j] and B[k = 8h + j][col r], j = 0..7; the accumulator
// register i of lane l holds C[row (i&3) + 8(i>>2) + 4h][col r].
#include <cstdlib>

#include "cnn.h"
#include "cnn_fwd_dev.h"
#include "common.h"

namespace p2cnn {
using namespace p2;

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

P2_DEVICE bf16x8_t as_bf16x8(uint4 v) { return __builtin_bit_cast(bf16x8_t, v); }
P2_DEVICE f32x16 mfma32(uint4 a, uint4 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(a), as_bf16x8(b), c, 0, 0, 0);
}
P2_DEVICE int acc_row(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

// ---------------------------------------------------------------------------
// 2. conv1 (1->32, 5x5, pad 2) + bias + ReLU + maxpool 2x2.  Grid (7, B):
//    block q of image b produces pooled rows 2q and 2q+1 (28 positions x 32
//    oc).  oc = tid & 31 is fixed per thread, so its 25 taps live in
//    registers; the 6x6 input window of a pooled output is read from LDS
//    (broadcast to the 32 oc lanes).  Results are staged in LDS and written
//    as whole 16-B chunks: P1 (HWC), AM1, and -- when training -- the two
//    rows of all five kx-shifted planar copies (P1s) this block owns,
//    including their zero padding columns.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void conv1_fwd_kernel(const uint8_t* __restrict__ x, const int64_t* __restrict__ idx,
                                                        const float* __restrict__ w1, const float* __restrict__ b1,
                                                        uint16_t* __restrict__ p1, uint8_t* __restrict__ am1,
                                                        uint16_t* __restrict__ p1s) {
  __shared__ Conv1Smem sm;
  conv1_body<false>(blockIdx.x, blockIdx.y, x, idx, w1, b1, p1, am1, p1s, sm);
}

void conv1_fwd(const uint8_t* x, const int64_t* idx, const float* params, Offsets off, uint16_t* p1, uint8_t* am1,
               uint16_t* p1s, int B, hipStream_t s) {
  hipLaunchKernelGGL(conv1_fwd_kernel, dim3(7, B), dim3(256), 0, s, x, idx, params + off.c1w, params + off.c1b, p1,
                     am1, p1s);
}

// ---------------------------------------------------------------------------
// 3. conv2 (32->64, 5x5, pad 2) as implicit GEMM on MFMA + bias/ReLU/maxpool.
//    Grid (7, 2, B): one wave per (pooled row, oc half, image) -- 448 waves,
//    so the whole chip is busy.  GEMM M = the 28 conv positions of two conv
//    rows (= one pooled row; lanes 28..31 duplicate a valid row and are
//    discarded), N = 32 oc, K = 25 taps x 32 ic with ic fastest: every A
//    fragment is one 16-B load of an HWC pixel (zero outside the image), every
//    B fragment one 16-B load of the (oc, tap, ic) weight copy, both straight
//    from L2/L1 -- no LDS staging.  Loads run one 5-tap chunk ahead of the
//    MFMAs (explicit double buffer; sched barriers stop the compiler from
//    serialising them).  The 2x2 pool is an exchange through 4 KB of LDS.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void conv2_fwd_kernel(const uint16_t* __restrict__ p1,
                                                       const uint16_t* __restrict__ w2r,
                                                       const float* __restrict__ b2, uint16_t* __restrict__ a1,
                                                       uint8_t* __restrict__ am2) {
  __shared__ float sout[32][33];
  conv2_body<false>(true, blockIdx.x, blockIdx.y, blockIdx.z, threadIdx.x, p1, w2r, b2, a1, am2, sout);
}

// Same conv2, LDS-staged: one 7-wave block per (oc half, image).  The kernel
// above streams every operand fragment from L2 per wave -- 50 KB of P1 pixels
// and 50 KB of weights for each of its 448 waves, ~175 KB per CU -- and is bound
// by what one CU can fetch (~11 B/cycle/CU, MI355X_MICROARCH.md).  Here the
// block copies the image's P1 (12.25 KB) and its 32 oc rows of the weight
// (50 KB) into LDS once (global_load_lds), and its 7 waves (pooled rows) read
// every fragment from LDS: ~62 KB fetched per block.  Same k order, MFMA
// sequence and pool epilogue as the streaming kernel (bitwise-equal results).
constexpr int kC2P1 = 196 * kC1 * 2;            // 12544 B
constexpr int kC2W = 32 * kTaps * kC1 * 2;      // 51200 B
constexpr int kC2Out = 7 * 32 * 33 * 4;         // per-wave pool exchange, 29568 B
constexpr int kC2Lds = kC2P1 + kC2W + kC2Out;   // 93312 B

P2_DEVICE void glds_copy_n(const uint16_t* src, char* dst, int bytes, int wave, int nwaves, int lane) {
  // 1 KB per wave instruction (64 lanes x 16 B); a partial last chunk masks lanes
  for (int c = wave; c * 1024 < bytes; c += nwaves)
    if (c * 1024 + lane * 16 < bytes)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + c * 512 + lane * 8),
                                       (__attribute__((address_space(3))) void*)(dst + c * 1024), 16, 0, 0);
}

__global__ __launch_bounds__(448) void conv2_fwd_lds_kernel(const uint16_t* __restrict__ p1,
                                                            const uint16_t* __restrict__ w2r,
                                                            const float* __restrict__ b2, uint16_t* __restrict__ a1,
                                                            uint8_t* __restrict__ am2) {
  __shared__ __attribute__((aligned(16))) char smem[kC2Lds];
  const int nh = blockIdx.x, b = blockIdx.y;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int py = wave;
  glds_copy_n(p1 + size_t(b) * 196 * kC1, smem, kC2P1, wave, 7, lane);
  glds_copy_n(w2r + size_t(nh * 32) * kTaps * kC1, smem + kC2P1, kC2W, wave, 7, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const uint16_t* img = reinterpret_cast<const uint16_t*>(smem) + 8 * h;
  const uint16_t* wrow = reinterpret_cast<const uint16_t*>(smem + kC2P1) + r * kTaps * kC1 + 8 * h;
  float(*sout)[33] = reinterpret_cast<float(*)[33]>(smem + kC2P1 + kC2W + wave * (32 * 33 * 4));
  const int rr = r < 28 ? r : 27;
  const int y = 2 * py + (rr >= 14 ? 1 : 0), x = rr >= 14 ? rr - 14 : rr;
  const uint4 z4 = make_uint4(0, 0, 0, 0);
  f32x16 acc = {};
#pragma unroll 10
  for (int s = 0; s < 50; ++s) {
    const int t = s >> 1, ky = t / 5, kx = t % 5, ic = (s & 1) * 16;
    const int iy = y + ky - 2, ix = x + kx - 2;
    const bool ok = iy >= 0 && iy < 14 && ix >= 0 && ix < 14;
    const uint4 v = *reinterpret_cast<const uint4*>(img + (ok ? iy * 14 + ix : 0) * kC1 + ic);
    const uint4 bq = *reinterpret_cast<const uint4*>(wrow + t * kC1 + ic);
    acc = mfma32(ok ? v : z4, bq, acc);
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int row = acc_row(i, h);
    if (row < 28) sout[row][r] = acc[i];
  }
  __syncthreads();
  for (int e = lane; e < 7 * 32; e += 64) {
    const int oc = e / 7, px = e % 7;
    const float v[4] = {sout[2 * px][oc], sout[2 * px + 1][oc], sout[14 + 2 * px][oc], sout[15 + 2 * px][oc]};
    float best = v[0];
    int arg = 0;
#pragma unroll
    for (int d = 1; d < 4; ++d)
      if (v[d] > best) {
        best = v[d];
        arg = d;
      }
    best += b2[nh * 32 + oc];
    const size_t o = size_t(b) * kFeat + (nh * 32 + oc) * 49 + py * 7 + px;
    a1[o] = f32_to_bf16(fmaxf(best, 0.f));
    am2[o] = best > 0.f ? uint8_t(arg) : uint8_t(4);
  }
}

// ---------------------------------------------------------------------------
// 2+3. conv1 + conv2 in one launch.  Grid (7, B), 256 threads.  Block q of image
//    b computes the pooled conv1 rows that conv2's pooled row q reads -- P1 rows
//    2q-2 .. 2q+3, clipped to the image -- into an LDS window (HWC), with
//    conv1_fwd_kernel's fp32 arithmetic in the same order (bitwise-equal values).
//    Waves 0 and 1 then run conv2_fwd_kernel's MFMA sequence for (row q, oc half =
//    wave), A fragments from the window instead of from global P1 (bitwise-equal
//    A1), while waves 2 and 3 write AM1 / P1s (and P1 if asked) of the block's own
//    rows 2q, 2q+1 -- what conv1_fwd_kernel block q writes.  The rows 2q +- 2 are
//    also computed by the neighbouring blocks (3x conv1's VALU work); in exchange
//    there is no P1 round trip through L2 and no second launch.  Measured arm,
//    opt-in (learning/fused_cnn.py P2PFL_CNN_CONV12=1): 16.3 us against conv1 4.6 +
//    conv2 6.0 us as two kernels (scripts/kbench.py, round 6) -- the recomputed
//    rows put ~10 us of serial VALU work in front of every block's conv2.
// ---------------------------------------------------------------------------
constexpr int kWinRows = 6;  // P1 rows 2q-2 .. 2q+3

__global__ __launch_bounds__(256) void conv12_fwd_kernel(const uint8_t* __restrict__ x,
                                                         const int64_t* __restrict__ idx, const float* __restrict__ w1,
                                                         const float* __restrict__ b1, const uint16_t* __restrict__ w2r,
                                                         const float* __restrict__ b2, uint16_t* __restrict__ p1,
                                                         uint8_t* __restrict__ am1, uint16_t* __restrict__ p1s,
                                                         uint16_t* __restrict__ a1, uint8_t* __restrict__ am2) {
  __shared__ float img[16][33];                                        // input rows 4q-6 .. 4q+9, padded
  __shared__ __attribute__((aligned(16))) uint16_t win[kWinRows * 14 * kC1];  // P1 window, [row][px][ic]
  __shared__ uint16_t sv[kC1][2][16];                                  // own rows, [oc][row][px], cols 14/15 zero
  __shared__ __attribute__((aligned(16))) uint8_t sa[28][kC1];         // own rows' argmax codes [pos][oc]
  __shared__ float sout[2][32][33];                                    // conv2 pool exchange, per wave
  const int b = blockIdx.y, q = blockIdx.x, tid = threadIdx.x;
  const int64_t row = idx ? idx[b] : b;
  const uint8_t* src = x + row * (kImg * kImg);
  for (int i = tid; i < 16 * 32; i += 256) {
    const int yy = i >> 5, xx = i & 31, sy = 4 * q - 6 + yy, sx = xx - 2;
    float v = 0.f;
    if (sy >= 0 && sy < kImg && sx >= 0 && sx < kImg) v = float(src[sy * kImg + sx]) * (1.f / 255.f);
    img[yy][xx] = v;
  }
  const int oc = tid & 31;
  float w[kTaps];
#pragma unroll
  for (int t = 0; t < kTaps; ++t) w[t] = w1[oc * kTaps + t];
  const float bias = b1[oc];
  if (tid < kC1 * 2 * 2) sv[tid >> 2][(tid >> 1) & 1][14 + (tid & 1)] = 0;
  __syncthreads();
  // conv1: 6 window rows x 14 pooled columns per oc; rows outside the image stay zero
  for (int k = tid >> 5; k < kWinRows * 14; k += 8) {
    const int wr = k / 14, px = k % 14, prow = 2 * q - 2 + wr;
    uint16_t out = 0;
    if (prow >= 0 && prow < 14) {
      float wv[6][6];
#pragma unroll
      for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int j = 0; j < 6; ++j) wv[i][j] = img[2 * wr + i][2 * px + j];
      float best = -3.4e38f;
      int arg = 0;
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const int dy = d >> 1, dx = d & 1;
        float sacc = bias;
#pragma unroll
        for (int ky = 0; ky < 5; ++ky)
#pragma unroll
          for (int kx = 0; kx < 5; ++kx) sacc = fmaf(w[ky * 5 + kx], wv[dy + ky][dx + kx], sacc);
        if (sacc > best) {
          best = sacc;
          arg = d;
        }
      }
      out = f32_to_bf16(fmaxf(best, 0.f));
      if (wr == 2 || wr == 3) {  // this block's own rows: AM1 / P1 / P1s come from here
        sv[oc][wr - 2][px] = out;
        sa[(wr - 2) * 14 + px][oc] = best > 0.f ? uint8_t(arg) : uint8_t(4);
      }
    }
    win[k * kC1 + oc] = out;
  }
  __syncthreads();
  const int wave = tid >> 6, lane = tid & 63;
  if (wave < 2) {
    // conv2 for pooled row q, oc half `wave`: conv2_fwd_kernel's loads and MFMA order
    const int nh = wave, r = lane & 31, h = lane >> 5;
    const int rr = r < 28 ? r : 27;
    const int y = 2 * q + (rr >= 14 ? 1 : 0), xq = rr >= 14 ? rr - 14 : rr;
    const uint16_t* wl = win + 8 * h;
    const uint16_t* wrow = w2r + size_t(nh * 32 + r) * kTaps * kC1 + 8 * h;
    const uint4 z4 = make_uint4(0, 0, 0, 0);
    auto load = [&](int c, uint4 (&A)[10], uint4 (&Bv)[10]) {
#pragma unroll
      for (int j = 0; j < 10; ++j) {
        const int st = c * 10 + j, t = st >> 1, ky = t / 5, kx = t % 5, ic = (st & 1) * 16;
        const int iy = y + ky - 2, ix = xq + kx - 2;
        const bool ok = iy >= 0 && iy < 14 && ix >= 0 && ix < 14;
        const int pix = ok ? (iy - 2 * q + 2) * 14 + ix : 0;
        const uint4 v = *reinterpret_cast<const uint4*>(wl + pix * kC1 + ic);
        A[j] = ok ? v : z4;
        Bv[j] = *reinterpret_cast<const uint4*>(wrow + t * kC1 + ic);
      }
    };
    uint4 A0[10], B0[10], A1[10], B1[10];
    f32x16 acc = {};
    load(0, A0, B0);
#pragma unroll
    for (int c = 0; c < 5; c += 2) {
      if (c + 1 < 5) load(c + 1, A1, B1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < 10; ++j) acc = mfma32(A0[j], B0[j], acc);
      __builtin_amdgcn_sched_barrier(0);
      if (c + 1 < 5) {
        if (c + 2 < 5) load(c + 2, A0, B0);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < 10; ++j) acc = mfma32(A1[j], B1[j], acc);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int rw = acc_row(i, h);
      if (rw < 28) sout[nh][rw][r] = acc[i];
    }
  } else {
    // conv1_fwd_kernel's stores of rows 2q, 2q+1 (threads 0..127 of waves 2-3)
    const int t2 = tid - 128;
    const size_t pix0 = size_t(b) * 196 + q * 28;
    if (p1 && t2 < 28 * 4) {
      const int k = t2 >> 2, c0 = (t2 & 3) * 8;
      uint16_t u[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) u[j] = sv[c0 + j][k / 14][k % 14];
      uint4 o;
      o.x = uint32_t(u[0]) | (uint32_t(u[1]) << 16);
      o.y = uint32_t(u[2]) | (uint32_t(u[3]) << 16);
      o.z = uint32_t(u[4]) | (uint32_t(u[5]) << 16);
      o.w = uint32_t(u[6]) | (uint32_t(u[7]) << 16);
      reinterpret_cast<uint4*>(p1 + (pix0 + k) * kC1)[t2 & 3] = o;
    }
    if (t2 < 28 * 2) {
      const int k = t2 >> 1, c0 = (t2 & 1) * 16;
      reinterpret_cast<uint4*>(am1 + (pix0 + k) * kC1)[t2 & 1] = *reinterpret_cast<const uint4*>(&sa[k][c0]);
    }
    if (p1s) {
      for (int i = t2; i < 5 * kC1 * 2 * 2; i += 128) {
        const int half = i & 1, rr2 = (i >> 1) & 1, o = (i >> 2) % kC1, kx = i / (4 * kC1);
        uint16_t u[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int xs = half * 8 + j + kx - 2;
          u[j] = (xs >= 0 && xs < 14) ? sv[o][rr2][xs] : uint16_t(0);
        }
        uint4 v;
        v.x = uint32_t(u[0]) | (uint32_t(u[1]) << 16);
        v.y = uint32_t(u[2]) | (uint32_t(u[3]) << 16);
        v.z = uint32_t(u[4]) | (uint32_t(u[5]) << 16);
        v.w = uint32_t(u[6]) | (uint32_t(u[7]) << 16);
        *reinterpret_cast<uint4*>(p1s + ((size_t(b) * 5 + kx) * kC1 + o) * kP1sPlane + (2 * q + rr2 + 2) * 16 + half * 8) = v;
      }
    }
  }
  __syncthreads();
  // conv2's bias + ReLU + 2x2 pool of both oc halves (conv2_fwd_kernel's epilogue)
  for (int e = tid; e < 2 * 7 * 32; e += 256) {
    const int nh = e / 224, ocx = (e % 224) / 7, px = e % 7;
    const float v[4] = {sout[nh][2 * px][ocx], sout[nh][2 * px + 1][ocx], sout[nh][14 + 2 * px][ocx],
                        sout[nh][15 + 2 * px][ocx]};
    float best = v[0];
    int arg = 0;
#pragma unroll
    for (int d = 1; d < 4; ++d)
      if (v[d] > best) {
        best = v[d];
        arg = d;
      }
    best += b2[nh * 32 + ocx];
    const size_t o = size_t(b) * kFeat + (nh * 32 + ocx) * 49 + q * 7 + px;
    a1[o] = f32_to_bf16(fmaxf(best, 0.f));
    am2[o] = best > 0.f ? uint8_t(arg) : uint8_t(4);
  }
}

void conv12_fwd(const uint8_t* x, const int64_t* idx, const float* params, Offsets off, const uint16_t* w2r,
                uint16_t* p1, uint8_t* am1, uint16_t* p1s, uint16_t* a1, uint8_t* am2, int B, hipStream_t s) {
  hipLaunchKernelGGL(conv12_fwd_kernel, dim3(7, B), dim3(256), 0, s, x, idx, params + off.c1w, params + off.c1b, w2r,
                     params + off.c2b, p1, am1, p1s, a1, am2);
}

void init_fwd_attributes() {}

void conv2_fwd(const uint16_t* p1, const uint16_t* w2r, const float* params, Offsets off, uint16_t* a1,
               uint8_t* am2, int B, hipStream_t s) {
  // P2CNN_CONV2_FWD_LDS=1: the LDS-staged kernel -- measured slower, 8.2 vs 6.0 us
  // (scripts/kbench.py, round 4): staging everything before the first MFMA
  // serialises what the 448 streaming waves overlap.  Kept as a measured arm.
  static const bool lds = [] {
    const char* e = getenv("P2CNN_CONV2_FWD_LDS");
    return e && atoi(e) != 0;
  }();
  // ... but at the evaluation passes' 128-image launches the staged copy is reused by
  // 7 waves x 2 blocks per image and wins: 9.2 vs 14.1 us (scripts/eval_fwd_probe.py)
  if (lds || B > 64)
    hipLaunchKernelGGL(conv2_fwd_lds_kernel, dim3(2, B), dim3(448), 0, s, p1, w2r, params + off.c2b, a1, am2);
  else
    hipLaunchKernelGGL(conv2_fwd_kernel, dim3(7, 2, B), dim3(64), 0, s, p1, w2r, params + off.c2b, a1, am2);
}

// ---------------------------------------------------------------------------
// 4/7. Skinny GEMM  slabs[s][m][n] = sum_{k in split s} A[m][k] * Bt[n][k]
//    (M = mrows = 32*MT rows, MT = 1, 2, 4; N multiple of 32, K multiple of 64).  Block =
//    32 output columns x one K split; its 4 waves take interleaved 64-wide K
//    groups.  Each lane streams 64 contiguous bytes of an A row and of a Bt row
//    per group (the two half-waves cover a full 128-B line), and the group's
//    four 16-wide MFMA k-steps consume them with the SAME k permutation on both
//    operands, so no shuffles are needed.  Waves reduce through LDS; one fp32
//    slab per split keeps the result deterministic.
// ---------------------------------------------------------------------------
// XA (XCD-aligned split layout, S <= 8): a 1-D grid of 8 x N/32 blocks; block b
// runs on XCD b % 8 (round-robin dispatch) and takes K split b % 8, column tile
// b / 8 (blocks of XCDs >= S exit), so XCD s reads -- through its own L2, plain
// loads -- exactly the W1 columns of split s: the feature columns the dA1 routing
// blocks on XCD s read next (route_rm_kernel, same alignment), from that L2
// instead of from the Infinity Cache.
template <int MT, bool XA>
__global__ __launch_bounds__(256) void gemm_skinny_kernel(const uint16_t* __restrict__ A,
                                                          const uint16_t* __restrict__ Bt, float* __restrict__ slabs,
                                                          int N, int K, int S) {
  constexpr int RT = MT < 2 ? MT : 2;  // row tiles reduced per LDS pass (<= 32 KB)
  __shared__ float red[4 * RT * 16 * 64];
  const int nt = XA ? int(blockIdx.x >> 3) : int(blockIdx.x), sp = XA ? int(blockIdx.x & 7) : int(blockIdx.y);
  if (XA && sp >= S) return;
  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const int n0 = nt * 32;
  const int ng = K / 64, gps = (ng + S - 1) / S;
  const int g0 = sp * gps, g1 = min(ng, g0 + gps);
  f32x16 acc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x16{};
  const uint16_t* brow = Bt + size_t(n0 + r) * K + 32 * h;
  const uint16_t* arow[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) arow[mt] = A + size_t(mt * 32 + r) * K + 32 * h;
  // software pipeline: the next group's 16-B loads are in flight while the
  // current group's MFMAs run
  uint4 bq[4], aq[MT][4];
  int g = g0 + wave;
  auto load = [&](int gg, uint4 (&bb)[4], uint4 (&aa)[MT][4]) {
    const int k0 = gg * 64;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      bb[q] = XA ? reinterpret_cast<const uint4*>(brow + k0)[q] : ld_nt16(brow + k0 + q * 8);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int q = 0; q < 4; ++q) aa[mt][q] = reinterpret_cast<const uint4*>(arow[mt] + k0)[q];
  };
  if (g < g1) load(g, bq, aq);
  for (; g < g1; g += 4) {
    uint4 nb[4], na[MT][4];
    const bool more = g + 4 < g1;
    if (more) load(g + 4, nb, na);
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) acc[mt] = mfma32(aq[mt][q], bq[q], acc[mt]);
    if (more) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        bq[q] = nb[q];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) aq[mt][q] = na[mt][q];
      }
    }
  }
  const int mrows = MT * 32;
#pragma unroll
  for (int m0 = 0; m0 < MT; m0 += RT) {
    if (m0) __syncthreads();  // previous pass's reads done
#pragma unroll
    for (int mt = 0; mt < RT; ++mt)
#pragma unroll
      for (int i = 0; i < 16; ++i) red[((wave * RT + mt) * 16 + i) * 64 + lane] = acc[m0 + mt][i];
    __syncthreads();
    for (int e = tid; e < RT * 1024; e += 256) {
      const float sum = red[e] + red[RT * 1024 + e] + red[2 * RT * 1024 + e] + red[3 * RT * 1024 + e];
      const int mt = m0 + (e >> 10), i = (e >> 6) & 15, ln = e & 63;
      const int row = mt * 32 + acc_row(i, ln >> 5), col = ln & 31;
      slabs[(size_t(sp) * mrows + row) * N + n0 + col] = sum;
    }
  }
}

// P2CNN_XCD_ALIGN=0: the skinny GEMM's (column tile, split) grid and the routing
// kernel's XCD-local tile runs, without the shared split <-> XCD layout
bool xcd_align() {
  static const bool on = [] {
    const char* e = getenv("P2CNN_XCD_ALIGN");
    return !(e && e[0] == '0');
  }();
  return on;
}

void gemm_skinny(const uint16_t* A, const uint16_t* Bt, float* slabs, int mrows, int N, int K, int S, hipStream_t s) {
#define P2_SKINNY(MT, XA, GRID) hipLaunchKernelGGL((gemm_skinny_kernel<MT, XA>), GRID, dim3(256), 0, s, A, Bt, slabs, N, K, S)
  if (xcd_align() && S == kXcdSplits && N == kHid && K == kFeat) {
    const dim3 grid(8 * (N / 32));
    if (mrows == 32) P2_SKINNY(1, true, grid);
    else if (mrows == 64) P2_SKINNY(2, true, grid);
    else P2_SKINNY(4, true, grid);
    return;
  }
  const dim3 grid(N / 32, S);
  if (mrows == 32) P2_SKINNY(1, false, grid);
  else if (mrows == 64) P2_SKINNY(2, false, grid);
  else P2_SKINNY(4, false, grid);
#undef P2_SKINNY
}

// ---------------------------------------------------------------------------
// 5. Head: FC1 epilogue (split-K reduce + bias + ReLU), FC2, softmax
//    cross-entropy (mean over the batch), accuracy, and the backward pass down
//    to dH = relu'(H) * (dlogits x W2).  Grid = mrows blocks (one per sample;
//    padding rows write zeros so the batch-dimension GEMMs stay exact).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void head_kernel(const float* __restrict__ slabs, int S, int mrows,
                                                   const float* __restrict__ bl1, const float* __restrict__ wl2,
                                                   const float* __restrict__ bl2, const int64_t* __restrict__ labels,
                                                   const int64_t* __restrict__ idx, int B, int train,
                                                   uint16_t* __restrict__ H, uint16_t* __restrict__ dH,
                                                   float* __restrict__ dlogits,
                                                   float* __restrict__ stats, const uint16_t* __restrict__ w2bf) {
  __shared__ float red[4][kCls];
  __shared__ float dl[kCls];
  const int b = blockIdx.x, tid = threadIdx.x, k0 = tid * 8;
  const int wave = tid >> 6, lane = tid & 63;
  if (b >= B) {
    if (train) {
      reinterpret_cast<uint4*>(dH + size_t(b) * kHid + k0)[0] = make_uint4(0, 0, 0, 0);
      reinterpret_cast<uint4*>(H + size_t(b) * kHid + k0)[0] = make_uint4(0, 0, 0, 0);
      if (tid < kCls) dlogits[b * kCls + tid] = 0.f;
    }
    return;
  }
  // the label is a dependent gather (idx -> labels): start it first, it is
  // only needed after the logits (measured: -3 us of a 9.4 us kernel)
  const int y_pref = (tid == 0) ? int(labels[idx ? idx[b] : b]) : 0;
  // issue every global load up front: this thread's 8-column slice of W2
  // (reused by the backward), the bias, and the split-K partial sums
  float wv[kCls][8];
  if (w2bf) {  // bf16 copy: 16 B per class row slice instead of 32
#pragma unroll
    for (int c = 0; c < kCls; ++c) {
      const uint4 q = *reinterpret_cast<const uint4*>(w2bf + size_t(c) * kHid + k0);
      const uint32_t u[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        wv[c][2 * j] = __uint_as_float(u[j] << 16);
        wv[c][2 * j + 1] = __uint_as_float(u[j] & 0xffff0000u);
      }
    }
  } else {
#pragma unroll
    for (int c = 0; c < kCls; ++c) {
      const float4* wp = reinterpret_cast<const float4*>(wl2 + size_t(c) * kHid + k0);
      const float4 u = wp[0], w = wp[1];
      wv[c][0] = u.x; wv[c][1] = u.y; wv[c][2] = u.z; wv[c][3] = u.w;
      wv[c][4] = w.x; wv[c][5] = w.y; wv[c][6] = w.z; wv[c][7] = w.w;
    }
  }
  float hv[8];
  {
    const float4* bp = reinterpret_cast<const float4*>(bl1 + k0);
    float4 u = bp[0], w = bp[1];
    hv[0] = u.x; hv[1] = u.y; hv[2] = u.z; hv[3] = u.w; hv[4] = w.x; hv[5] = w.y; hv[6] = w.z; hv[7] = w.w;
#pragma unroll 4
    for (int s = 0; s < S; ++s) {
      const float4* sp = reinterpret_cast<const float4*>(slabs + (size_t(s) * mrows + b) * kHid + k0);
      u = sp[0];
      w = sp[1];
      hv[0] += u.x; hv[1] += u.y; hv[2] += u.z; hv[3] += u.w; hv[4] += w.x; hv[5] += w.y; hv[6] += w.z; hv[7] += w.w;
    }
  }
  uint4 hb;
#pragma unroll
  for (int j = 0; j < 8; ++j) hv[j] = fmaxf(hv[j], 0.f);
  hb.x = pack_bf16x2(hv[0], hv[1]);
  hb.y = pack_bf16x2(hv[2], hv[3]);
  hb.z = pack_bf16x2(hv[4], hv[5]);
  hb.w = pack_bf16x2(hv[6], hv[7]);
  reinterpret_cast<uint4*>(H + size_t(b) * kHid + k0)[0] = hb;

  float part[kCls];
#pragma unroll
  for (int c = 0; c < kCls; ++c) {
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc = fmaf(hv[j], wv[c][j], acc);
    part[c] = wave_sum(acc);
  }
  if (lane == 0)
#pragma unroll
    for (int c = 0; c < kCls; ++c) red[wave][c] = part[c];
  __syncthreads();
  if (tid == 0) {
    float lg[kCls], mx = -3.4e38f;
    int am = 0;
#pragma unroll
    for (int c = 0; c < kCls; ++c) {
      lg[c] = red[0][c] + red[1][c] + red[2][c] + red[3][c] + bl2[c];
      if (lg[c] > mx) {
        mx = lg[c];
        am = c;
      }
    }
    float se = 0.f;
#pragma unroll
    for (int c = 0; c < kCls; ++c) se += __expf(lg[c] - mx);
    const float lse = mx + __logf(se);
    const int y = y_pref;
    atomicAdd(&stats[0], lse - lg[y]);
    atomicAdd(&stats[1], am == y ? 1.f : 0.f);
    const float invB = 1.f / float(B);
#pragma unroll
    for (int c = 0; c < kCls; ++c) {
      const float g = (__expf(lg[c] - lse) - (c == y ? 1.f : 0.f)) * invB;
      dl[c] = g;
      if (train) dlogits[b * kCls + c] = g;
    }
  }
  if (!train) return;
  __syncthreads();
  float g[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) g[j] = 0.f;
#pragma unroll
  for (int c = 0; c < kCls; ++c) {
    const float d = dl[c];
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = fmaf(d, wv[c][j], g[j]);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) g[j] = hv[j] > 0.f ? g[j] : 0.f;
  uint4 gb;
  gb.x = pack_bf16x2(g[0], g[1]);
  gb.y = pack_bf16x2(g[2], g[3]);
  gb.z = pack_bf16x2(g[4], g[5]);
  gb.w = pack_bf16x2(g[6], g[7]);
  reinterpret_cast<uint4*>(dH + size_t(b) * kHid + k0)[0] = gb;
}

void head(const float* slabs, int S, int mrows, const float* params, Offsets off, const int64_t* labels,
          const int64_t* idx, int B, int train, uint16_t* H, uint16_t* dH, float* dlogits,
          float* stats, const uint16_t* w2bf, hipStream_t s) {
  hipLaunchKernelGGL(head_kernel, dim3(train ? mrows : B), dim3(256), 0, s, slabs, S, mrows, params + off.l1b,
                     params + off.l2w, params + off.l2b, labels, idx, B, train, H, dH, dlogits, stats, w2bf);
}

// ---------------------------------------------------------------------------
// bf16 shadows from fp32 params (used after set_parameters / before training)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void pack_shadows_kernel(const float* __restrict__ params, Offsets off,
                                                           uint16_t* __restrict__ w2r, uint16_t* __restrict__ w2q,
                                                           uint16_t* __restrict__ w1bf,
                                                           uint16_t* __restrict__ w1tbf, uint16_t* __restrict__ w2bf) {
  const int64_t n2 = int64_t(kC2) * kC1 * kTaps, n1 = int64_t(kHid) * kFeat;
  if (w2bf)
    for (int64_t e = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; e < int64_t(kCls) * kHid;
         e += int64_t(gridDim.x) * blockDim.x)
      w2bf[e] = f32_to_bf16(params[off.l2w + e]);
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  for (int64_t e = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; e < n2 + n1; e += stride) {
    if (e < n2) {
      const int oc = int(e / (kC1 * kTaps)), rem = int(e % (kC1 * kTaps)), ic = rem / kTaps, t = rem % kTaps;
      const uint16_t v = f32_to_bf16(params[off.c2w + e]);
      w2r[(oc * kTaps + t) * kC1 + ic] = v;
      w2q[(ic * kTaps + t) * kC2 + oc] = v;
    } else {
      const int64_t j = e - n2;
      const int n = int(j / kFeat), k = int(j % kFeat);
      const uint16_t v = f32_to_bf16(params[off.l1w + j]);
      w1bf[j] = v;
      if (w1tbf) w1tbf[size_t(k) * kHid + n] = v;
    }
  }
}

void pack_shadows(const float* params, Offsets off, uint16_t* w2r, uint16_t* w2q, uint16_t* w1bf, uint16_t* w1tbf,
                  uint16_t* w2bf, hipStream_t s) {
  hipLaunchKernelGGL(pack_shadows_kernel, dim3(2048), dim3(256), 0, s, params, off, w2r, w2q, w1bf, w1tbf, w2bf);
}

}  // namespace p2cnn
