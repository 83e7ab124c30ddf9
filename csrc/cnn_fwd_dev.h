// Device bodies of the fused MNIST-CNN forward convolutions (cnn_fwd.hip), shared
// by their stand-alone kernels and by the backward's last launch, which runs the
// NEXT step's conv1 + conv2 beside the FC1 Adam stream (cnn_bwd.hip
// fc1_conv_adam_fwd_kernel).  WT (write-through): inside that launch the conv
// weights were just rewritten by other workgroups (the conv-parameter Adam blocks)
// and P1 travels from the conv1 to the conv2 workgroups -- possibly on other XCDs,
// whose L2s are not coherent with each other -- so the weights and P1 are read
// with device-coherent (sc1) loads and P1 is stored write-through (sc1), the
// hand-off of gemm_core.h's split-K reduction.  WT = false: plain loads / stores.
#pragma once
#include "cnn.h"
#include "common.h"

namespace p2cnn {
using namespace p2;

typedef __bf16 bf16x8_dev_t __attribute__((ext_vector_type(8)));

P2_DEVICE f32x16 mfma32_fwd(uint4 a, uint4 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_dev_t, a), __builtin_bit_cast(bf16x8_dev_t, b),
                                                 c, 0, 0, 0);
}
P2_DEVICE int acc_row_fwd(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

// sc1 (device-coherent) accesses through a wave-uniform base and per-lane byte offsets
P2_DEVICE __amdgpu_buffer_rsrc_t rsrc_of(const void* base, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, bytes, 0x00020000);
}
template <bool WT>
P2_DEVICE float ldf(const float* p) {
  if constexpr (WT) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return *p;
}

// LDS of one conv1 workgroup
struct Conv1Smem {
  float img[8][33];                                 // padded input rows 4q .. 4q+7
  uint16_t sv[kC1][2][16];                          // pooled values [oc][row][px], cols 14/15 zero
  __attribute__((aligned(16))) uint8_t sa[28][kC1];  // argmax codes [pos][oc]
};

// conv1 (1->32, 5x5, pad 2) + bias + ReLU + maxpool 2x2 of pooled rows 2q, 2q+1 of
// image b (see conv1_fwd_kernel); 256 threads.
template <bool WT>
P2_DEVICE void conv1_body(int q, int b, const uint8_t* __restrict__ x, const int64_t* __restrict__ idx,
                          const float* __restrict__ w1, const float* __restrict__ b1, uint16_t* __restrict__ p1,
                          uint8_t* __restrict__ am1, uint16_t* __restrict__ p1s, Conv1Smem& sm) {
  const int tid = threadIdx.x;
  const int64_t row = idx ? idx[b] : b;
  const uint8_t* src = x + row * (kImg * kImg);
  {
    const int i = tid, yy = i >> 5, xx = i & 31, sy = 4 * q + yy - 2, sx = xx - 2;
    float v = 0.f;
    if (sy >= 0 && sy < kImg && sx >= 0 && sx < kImg) v = float(src[sy * kImg + sx]) * (1.f / 255.f);
    sm.img[yy][xx] = v;
  }
  const int oc = tid & 31;
  float w[kTaps];
#pragma unroll
  for (int t = 0; t < kTaps; ++t) w[t] = ldf<WT>(w1 + oc * kTaps + t);
  const float bias = ldf<WT>(b1 + oc);
  if (tid < kC1 * 2 * 2) sm.sv[tid >> 2][(tid >> 1) & 1][14 + (tid & 1)] = 0;
  __syncthreads();
  for (int k = tid >> 5; k < 28; k += 8) {
    const int rr = k / 14, px = k % 14;
    float win[6][6];
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
      for (int j = 0; j < 6; ++j) win[i][j] = sm.img[2 * rr + i][2 * px + j];
    float best = -3.4e38f;
    int arg = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const int dy = d >> 1, dx = d & 1;
      float s = bias;
#pragma unroll
      for (int ky = 0; ky < 5; ++ky)
#pragma unroll
        for (int kx = 0; kx < 5; ++kx) s = fmaf(w[ky * 5 + kx], win[dy + ky][dx + kx], s);
      if (s > best) {
        best = s;
        arg = d;
      }
    }
    sm.sv[oc][rr][px] = f32_to_bf16(fmaxf(best, 0.f));
    sm.sa[k][oc] = best > 0.f ? uint8_t(arg) : uint8_t(4);
  }
  __syncthreads();
  const size_t pix0 = size_t(b) * 196 + q * 28;
  // P1 (HWC): 28 pixels x 4 chunks of 8 channels;  AM1: 28 pixels x 2 chunks of 16
  if (tid < 28 * 4) {
    const int k = tid >> 2, c0 = (tid & 3) * 8;
    uint16_t u[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) u[j] = sm.sv[c0 + j][k / 14][k % 14];
    uint4 o;
    o.x = uint32_t(u[0]) | (uint32_t(u[1]) << 16);
    o.y = uint32_t(u[2]) | (uint32_t(u[3]) << 16);
    o.z = uint32_t(u[4]) | (uint32_t(u[5]) << 16);
    o.w = uint32_t(u[6]) | (uint32_t(u[7]) << 16);
    if constexpr (WT)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), rsrc_of(p1 + pix0 * kC1, 28 * kC1 * 2),
                                             (k * kC1 + c0) * 2, 0, 16);
    else
      reinterpret_cast<uint4*>(p1 + (pix0 + k) * kC1)[tid & 3] = o;
  } else if (tid < 28 * 4 + 28 * 2) {
    const int i = tid - 28 * 4, k = i >> 1, c0 = (i & 1) * 16;
    reinterpret_cast<uint4*>(am1 + (pix0 + k) * kC1)[i & 1] = *reinterpret_cast<const uint4*>(&sm.sa[k][c0]);
  }
  if (p1s) {
    // P1s[b][kx][oc][2q + rr + 2][c] = P1[oc][2q + rr][c + kx - 2]  (0 outside)
    for (int i = tid; i < 5 * kC1 * 2 * 2; i += 256) {
      const int half = i & 1, rr = (i >> 1) & 1, o = (i >> 2) % kC1, kx = i / (4 * kC1);
      uint16_t u[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int xs = half * 8 + j + kx - 2;
        u[j] = (xs >= 0 && xs < 14) ? sm.sv[o][rr][xs] : uint16_t(0);
      }
      uint4 v;
      v.x = uint32_t(u[0]) | (uint32_t(u[1]) << 16);
      v.y = uint32_t(u[2]) | (uint32_t(u[3]) << 16);
      v.z = uint32_t(u[4]) | (uint32_t(u[5]) << 16);
      v.w = uint32_t(u[6]) | (uint32_t(u[7]) << 16);
      *reinterpret_cast<uint4*>(p1s + ((size_t(b) * 5 + kx) * kC1 + o) * kP1sPlane + (2 * q + rr + 2) * 16 + half * 8) = v;
    }
  }
}

// conv2 (32->64, 5x5, pad 2) on MFMA + bias / ReLU / maxpool of pooled row py, oc half
// nh, image b: ONE wave (lane 0..63), see conv2_fwd_kernel.  `on` false: the wave only
// takes part in the barrier (a 4-wave workgroup whose last items ran out).
template <bool WT>
P2_DEVICE void conv2_body(bool on, int py, int nh, int b, int lane, const uint16_t* __restrict__ p1,
                          const uint16_t* __restrict__ w2r, const float* __restrict__ b2, uint16_t* __restrict__ a1,
                          uint8_t* __restrict__ am2, float (*sout)[33]) {
  const int r = lane & 31, h = lane >> 5;
  if (on) {
    const int rr = r < 28 ? r : 27;
    const int y = 2 * py + (rr >= 14 ? 1 : 0), x = rr >= 14 ? rr - 14 : rr;
    const uint16_t* img = p1 + size_t(b) * 196 * kC1;
    const uint16_t* wbase = w2r + size_t(nh * 32) * kTaps * kC1;
    const auto rimg = rsrc_of(img, 196 * kC1 * 2);
    const auto rw = rsrc_of(wbase, 32 * kTaps * kC1 * 2);
    const uint4 z4 = make_uint4(0, 0, 0, 0);
    auto load = [&](int c, uint4 (&A)[10], uint4 (&Bv)[10]) {
#pragma unroll
      for (int j = 0; j < 10; ++j) {
        const int s = c * 10 + j, t = s >> 1, ky = t / 5, kx = t % 5, ic = (s & 1) * 16;
        const int iy = y + ky - 2, ix = x + kx - 2;
        const bool ok = iy >= 0 && iy < 14 && ix >= 0 && ix < 14;
        const int pix = ok ? iy * 14 + ix : 0;
        const int ao = (pix * kC1 + ic + 8 * h) * 2, bo = ((r * kTaps + t) * kC1 + ic + 8 * h) * 2;
        uint4 v, wv;
        if constexpr (WT) {
          v = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rimg, ao, 0, 16));
          wv = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rw, bo, 0, 16));
        } else {
          v = *reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(img) + ao);
          wv = *reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(wbase) + bo);
        }
        A[j] = ok ? v : z4;
        Bv[j] = wv;
      }
    };
    f32x16 acc = {};
    if constexpr (WT) {
      // beside the FC1 Adam stream (fc1_conv_adam_fwd_kernel): 10 fragments in flight
      // per chunk, no second buffer -- the launch's register budget is the stream's
      // occupancy (same k order as below: bitwise-equal results)
#pragma unroll 1
      for (int c = 0; c < 5; ++c) {
        uint4 A0[10], B0[10];
        load(c, A0, B0);
#pragma unroll
        for (int j = 0; j < 10; ++j) acc = mfma32_fwd(A0[j], B0[j], acc);
      }
    } else {
      uint4 A0[10], B0[10], A1[10], B1[10];
      load(0, A0, B0);
#pragma unroll
      for (int c = 0; c < 5; c += 2) {
        if (c + 1 < 5) load(c + 1, A1, B1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < 10; ++j) acc = mfma32_fwd(A0[j], B0[j], acc);
        __builtin_amdgcn_sched_barrier(0);
        if (c + 1 < 5) {
          if (c + 2 < 5) load(c + 2, A0, B0);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int j = 0; j < 10; ++j) acc = mfma32_fwd(A1[j], B1[j], acc);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int row = acc_row_fwd(i, h);
      if (row < 28) sout[row][r] = acc[i];
    }
  }
  __syncthreads();
  if (!on) return;
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
    best += ldf<WT>(b2 + nh * 32 + oc);
    const size_t o = size_t(b) * kFeat + (nh * 32 + oc) * 49 + py * 7 + px;
    a1[o] = f32_to_bf16(fmaxf(best, 0.f));
    am2[o] = best > 0.f ? uint8_t(arg) : uint8_t(4);
  }
}

}  // namespace p2cnn
