// Kernel lab: head kernel variants (atomics vs per-sample stats, label prefetch)
// and FC1 split-K choices.   hipcc -O3 --offload-arch=gfx950 -Icsrc tools/lab/head_lab.hip
#include "../../csrc/cnn_fwd.hip"
#include <cstdio>
namespace p2cnn {
__global__ __launch_bounds__(256) void head_noatomic(const float* __restrict__ slabs, int S, int mrows,
                                                   const float* __restrict__ bl1, const float* __restrict__ wl2,
                                                   const float* __restrict__ bl2, const int64_t* __restrict__ labels,
                                                   const int64_t* __restrict__ idx, int B, int train,
                                                   uint16_t* __restrict__ H, uint16_t* __restrict__ dH,
                                                   float* __restrict__ dlogits,
                                                   float* __restrict__ stats) {
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
  // issue every global load up front: this thread's 8-column slice of W2
  // (reused by the backward), the bias, and the split-K partial sums
  float wv[kCls][8];
#pragma unroll
  for (int c = 0; c < kCls; ++c) {
    const float4* wp = reinterpret_cast<const float4*>(wl2 + size_t(c) * kHid + k0);
    const float4 u = wp[0], w = wp[1];
    wv[c][0] = u.x; wv[c][1] = u.y; wv[c][2] = u.z; wv[c][3] = u.w;
    wv[c][4] = w.x; wv[c][5] = w.y; wv[c][6] = w.z; wv[c][7] = w.w;
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
    const int y = int(labels[idx ? idx[b] : b]);
    stats[2 * b] = lse - lg[y];
    stats[2 * b + 1] = am == y ? 1.f : 0.f;
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

__global__ __launch_bounds__(256) void head_noatomic_pref(const float* __restrict__ slabs, int S, int mrows,
                                                   const float* __restrict__ bl1, const float* __restrict__ wl2,
                                                   const float* __restrict__ bl2, const int64_t* __restrict__ labels,
                                                   const int64_t* __restrict__ idx, int B, int train,
                                                   uint16_t* __restrict__ H, uint16_t* __restrict__ dH,
                                                   float* __restrict__ dlogits,
                                                   float* __restrict__ stats) {
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
  const int y_pref = (tid == 0) ? int(labels[idx ? idx[b] : b]) : 0;
  // issue every global load up front: this thread's 8-column slice of W2
  // (reused by the backward), the bias, and the split-K partial sums
  float wv[kCls][8];
#pragma unroll
  for (int c = 0; c < kCls; ++c) {
    const float4* wp = reinterpret_cast<const float4*>(wl2 + size_t(c) * kHid + k0);
    const float4 u = wp[0], w = wp[1];
    wv[c][0] = u.x; wv[c][1] = u.y; wv[c][2] = u.z; wv[c][3] = u.w;
    wv[c][4] = w.x; wv[c][5] = w.y; wv[c][6] = w.z; wv[c][7] = w.w;
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
    stats[2 * b] = lse - lg[y];
    stats[2 * b + 1] = am == y ? 1.f : 0.f;
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

}  // namespace p2cnn
using namespace p2cnn;
template <typename F>
static float time_us(F f, int reps = 200) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int i = 0; i < 10; ++i) f();
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(a);
  for (int i = 0; i < reps; ++i) f();
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms * 1000.f / reps;
}
int main() {
  float *slabs, *params, *dlog, *stats;
  uint16_t *H, *dH, *A, *W;
  int64_t* labels;
  P2_CHECK(hipMalloc(&slabs, 16 * 32 * kHid * 4));
  P2_CHECK(hipMalloc(&params, 6600000 * 4));
  P2_CHECK(hipMalloc(&dlog, 64 * 10 * 4));
  P2_CHECK(hipMalloc(&stats, 256 * 4));
  P2_CHECK(hipMalloc(&H, 64 * kHid * 2));
  P2_CHECK(hipMalloc(&dH, 64 * kHid * 2));
  P2_CHECK(hipMalloc(&A, 64 * kFeat * 2));
  P2_CHECK(hipMalloc(&W, size_t(kHid) * kFeat * 2));
  P2_CHECK(hipMalloc(&labels, 64 * 8));
  P2_CHECK(hipMemset(slabs, 0, 16 * 32 * kHid * 4));
  P2_CHECK(hipMemset(params, 0, 6600000 * 4));
  P2_CHECK(hipMemset(labels, 0, 64 * 8));
  P2_CHECK(hipMemset(A, 0, 64 * kFeat * 2));
  P2_CHECK(hipMemset(W, 0, size_t(kHid) * kFeat * 2));
  Offsets off{0, 832, 896, 52096, 52160, 6474816, 6476864, 6497344};
  const float* pb1 = params + off.l1b; const float* pw2 = params + off.l2w; const float* pb2 = params + off.l2b;
  for (int S : {7, 4}) {
    printf("S=%d head prod (atomics)     %7.2f us\n", S, time_us([&] { head(slabs, S, 32, params, off, labels, nullptr, 32, 1, H, dH, dlog, stats, 0); }));
    printf("S=%d head no atomics         %7.2f us\n", S, time_us([&] { hipLaunchKernelGGL(head_noatomic, dim3(32), dim3(256), 0, 0, slabs, S, 32, pb1, pw2, pb2, labels, nullptr, 32, 1, H, dH, dlog, stats); }));
    printf("S=%d head no atomics + pref  %7.2f us\n", S, time_us([&] { hipLaunchKernelGGL(head_noatomic_pref, dim3(32), dim3(256), 0, 0, slabs, S, 32, pb1, pw2, pb2, labels, nullptr, 32, 1, H, dH, dlog, stats); }));
  }
  for (int S : {4, 7, 8, 14})
    printf("gemm fc1 S=%2d               %7.2f us\n", S, time_us([&] { gemm_skinny(A, W, slabs, 32, kHid, kFeat, S, 0); }));
  return 0;
}
