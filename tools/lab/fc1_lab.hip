// Kernel lab: where does fc1_wgrad_adam's time go?  Variants of the production
// kernel (copied, with write knobs) plus pure streaming-Adam references.
//   hipcc -O3 --offload-arch=gfx950 -Icsrc tools/lab/fc1_lab.hip -o /tmp/fc1_lab
#include "../../csrc/cnn_bwd.hip"
namespace p2cnn {
void init_fwd_attributes() {}
}
#include <cstdio>
using namespace p2cnn;

namespace p2cnn {
template <int MR, int VAR>
__global__ __launch_bounds__(256) void fc1_var(const uint16_t* __restrict__ dH,
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
  const int k0 = kb + wave * 32;
  const bool valid = k0 < kFeat;
  // This lane's 16 Adam elements: all 48 fp32 loads (W1, m, v) are issued
  // first, so their latency overlaps the staging and the MFMA (one memory
  // round trip per lane instead of one per element).
  float* pw = p + off.l1w;
  float* mw = m + off.l1w;
  float* vw = v + off.l1w;
  float pr[16], mr[16], vr[16];
  if (valid) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int64_t e = int64_t(n0 + acc_row_b(i, h)) * kFeat + k0 + r;
      pr[i] = pw[e];
      mr[i] = mw[e];
      vr[i] = vw[e];
    }
  }
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
  f32x16 acc = {};
#pragma unroll
  for (int ks = 0; ks < MR / 16; ++ks) {
    const uint4 a = *reinterpret_cast<const uint4*>(&sdh[r][ks * 16 + 8 * h]);
    const uint4 b = *reinterpret_cast<const uint4*>(&sa1[wave * 32 + r][ks * 16 + 8 * h]);
    acc = mfma32b(a, b, acc);
  }
  const AdamScal s = adam_scal(cfg, adam_t, t_off);
  if (valid) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int nl = acc_row_b(i, h);
      const int64_t e = int64_t(n0 + nl) * kFeat + k0 + r;
      if (gdump) gdump[off.l1w + e] = acc[i];
      adam_regs(pr[i], mr[i], vr[i], acc[i], cfg, s);
      pw[e] = pr[i];
      mw[e] = mr[i];
      vw[e] = vr[i];
      const uint16_t hb = f32_to_bf16(pr[i]);
      if (!(VAR & 2)) w1bf[e] = hb;
      tr[wave * 32 + r][nl] = hb;
    }
  }
  __syncthreads();
  for (int j = tid; j < 128 * 4; j += 256) {
    const int kl = j >> 2, q = j & 3;
    const int k = kb + kl;
    if (!(VAR & 1) && k < kFeat)
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

}  // namespace p2cnn

// streaming Adam over n elements, 1 element per thread-iteration
__global__ __launch_bounds__(256) void adam_stream1(float* __restrict__ p, float* __restrict__ m, float* __restrict__ v,
                                                    const float* __restrict__ g, int n, AdamCfg cfg, const int* t) {
  const AdamScal s = adam_scal(cfg, t, 1);
  for (int e = blockIdx.x * 256 + threadIdx.x; e < n; e += gridDim.x * 256) {
    float pv = p[e], mv = m[e], vv = v[e];
    adam_regs(pv, mv, vv, g[e & 1023], cfg, s);
    p[e] = pv; m[e] = mv; v[e] = vv;
  }
}
// 4 elements per lane, 16-B accesses, + bf16 shadow
__global__ __launch_bounds__(256) void adam_stream4(float* __restrict__ p, float* __restrict__ m, float* __restrict__ v,
                                                    const float* __restrict__ g, uint16_t* __restrict__ sh, int n4, AdamCfg cfg, const int* t) {
  const AdamScal s = adam_scal(cfg, t, 1);
  for (int e = blockIdx.x * 256 + threadIdx.x; e < n4; e += gridDim.x * 256) {
    float4 pv = reinterpret_cast<float4*>(p)[e], mv = reinterpret_cast<float4*>(m)[e], vv = reinterpret_cast<float4*>(v)[e];
    const float gg = g[e & 1023];
    adam_regs(pv.x, mv.x, vv.x, gg, cfg, s);
    adam_regs(pv.y, mv.y, vv.y, gg, cfg, s);
    adam_regs(pv.z, mv.z, vv.z, gg, cfg, s);
    adam_regs(pv.w, mv.w, vv.w, gg, cfg, s);
    reinterpret_cast<float4*>(p)[e] = pv; reinterpret_cast<float4*>(m)[e] = mv; reinterpret_cast<float4*>(v)[e] = vv;
    if (sh) {
      uint2 o;
      o.x = pack_bf16x2(pv.x, pv.y);
      o.y = pack_bf16x2(pv.z, pv.w);
      reinterpret_cast<uint2*>(sh)[e] = o;
    }
  }
}

template <typename F>
static float time_us(F f, int reps = 100) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int i = 0; i < 5; ++i) f();
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
  const size_t np = 6600000, nw = size_t(kHid) * kFeat;
  uint16_t *dH, *a1, *w1bf, *w1tbf;
  float *p, *m, *v, *g;
  int* t;
  P2_CHECK(hipMalloc(&dH, 32 * kHid * 2));
  P2_CHECK(hipMalloc(&a1, 32 * kFeat * 2));
  P2_CHECK(hipMalloc(&w1bf, nw * 2));
  P2_CHECK(hipMalloc(&w1tbf, nw * 2));
  P2_CHECK(hipMalloc(&p, np * 4));
  P2_CHECK(hipMalloc(&m, np * 4));
  P2_CHECK(hipMalloc(&v, np * 4));
  P2_CHECK(hipMalloc(&g, 4096 * 4));
  P2_CHECK(hipMalloc(&t, 4));
  P2_CHECK(hipMemset(dH, 0, 32 * kHid * 2));
  P2_CHECK(hipMemset(a1, 0, 32 * kFeat * 2));
  P2_CHECK(hipMemset(p, 0, np * 4));
  P2_CHECK(hipMemset(m, 0, np * 4));
  P2_CHECK(hipMemset(v, 0, np * 4));
  P2_CHECK(hipMemset(g, 0, 4096 * 4));
  P2_CHECK(hipMemset(t, 0, 4));
  Offsets off{0, 832, 896, 52096, 52160, 6474816, 6476864, 6497344};
  AdamCfg cfg{1e-3f, 0.9f, 0.999f, 1e-8f, 0.f};
  const dim3 grid((kFeat + 127) / 128, kHid / 32);
  printf("fc1 prod                 %7.2f us\n", time_us([&] { fc1_wgrad_adam(dH, a1, 32, p, m, v, nullptr, w1bf, w1tbf, off, t, 1, cfg, 0); }));
  printf("fc1 no W1T write         %7.2f us\n", time_us([&] { hipLaunchKernelGGL((fc1_var<32, 1>), grid, dim3(256), 0, 0, dH, a1, p, m, v, nullptr, w1bf, w1tbf, off, t, 1, cfg); }));
  printf("fc1 no shadow writes     %7.2f us\n", time_us([&] { hipLaunchKernelGGL((fc1_var<32, 3>), grid, dim3(256), 0, 0, dH, a1, p, m, v, nullptr, w1bf, w1tbf, off, t, 1, cfg); }));
  printf("adam stream1 (6.4M)      %7.2f us\n", time_us([&] { hipLaunchKernelGGL(adam_stream1, dim3(2048), dim3(256), 0, 0, p + off.l1w, m + off.l1w, v + off.l1w, g, int(nw), cfg, t); }));
  printf("adam stream4 (6.4M)      %7.2f us\n", time_us([&] { hipLaunchKernelGGL(adam_stream4, dim3(2048), dim3(256), 0, 0, p + off.l1w, m + off.l1w, v + off.l1w, g, nullptr, int(nw / 4), cfg, t); }));
  printf("adam stream4 + bf16 sh   %7.2f us\n", time_us([&] { hipLaunchKernelGGL(adam_stream4, dim3(2048), dim3(256), 0, 0, p + off.l1w, m + off.l1w, v + off.l1w, g, w1bf, int(nw / 4), cfg, t); }));
  printf("adam stream4 grid 8192   %7.2f us\n", time_us([&] { hipLaunchKernelGGL(adam_stream4, dim3(8192), dim3(256), 0, 0, p + off.l1w, m + off.l1w, v + off.l1w, g, w1bf, int(nw / 4), cfg, t); }));
  return 0;
}
