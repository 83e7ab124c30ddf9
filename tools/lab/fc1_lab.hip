// Kernel lab: where does fc1_wgrad_adam's time go?  Variants of the production
// kernel (copied, with write knobs) plus pure streaming-Adam references.
//   hipcc -O3 --offload-arch=gfx950 -Icsrc tools/lab/fc1_lab.hip -o /tmp/fc1_lab
#include "../../csrc/cnn_bwd.hip"
namespace p2cnn {
void init_fwd_attributes() {}
}
#include <cstdio>
#include <vector>
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


// Variant: gradient tile transposed through LDS so every lane owns 4
// consecutive k of one row -> 16-B p/m/v loads and stores, 8-B bf16 shadow
// stores (the production kernel does 4-B / 2-B accesses in the MFMA
// accumulator layout).
template <int MR>
__global__ __launch_bounds__(256) void fc1_vec(const uint16_t* __restrict__ dH, const uint16_t* __restrict__ a1,
                                               float* __restrict__ p, float* __restrict__ m, float* __restrict__ v,
                                               float* __restrict__ gdump, uint16_t* __restrict__ w1bf,
                                               uint16_t* __restrict__ w1tbf, Offsets off,
                                               const int* __restrict__ adam_t, int t_off, AdamCfg cfg) {
  constexpr int P = MR + 8;
  constexpr int GP = 132;  // fp32 pitch of the gradient tile
  constexpr int kStage = (32 + 128) * P * 2;
  constexpr int kGrad = 32 * GP * 4;
  __shared__ __attribute__((aligned(16))) char smem[kStage > kGrad ? kStage : kGrad];
  __shared__ __attribute__((aligned(16))) uint16_t tr[128][40];
  uint16_t(*sdh)[P] = reinterpret_cast<uint16_t(*)[P]>(smem);
  uint16_t(*sa1)[P] = reinterpret_cast<uint16_t(*)[P]>(smem + 32 * P * 2);
  float(*gt)[GP] = reinterpret_cast<float(*)[GP]>(smem);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const int n0 = blockIdx.y * 32;
  const int kb = blockIdx.x * 128;
  // this thread's Adam elements: row nl, k = kb + kq + 32 j + [0, 4)
  const int nl = tid >> 3, kq = (tid & 7) * 4;
  float* pw = p + off.l1w;
  float* mw = m + off.l1w;
  float* vw = v + off.l1w;
  float4 pr[4], mr[4], vr[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int k = kb + kq + 32 * j;
    if (k < kFeat) {
      const int64_t e = int64_t(n0 + nl) * kFeat + k;
      pr[j] = *reinterpret_cast<const float4*>(pw + e);
      mr[j] = *reinterpret_cast<const float4*>(mw + e);
      vr[j] = *reinterpret_cast<const float4*>(vw + e);
    }
  }
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
  const AdamScal s = adam_scal(cfg, adam_t, t_off);
  if (blockIdx.x == 0 && wave == 0 && lane < 32) {  // FC1 bias (reads sdh before the tile reuses it)
    const int n = n0 + lane;
    float g = 0.f;
    for (int b = 0; b < MR; ++b) g += bf16_to_f32(sdh[lane][b]);
    if (gdump) gdump[off.l1b + n] = g;
    adam_apply(p, m, v, off.l1b + n, g, cfg, s);
  }
  f32x16 acc = {};
#pragma unroll
  for (int ks = 0; ks < MR / 16; ++ks) {
    const uint4 a = *reinterpret_cast<const uint4*>(&sdh[r][ks * 16 + 8 * h]);
    const uint4 b = *reinterpret_cast<const uint4*>(&sa1[wave * 32 + r][ks * 16 + 8 * h]);
    acc = mfma32b(a, b, acc);
  }
  __syncthreads();  // staging dead -> gradient tile
#pragma unroll
  for (int i = 0; i < 16; ++i) gt[acc_row_b(i, h)][wave * 32 + r] = acc[i];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int kl = kq + 32 * j, k = kb + kl;
    if (k >= kFeat) continue;
    const float4 g = *reinterpret_cast<const float4*>(&gt[nl][kl]);
    const int64_t e = int64_t(n0 + nl) * kFeat + k;
    if (gdump) *reinterpret_cast<float4*>(gdump + off.l1w + e) = g;
    adam_regs(pr[j].x, mr[j].x, vr[j].x, g.x, cfg, s);
    adam_regs(pr[j].y, mr[j].y, vr[j].y, g.y, cfg, s);
    adam_regs(pr[j].z, mr[j].z, vr[j].z, g.z, cfg, s);
    adam_regs(pr[j].w, mr[j].w, vr[j].w, g.w, cfg, s);
    *reinterpret_cast<float4*>(pw + e) = pr[j];
    *reinterpret_cast<float4*>(mw + e) = mr[j];
    *reinterpret_cast<float4*>(vw + e) = vr[j];
    const uint16_t b0 = f32_to_bf16(pr[j].x), b1 = f32_to_bf16(pr[j].y), b2 = f32_to_bf16(pr[j].z),
                   b3 = f32_to_bf16(pr[j].w);
    uint2 o;
    o.x = uint32_t(b0) | (uint32_t(b1) << 16);
    o.y = uint32_t(b2) | (uint32_t(b3) << 16);
    *reinterpret_cast<uint2*>(w1bf + e) = o;
    tr[kl][nl] = b0;
    tr[kl + 1][nl] = b1;
    tr[kl + 2][nl] = b2;
    tr[kl + 3][nl] = b3;
  }
  __syncthreads();
  for (int j = tid; j < 128 * 4; j += 256) {
    const int kl = j >> 2, q = j & 3;
    const int k = kb + kl;
    if (k < kFeat)
      *reinterpret_cast<uint4*>(w1tbf + size_t(k) * kHid + n0 + q * 8) = *reinterpret_cast<const uint4*>(&tr[kl][q * 8]);
  }
}
}  // namespace p2cnn

__global__ void fill_rand(float* x, size_t n, uint32_t seed, float scale, float bias) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += size_t(gridDim.x) * 256) {
    uint32_t h = uint32_t(i) * 2654435761u ^ seed;
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    x[i] = bias + scale * (float(h & 0xffffff) / 16777216.f - 0.5f);
  }
}
__global__ void fill_rand_bf16(uint16_t* x, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += size_t(gridDim.x) * 256) {
    uint32_t h = uint32_t(i) * 2654435761u ^ seed;
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    x[i] = f32_to_bf16(float(h & 0xffff) / 65536.f - 0.5f);
  }
}

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
  {  // correctness: production vs vectorised variant from identical random state
    float *p2, *m2, *v2;
    uint16_t *b1, *b2, *t1, *t2;
    P2_CHECK(hipMalloc(&p2, np * 4));
    P2_CHECK(hipMalloc(&m2, np * 4));
    P2_CHECK(hipMalloc(&v2, np * 4));
    P2_CHECK(hipMalloc(&b1, nw * 2));
    P2_CHECK(hipMalloc(&b2, nw * 2));
    P2_CHECK(hipMalloc(&t1, nw * 2));
    P2_CHECK(hipMalloc(&t2, nw * 2));
    hipLaunchKernelGGL(fill_rand, dim3(2048), dim3(256), 0, 0, p, np, 1u, 0.1f, 0.f);
    hipLaunchKernelGGL(fill_rand, dim3(2048), dim3(256), 0, 0, m, np, 2u, 0.01f, 0.f);
    hipLaunchKernelGGL(fill_rand, dim3(2048), dim3(256), 0, 0, v, np, 3u, 0.0001f, 0.0001f);
    hipLaunchKernelGGL(fill_rand_bf16, dim3(256), dim3(256), 0, 0, dH, size_t(32) * kHid, 4u);
    hipLaunchKernelGGL(fill_rand_bf16, dim3(256), dim3(256), 0, 0, a1, size_t(32) * kFeat, 5u);
    P2_CHECK(hipMemcpy(p2, p, np * 4, hipMemcpyDeviceToDevice));
    P2_CHECK(hipMemcpy(m2, m, np * 4, hipMemcpyDeviceToDevice));
    P2_CHECK(hipMemcpy(v2, v, np * 4, hipMemcpyDeviceToDevice));
    fc1_wgrad_adam(dH, a1, 32, p, m, v, nullptr, b1, t1, off, t, 1, cfg, 0);
    hipLaunchKernelGGL((fc1_vec<32>), grid, dim3(256), 0, 0, dH, a1, p2, m2, v2, nullptr, b2, t2, off, t, 1, cfg);
    P2_CHECK(hipDeviceSynchronize());
    auto cmp = [&](const void* x, const void* y, size_t bytes, const char* name) {
      std::vector<unsigned char> hx(bytes), hy(bytes);
      P2_CHECK(hipMemcpy(hx.data(), x, bytes, hipMemcpyDeviceToHost));
      P2_CHECK(hipMemcpy(hy.data(), y, bytes, hipMemcpyDeviceToHost));
      size_t diff = 0;
      for (size_t i = 0; i < bytes; ++i) diff += hx[i] != hy[i];
      printf("check %-6s %s (%zu differing bytes)\n", name, diff ? "MISMATCH" : "bitwise equal", diff);
    };
    cmp(p + off.l1w, p2 + off.l1w, nw * 4, "W1");
    cmp(m + off.l1w, m2 + off.l1w, nw * 4, "m");
    cmp(v + off.l1w, v2 + off.l1w, nw * 4, "v");
    cmp(p + off.l1b, p2 + off.l1b, kHid * 4, "b1");
    cmp(b1, b2, nw * 2, "W1bf");
    cmp(t1, t2, nw * 2, "W1Tbf");
  }
  printf("fc1 vec (16-B accesses)  %7.2f us\n", time_us([&] { hipLaunchKernelGGL((fc1_vec<32>), grid, dim3(256), 0, 0, dH, a1, p, m, v, nullptr, w1bf, w1tbf, off, t, 1, cfg); }));
  printf("fc1 prod                 %7.2f us\n", time_us([&] { fc1_wgrad_adam(dH, a1, 32, p, m, v, nullptr, w1bf, w1tbf, off, t, 1, cfg, 0); }));
  printf("fc1 no W1T write         %7.2f us\n", time_us([&] { hipLaunchKernelGGL((fc1_var<32, 1>), grid, dim3(256), 0, 0, dH, a1, p, m, v, nullptr, w1bf, w1tbf, off, t, 1, cfg); }));
  printf("fc1 no shadow writes     %7.2f us\n", time_us([&] { hipLaunchKernelGGL((fc1_var<32, 3>), grid, dim3(256), 0, 0, dH, a1, p, m, v, nullptr, w1bf, w1tbf, off, t, 1, cfg); }));
  printf("adam stream1 (6.4M)      %7.2f us\n", time_us([&] { hipLaunchKernelGGL(adam_stream1, dim3(2048), dim3(256), 0, 0, p + off.l1w, m + off.l1w, v + off.l1w, g, int(nw), cfg, t); }));
  printf("adam stream4 (6.4M)      %7.2f us\n", time_us([&] { hipLaunchKernelGGL(adam_stream4, dim3(2048), dim3(256), 0, 0, p + off.l1w, m + off.l1w, v + off.l1w, g, nullptr, int(nw / 4), cfg, t); }));
  printf("adam stream4 + bf16 sh   %7.2f us\n", time_us([&] { hipLaunchKernelGGL(adam_stream4, dim3(2048), dim3(256), 0, 0, p + off.l1w, m + off.l1w, v + off.l1w, g, w1bf, int(nw / 4), cfg, t); }));
  printf("adam stream4 grid 8192   %7.2f us\n", time_us([&] { hipLaunchKernelGGL(adam_stream4, dim3(8192), dim3(256), 0, 0, p + off.l1w, m + off.l1w, v + off.l1w, g, w1bf, int(nw / 4), cfg, t); }));
  return 0;
}
