// Kernel lab: is fc1_wgrad_adam's gap to a streaming Adam its access pattern?
//   hipcc -O3 --offload-arch=gfx950 -Icsrc tools/lab/adam_pattern_lab.hip
#include "../../csrc/cnn_bwd.hip"
namespace p2cnn { void init_fwd_attributes() {} }
#include <cstdio>
using namespace p2cnn;

// fc1's pattern: lane (r, h) owns column k0 + r and 16 rows acc_row(i, h) of a 32x32 tile
__global__ __launch_bounds__(256) void adam_mfma_pattern(float* p, float* m, float* v, uint16_t* sh, AdamCfg cfg, const int* t) {
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const int n0 = blockIdx.y * 32, k0 = blockIdx.x * 128 + wave * 32;
  if (k0 >= kFeat) return;
  const AdamScal s = adam_scal(cfg, t, 1);
  float pr[16], mr[16], vr[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int64_t e = int64_t(n0 + acc_row_b(i, h)) * kFeat + k0 + r;
    pr[i] = p[e]; mr[i] = m[e]; vr[i] = v[e];
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int64_t e = int64_t(n0 + acc_row_b(i, h)) * kFeat + k0 + r;
    adam_regs(pr[i], mr[i], vr[i], 1e-3f, cfg, s);
    p[e] = pr[i]; m[e] = mr[i]; v[e] = vr[i];
    sh[e] = f32_to_bf16(pr[i]);
  }
}
// same 4096-element tiles (rows x TK), coalesced: consecutive threads take
// consecutive 16-B chunks of a row (q-th chunk group strided by 256 threads)
template <int TK>
__global__ __launch_bounds__(256) void adam_row_pattern(float* p, float* m, float* v, uint16_t* sh, AdamCfg cfg, const int* t) {
  constexpr int C4 = TK / 4;  // float4 per tile row
  const int tid = threadIdx.x;
  const AdamScal s = adam_scal(cfg, t, 1);
  float4 pv[4], mv[4], vv[4];
  int64_t ee[4];
  bool ok[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int f = q * 256 + tid, row = f / C4, c4 = f % C4;
    const int n = blockIdx.y * (1024 / C4) + row, k = blockIdx.x * TK + c4 * 4;
    ok[q] = n < kHid && k < kFeat;
    ee[q] = ok[q] ? int64_t(n) * kFeat + k : 0;
    pv[q] = reinterpret_cast<float4*>(p + ee[q])[0]; mv[q] = reinterpret_cast<float4*>(m + ee[q])[0]; vv[q] = reinterpret_cast<float4*>(v + ee[q])[0];
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (!ok[q]) continue;
    adam_regs(pv[q].x, mv[q].x, vv[q].x, 1e-3f, cfg, s);
    adam_regs(pv[q].y, mv[q].y, vv[q].y, 1e-3f, cfg, s);
    adam_regs(pv[q].z, mv[q].z, vv[q].z, 1e-3f, cfg, s);
    adam_regs(pv[q].w, mv[q].w, vv[q].w, 1e-3f, cfg, s);
    reinterpret_cast<float4*>(p + ee[q])[0] = pv[q]; reinterpret_cast<float4*>(m + ee[q])[0] = mv[q]; reinterpret_cast<float4*>(v + ee[q])[0] = vv[q];
    uint2 o;
    o.x = pack_bf16x2(pv[q].x, pv[q].y); o.y = pack_bf16x2(pv[q].z, pv[q].w);
    reinterpret_cast<uint2*>(sh + ee[q])[0] = o;
  }
}
// fully streaming, grid-stride float4
__global__ __launch_bounds__(256) void adam_stream(float* p, float* m, float* v, uint16_t* sh, AdamCfg cfg, const int* t, int64_t n4) {
  const AdamScal s = adam_scal(cfg, t, 1);
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n4; i += gridDim.x * 256ll) {
    float4 pv = reinterpret_cast<float4*>(p)[i], mv = reinterpret_cast<float4*>(m)[i], vv = reinterpret_cast<float4*>(v)[i];
    adam_regs(pv.x, mv.x, vv.x, 1e-3f, cfg, s);
    adam_regs(pv.y, mv.y, vv.y, 1e-3f, cfg, s);
    adam_regs(pv.z, mv.z, vv.z, 1e-3f, cfg, s);
    adam_regs(pv.w, mv.w, vv.w, 1e-3f, cfg, s);
    reinterpret_cast<float4*>(p)[i] = pv; reinterpret_cast<float4*>(m)[i] = mv; reinterpret_cast<float4*>(v)[i] = vv;
    uint2 o;
    o.x = pack_bf16x2(pv.x, pv.y); o.y = pack_bf16x2(pv.z, pv.w);
    reinterpret_cast<uint2*>(sh)[i] = o;
  }
}

template <typename F>
static float time_us(F f, int reps = 100) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a); (void)hipEventCreate(&b);
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
  const size_t nw = size_t(kHid) * kFeat;
  float *p, *m, *v; uint16_t* sh; int* t;
  P2_CHECK(hipMalloc(&p, nw * 4)); P2_CHECK(hipMalloc(&m, nw * 4)); P2_CHECK(hipMalloc(&v, nw * 4));
  P2_CHECK(hipMalloc(&sh, nw * 2)); P2_CHECK(hipMalloc(&t, 4));
  P2_CHECK(hipMemset(p, 0, nw * 4)); P2_CHECK(hipMemset(m, 0, nw * 4)); P2_CHECK(hipMemset(v, 0, nw * 4)); P2_CHECK(hipMemset(t, 0, 4));
  AdamCfg cfg{1e-3f, 0.9f, 0.999f, 1e-8f, 0.f};
  printf("mfma pattern 32x128 tiles     %7.2f us\n", time_us([&] { hipLaunchKernelGGL(adam_mfma_pattern, dim3(25, 64), dim3(256), 0, 0, p, m, v, sh, cfg, t); }));
  printf("row pattern  32x128 (coal.)   %7.2f us\n", time_us([&] { hipLaunchKernelGGL(adam_row_pattern<128>, dim3(25, 64), dim3(256), 0, 0, p, m, v, sh, cfg, t); }));
  printf("row pattern  16x256 (coal.)   %7.2f us\n", time_us([&] { hipLaunchKernelGGL(adam_row_pattern<256>, dim3(13, 128), dim3(256), 0, 0, p, m, v, sh, cfg, t); }));
  printf("row pattern   8x512 (coal.)   %7.2f us\n", time_us([&] { hipLaunchKernelGGL(adam_row_pattern<512>, dim3(7, 256), dim3(256), 0, 0, p, m, v, sh, cfg, t); }));
  printf("row pattern  4x1024 (coal.)   %7.2f us\n", time_us([&] { hipLaunchKernelGGL(adam_row_pattern<1024>, dim3(4, 512), dim3(256), 0, 0, p, m, v, sh, cfg, t); }));
  for (int g : {1024, 2048, 4096, 8192})
    printf("stream grid %5d              %7.2f us\n", g, time_us([&] { hipLaunchKernelGGL(adam_stream, dim3(g), dim3(256), 0, 0, p, m, v, sh, cfg, t, int64_t(nw / 4)); }));
  return 0;
}
