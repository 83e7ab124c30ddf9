// Kernel lab: times variants of the dA1/route kernel in isolation to locate
// where its time goes (launch floor, loads, MFMA, epilogue, extra FC2 blocks).
// Standalone (no torch):  hipcc -O3 --offload-arch=gfx950 -Icsrc tools/lab/route_lab.hip -o /tmp/route_lab
#include "../../csrc/cnn_bwd.hip"
namespace p2cnn {
void init_fwd_attributes() {}
}

#include <cstdio>
#include <vector>

using namespace p2cnn;

__global__ void noop_kernel(int* p) {
  if (p && threadIdx.x == 9999) p[0] = 1;
}

// route body, variant flags: LOADS (1 = issue W1T/dH loads), MFMA, EPI (0 none, 1 gb only, 2 full)
template <int EPI, bool NT>
__global__ __launch_bounds__(512) void route_var(const uint16_t* __restrict__ dH, const uint16_t* __restrict__ w1t,
                                                 const uint8_t* __restrict__ am2, int B, uint16_t* __restrict__ dc2m,
                                                 float* __restrict__ gb) {
  __shared__ float red[8 * 1024];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const int n0 = blockIdx.x * 32;
  constexpr int K = kHid, NG = K / 64, NGW = NG / 8;
  f32x16 acc = {};
  const uint16_t* brow = w1t + size_t(n0 + r) * K + 32 * h;
  uint4 bq[NGW][4], aq[NGW][4];
#pragma unroll
  for (int gi = 0; gi < NGW; ++gi) {
    const int k0 = (wave + 8 * gi) * 64;
#pragma unroll
    for (int q = 0; q < 4; ++q) bq[gi][q] = NT ? ld_nt16(brow + k0 + q * 8) : *reinterpret_cast<const uint4*>(brow + k0 + q * 8);
#pragma unroll
    for (int q = 0; q < 4; ++q) aq[gi][q] = reinterpret_cast<const uint4*>(dH + size_t(r) * K + 32 * h + k0)[q];
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int gi = 0; gi < NGW; ++gi)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc = mfma32b(aq[gi][q], bq[gi][q], acc);
#pragma unroll
  for (int i = 0; i < 16; ++i) red[(wave * 16 + i) * 64 + lane] = acc[i];
  __syncthreads();
  for (int e = tid; e < 1024; e += 512) {
    float g = 0.f;
#pragma unroll
    for (int w = 0; w < 8; ++w) g += red[w * 1024 + e];
    const int i = (e >> 6) & 15, ln = e & 63;
    const int b = acc_row_b(i, ln >> 5), feat = n0 + (ln & 31);
    if (b >= B) continue;
    if (EPI == 0) {
      if (g == 12345.f) gb[0] = g;
      continue;
    }
    if (EPI == 1) {
      gb[size_t(b) * kFeat + feat] = g;
      continue;
    }
    const uint8_t a = am2[size_t(b) * kFeat + feat];
    const int oc = feat / 49, pp = feat % 49, py = pp / 7, px = pp % 7;
    gb[size_t(b) * kFeat + feat] = a < 4 ? g : 0.f;
    const uint16_t gv = f32_to_bf16(g);
    uint16_t* row = dc2m + (size_t(b) * kC2 + oc) * 224 + (2 * py) * 16 + 2 * px;
    const uint32_t top = (a == 0 ? gv : 0u) | (uint32_t(a == 1 ? gv : 0u) << 16);
    const uint32_t bot = (a == 2 ? gv : 0u) | (uint32_t(a == 3 ? gv : 0u) << 16);
    *reinterpret_cast<uint32_t*>(row) = top;
    *reinterpret_cast<uint32_t*>(row + 16) = bot;
  }
}

// split-K variant: grid (98, S); each block reduces over K/S and writes fp32 partial slabs
template <int S>
__global__ __launch_bounds__(256) void route_splitk(const uint16_t* __restrict__ dH, const uint16_t* __restrict__ w1t,
                                                    float* __restrict__ slabs) {
  __shared__ float red[4 * 1024];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const int n0 = blockIdx.x * 32, sp = blockIdx.y;
  constexpr int NG = kHid / 64 / S;  // groups per split
  constexpr int NGW = NG / 4;
  f32x16 acc = {};
  const uint16_t* brow = w1t + size_t(n0 + r) * kHid + 32 * h;
  uint4 bq[NGW][4], aq[NGW][4];
#pragma unroll
  for (int gi = 0; gi < NGW; ++gi) {
    const int k0 = (sp * NG + wave + 4 * gi) * 64;
#pragma unroll
    for (int q = 0; q < 4; ++q) bq[gi][q] = ld_nt16(brow + k0 + q * 8);
#pragma unroll
    for (int q = 0; q < 4; ++q) aq[gi][q] = reinterpret_cast<const uint4*>(dH + size_t(r) * kHid + 32 * h + k0)[q];
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int gi = 0; gi < NGW; ++gi)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc = mfma32b(aq[gi][q], bq[gi][q], acc);
#pragma unroll
  for (int i = 0; i < 16; ++i) red[(wave * 16 + i) * 64 + lane] = acc[i];
  __syncthreads();
  for (int e = tid; e < 1024; e += 256) {
    const float g = (red[e] + red[1024 + e]) + (red[2048 + e] + red[3072 + e]);
    const int i = (e >> 6) & 15, ln = e & 63;
    slabs[(size_t(sp) * 32 + acc_row_b(i, ln >> 5)) * kFeat + n0 + (ln & 31)] = g;
  }
}

template <typename F>
static float time_us(F f, int reps = 200) {
  hipEvent_t a, b;
  P2_CHECK(hipEventCreate(&a));
  P2_CHECK(hipEventCreate(&b));
  for (int i = 0; i < 10; ++i) f();
  P2_CHECK(hipDeviceSynchronize());
  P2_CHECK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) f();
  P2_CHECK(hipEventRecord(b));
  P2_CHECK(hipEventSynchronize(b));
  float ms = 0.f;
  P2_CHECK(hipEventElapsedTime(&ms, a, b));
  return ms * 1000.f / reps;
}

int main() {
  const int B = 32;
  uint16_t *dH, *w1t, *dc2m, *H;
  uint8_t* am2;
  float *gb, *slabs, *dlog, *p, *m, *v;
  int* adam_t;
  P2_CHECK(hipMalloc(&dH, 32 * kHid * 2));
  P2_CHECK(hipMalloc(&w1t, size_t(kFeat) * kHid * 2));
  P2_CHECK(hipMalloc(&dc2m, 32 * 64 * 224 * 2));
  P2_CHECK(hipMalloc(&H, 32 * kHid * 2));
  P2_CHECK(hipMalloc(&am2, 32 * kFeat));
  P2_CHECK(hipMalloc(&gb, 32 * kFeat * 4));
  P2_CHECK(hipMalloc(&slabs, 8 * 32 * kFeat * 4));
  P2_CHECK(hipMalloc(&dlog, 32 * 10 * 4));
  const size_t np = 6600000;
  P2_CHECK(hipMalloc(&p, np * 4));
  P2_CHECK(hipMalloc(&m, np * 4));
  P2_CHECK(hipMalloc(&v, np * 4));
  P2_CHECK(hipMalloc(&adam_t, 4));
  P2_CHECK(hipMemset(dH, 0, 32 * kHid * 2));
  P2_CHECK(hipMemset(w1t, 0, size_t(kFeat) * kHid * 2));
  P2_CHECK(hipMemset(am2, 1, 32 * kFeat));
  P2_CHECK(hipMemset(H, 0, 32 * kHid * 2));
  P2_CHECK(hipMemset(dlog, 0, 32 * 40));
  P2_CHECK(hipMemset(p, 0, np * 4));
  P2_CHECK(hipMemset(m, 0, np * 4));
  P2_CHECK(hipMemset(v, 0, np * 4));
  P2_CHECK(hipMemset(adam_t, 0, 4));
  Offsets off{0, 800, 832, 52032, 52096, 6474816, 6476864, 6497344};
  AdamCfg cfg{1e-3f, 0.9f, 0.999f, 1e-8f, 0.f};
  hipStream_t s = nullptr;
  printf("noop 1 block        %7.2f us\n", time_us([&] { hipLaunchKernelGGL(noop_kernel, dim3(1), dim3(64), 0, s, nullptr); }));
  printf("noop 98x512         %7.2f us\n", time_us([&] { hipLaunchKernelGGL(noop_kernel, dim3(98), dim3(512), 0, s, nullptr); }));
  printf("noop 1600x256       %7.2f us\n", time_us([&] { hipLaunchKernelGGL(noop_kernel, dim3(1600), dim3(256), 0, s, nullptr); }));
  printf("route_fc2 (prod)    %7.2f us\n", time_us([&] { route_fc2(dH, w1t, am2, 32, B, dc2m, gb, dlog, H, p, m, v, nullptr, off, adam_t, 1, cfg, s); }));
  printf("route epi=full nt   %7.2f us\n", time_us([&] { hipLaunchKernelGGL((route_var<2, true>), dim3(98), dim3(512), 0, s, dH, w1t, am2, B, dc2m, gb); }));
  printf("route epi=full      %7.2f us\n", time_us([&] { hipLaunchKernelGGL((route_var<2, false>), dim3(98), dim3(512), 0, s, dH, w1t, am2, B, dc2m, gb); }));
  printf("route epi=gb        %7.2f us\n", time_us([&] { hipLaunchKernelGGL((route_var<1, true>), dim3(98), dim3(512), 0, s, dH, w1t, am2, B, dc2m, gb); }));
  printf("route epi=none      %7.2f us\n", time_us([&] { hipLaunchKernelGGL((route_var<0, true>), dim3(98), dim3(512), 0, s, dH, w1t, am2, B, dc2m, gb); }));
  printf("route splitK=2      %7.2f us\n", time_us([&] { hipLaunchKernelGGL((route_splitk<2>), dim3(98, 2), dim3(256), 0, s, dH, w1t, slabs); }));
  printf("route splitK=4      %7.2f us\n", time_us([&] { hipLaunchKernelGGL((route_splitk<4>), dim3(98, 4), dim3(256), 0, s, dH, w1t, slabs); }));
  printf("route splitK=8      %7.2f us\n", time_us([&] { hipLaunchKernelGGL((route_splitk<8>), dim3(98, 8), dim3(256), 0, s, dH, w1t, slabs); }));
  // graph of 20 back-to-back noops: per-node cost inside a graph
  {
    hipGraph_t g;
    hipGraphExec_t ge;
    hipStream_t cs;
    P2_CHECK(hipStreamCreate(&cs));
    P2_CHECK(hipStreamBeginCapture(cs, hipStreamCaptureModeGlobal));
    for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(noop_kernel, dim3(98), dim3(512), 0, cs, nullptr);
    P2_CHECK(hipStreamEndCapture(cs, &g));
    P2_CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    printf("graph noop per node %7.2f us\n", time_us([&] { P2_CHECK(hipGraphLaunch(ge, cs)); }, 50) / 20);
    P2_CHECK(hipStreamBeginCapture(cs, hipStreamCaptureModeGlobal));
    for (int i = 0; i < 20; ++i)
      hipLaunchKernelGGL((route_var<2, true>), dim3(98), dim3(512), 0, cs, dH, w1t, am2, B, dc2m, gb);
    P2_CHECK(hipStreamEndCapture(cs, &g));
    P2_CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    printf("graph route per node%7.2f us\n", time_us([&] { P2_CHECK(hipGraphLaunch(ge, cs)); }, 50) / 20);
  }
  return 0;
}
