// Kernel lab: conv2_bwd roles timed separately (dgrad: per-wave w2q streaming
// from L2; wgrad).   hipcc -O3 --offload-arch=gfx950 -Icsrc tools/lab/conv_lab.hip
#include "../../csrc/cnn_bwd.hip"
namespace p2cnn { void init_fwd_attributes() {} }
#include <cstdio>
using namespace p2cnn;

__global__ __launch_bounds__(256) void dgrad_only(const uint16_t* dc2m, const uint8_t* am1, const uint16_t* w2q, const uint8_t* x,
                                                  float* wslab1) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  conv2_dgrad_block(blockIdx.x & 1, blockIdx.x >> 1, dc2m, am1, w2q, x, nullptr, wslab1, smem);
}
__global__ __launch_bounds__(64) void wgrad_only(const uint16_t* dc2m, const uint16_t* p1s, float* wslab2, int B) {
  conv2_wgrad_role(blockIdx.x % kTaps, blockIdx.x / kTaps, dc2m, p1s, wslab2, B);
}

template <typename F>
static float time_us(F f, int reps = 200) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a); (void)hipEventCreate(&b);
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
  const int B = 32;
  uint16_t *dc2m, *w2q, *p1s; uint8_t *am1, *x; float *ws1, *ws2;
  P2_CHECK(hipMalloc(&dc2m, B * 64 * 224 * 2)); P2_CHECK(hipMalloc(&w2q, 51200 * 2)); P2_CHECK(hipMalloc(&p1s, size_t(B) * kP1s * 2));
  P2_CHECK(hipMalloc(&am1, B * 196 * 32)); P2_CHECK(hipMalloc(&x, B * 784)); P2_CHECK(hipMalloc(&ws1, B * 7 * 832 * 4)); P2_CHECK(hipMalloc(&ws2, 16 * 51200 * 4));
  P2_CHECK(hipMemset(dc2m, 0, B * 64 * 224 * 2)); P2_CHECK(hipMemset(w2q, 0, 51200 * 2)); P2_CHECK(hipMemset(p1s, 0, size_t(B) * kP1s * 2));
  P2_CHECK(hipMemset(am1, 1, B * 196 * 32)); P2_CHECK(hipMemset(x, 3, B * 784));
  printf("conv2_bwd (both roles)   %7.2f us\n", time_us([&] { conv2_bwd(dc2m, p1s, am1, w2q, x, nullptr, ws1, ws2, B, 0); }));
  P2_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(dgrad_only), hipFuncAttributeMaxDynamicSharedMemorySize, kDgLds));
  init_attributes();
  printf("dgrad blocks only (2B)   %7.2f us\n", time_us([&] { hipLaunchKernelGGL(dgrad_only, dim3(2 * B), dim3(256), kDgLds, 0, dc2m, am1, w2q, x, ws1); }));
  printf("wgrad role only (400)    %7.2f us\n", time_us([&] { hipLaunchKernelGGL(wgrad_only, dim3(kTaps * 16), dim3(64), 0, 0, dc2m, p1s, ws2, B); }));
  return 0;
}
