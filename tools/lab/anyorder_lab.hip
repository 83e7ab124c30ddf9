// Does hipExtAnyOrderLaunch let a kernel overlap its predecessor on one stream
// (eagerly and inside a captured graph) on gfx950?
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);      \
      return 1;                                                            \
    }                                                                      \
  } while (0)

// bandwidth-bound: y = a*x + y over n floats
__global__ void axpy(const float4* __restrict__ x, float4* __restrict__ y, size_t n4) {
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n4; i += size_t(gridDim.x) * blockDim.x) {
    float4 a = x[i], b = y[i];
    b.x += 0.5f * a.x; b.y += 0.5f * a.y; b.z += 0.5f * a.z; b.w += 0.5f * a.w;
    y[i] = b;
  }
}
// latency-bound: a dependent chain of loads per lane
__global__ void chase(const int* __restrict__ nxt, int* __restrict__ out, int steps) {
  int j = (blockIdx.x * 64 + threadIdx.x) & 1023;
  for (int s = 0; s < steps; ++s) j = nxt[j * 1024 + (s & 1023)] & 1023;
  if (j == -1) out[0] = j;
}

template <typename F>
static float time_us(F f, hipStream_t s, int reps = 50) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 5; ++i) f();
  hipStreamSynchronize(s);
  hipEventRecord(a, s);
  for (int i = 0; i < reps; ++i) f();
  hipEventRecord(b, s);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms * 1000.f / reps;
}

int main() {
  const size_t n = 32u << 20;  // 32M floats = 128 MB each
  float *x, *y;
  int *nxt, *out;
  CK(hipMalloc(&x, n * 4));
  CK(hipMalloc(&y, n * 4));
  CK(hipMalloc(&nxt, 1024 * 1024 * 4));
  CK(hipMalloc(&out, 4));
  CK(hipMemset(x, 0, n * 4));
  CK(hipMemset(y, 0, n * 4));
  CK(hipMemset(nxt, 0, 1024 * 1024 * 4));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  const size_t n4 = n / 4;
  auto A = [&] { hipLaunchKernelGGL(axpy, dim3(2048), dim3(256), 0, s, (const float4*)x, (float4*)y, n4); };
  auto Bn = [&] { hipLaunchKernelGGL(chase, dim3(128), dim3(64), 0, s, nxt, out, 400); };
  auto Bany = [&] { hipExtLaunchKernelGGL(chase, dim3(128), dim3(64), 0, s, nullptr, nullptr, hipExtAnyOrderLaunch, nxt, out, 400); };
  printf("axpy alone          %8.2f us\n", time_us(A, s));
  printf("chase alone         %8.2f us\n", time_us(Bn, s));
  printf("axpy;chase          %8.2f us\n", time_us([&] { A(); Bn(); }, s));
  printf("axpy;chase(any)     %8.2f us\n", time_us([&] { A(); Bany(); }, s));
  // graph versions
  for (int any = 0; any < 2; ++any) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int i = 0; i < 10; ++i) {
      A();
      if (any) Bany(); else Bn();
    }
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    printf("graph axpy;chase%s %8.2f us per pair\n", any ? "(any)" : "     ",
           time_us([&] { hipGraphLaunch(ge, s); }, s, 10) / 10);
  }
  return 0;
}
