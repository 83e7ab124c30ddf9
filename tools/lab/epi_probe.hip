// Kernel lab: what does a GEMM launch with no K loop cost on the ViT output
// shapes?  (scripts/gemm_anatomy.py: the ping-pong kernel's "no K loop" probe
// takes 12.9 us on the 6304 x 2304 qkv output where torch's fill_ of the same
// 29 MB takes 6.5 us.)  Each kernel writes a 256 x 256 bf16 tile per workgroup
// of 512 threads (or 128 x 128 per 256 threads) of C[M][N], with 132 KB of
// LDS declared like the real kernels.
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/epi_probe tools/lab/epi_probe.hip && /tmp/epi_probe
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int LDS = 256 * (256 * 2 + 16);  // the ping-pong kernel's epilogue image (132 KB)

// K0: nothing but the LDS declaration
__global__ __launch_bounds__(512) void k_empty(uint16_t* c, int M, int N, int tn) {
  __shared__ __attribute__((aligned(16))) char smem[LDS];
  if (threadIdx.x == 999) c[0] = smem[blockIdx.x];
}

// K1: stores straight from registers, 16 x 16 B per thread, the real kernels' chunk order
__global__ __launch_bounds__(512) void k_store(uint16_t* c, int M, int N, int tn) {
  __shared__ __attribute__((aligned(16))) char smem[LDS];
  const int m0 = (blockIdx.x / tn) * 256, n0 = (blockIdx.x % tn) * 256, tid = threadIdx.x;
  const uint4 v = make_uint4(tid, blockIdx.x, 0, 0);
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int chunk = q * 512 + tid, r = chunk >> 5, cc = chunk & 31;
    const int m = m0 + r, n = n0 + cc * 8;
    if (m < M && n < N) *reinterpret_cast<uint4*>(c + int64_t(m) * N + n) = v;
  }
  if (tid == 999) c[0] = smem[0];
}

// K2: the real epilogue's shape: registers -> LDS image -> barrier -> 16 x 16 B stores
__global__ __launch_bounds__(512) void k_staged(uint16_t* c, int M, int N, int tn) {
  __shared__ __attribute__((aligned(16))) char smem[LDS];
  constexpr int LROW = 256 * 2 + 16;
  const int m0 = (blockIdx.x / tn) * 256, n0 = (blockIdx.x % tn) * 256, tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63, wr = wave >> 2, wc = wave & 3;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int r = 128 * (i >> 1) + 64 * wr + 32 * (i & 1) + (lane & 31);
        const int col = 128 * j + 32 * wc + 8 * g + 4 * (lane >> 5);
        *reinterpret_cast<uint2*>(smem + r * LROW + col * 2) = make_uint2(i + tid, j + g);
      }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int chunk = q * 512 + tid, r = chunk >> 5, cc = chunk & 31;
    const int m = m0 + r, n = n0 + cc * 8;
    if (m < M && n < N) *reinterpret_cast<uint4*>(c + int64_t(m) * N + n) = *reinterpret_cast<const uint4*>(smem + r * LROW + cc * 16);
  }
}

// K3: no LDS declared, 4 workgroups of 128 x 128 per 256 threads each -- the fill-like shape
__global__ __launch_bounds__(256) void k_store128(uint16_t* c, int M, int N, int tn) {
  const int m0 = (blockIdx.x / tn) * 128, n0 = (blockIdx.x % tn) * 128, tid = threadIdx.x;
  const uint4 v = make_uint4(tid, blockIdx.x, 0, 0);
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int chunk = q * 256 + tid, r = chunk >> 4, cc = chunk & 15;
    const int m = m0 + r, n = n0 + cc * 8;
    if (m < M && n < N) *reinterpret_cast<uint4*>(c + int64_t(m) * N + n) = v;
  }
}

// K4: grid-stride fill (what a torch fill_ does)
__global__ __launch_bounds__(256) void k_fill(uint4* c, int64_t n16) {
  for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n16; i += int64_t(gridDim.x) * 256) c[i] = make_uint4(1, 2, 3, 4);
}

template <class F>
float timed(F launch, int reps) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 3; ++i) launch();
  hipDeviceSynchronize();
  hipEventRecord(a);
  for (int i = 0; i < reps; ++i) launch();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms * 1000.f / reps;
}

int main() {
  const int shapes[][2] = {{6304, 2304}, {6304, 768}, {6304, 3072}, {4096, 4096}};
  uint16_t* c;
  CK(hipMalloc(&c, size_t(6304) * 4096 * 2));
  for (auto& s : shapes) {
    const int M = s[0], N = s[1];
    const int tm = (M + 255) / 256, tn = (N + 255) / 256, g = tm * tn;
    const int tm1 = (M + 127) / 128, tn1 = (N + 127) / 128;
    const double mb = double(M) * N * 2 / 1e6;
    const int reps = 50;
    float t0 = timed([&] { hipLaunchKernelGGL(k_empty, dim3(g), dim3(512), 0, 0, c, M, N, tn); }, reps);
    float t1 = timed([&] { hipLaunchKernelGGL(k_store, dim3(g), dim3(512), 0, 0, c, M, N, tn); }, reps);
    float t2 = timed([&] { hipLaunchKernelGGL(k_staged, dim3(g), dim3(512), 0, 0, c, M, N, tn); }, reps);
    float t3 = timed([&] { hipLaunchKernelGGL(k_store128, dim3(tm1 * tn1), dim3(256), 0, 0, c, M, N, tn1); }, reps);
    const int64_t n16 = int64_t(M) * N / 8;
    float t4 = timed([&] { hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, reinterpret_cast<uint4*>(c), n16); }, reps);
    printf("C %dx%d (%.1f MB, %d tiles of 256^2): empty %.2f us | reg stores %.2f | LDS-staged %.2f | 128-tile stores (no LDS) %.2f | fill %.2f us (%.2f TB/s)\n",
           M, N, mb, g, t0, t1, t2, t3, t4, mb / t4 / 1e6 * 1e6 / 1e6);
  }
  CK(hipFree(c));
  return 0;
}
