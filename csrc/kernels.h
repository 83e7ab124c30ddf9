// Host-side launch API of the p2pfl_amd HIP kernels (raw pointers + stream;
// no torch headers, so kernel files compile fast and stay reusable from C++).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace p2 {

constexpr int kMaxInputs = 16;

// out[i] = scale * (acc_in[i] + sum_j weights[j] * srcs[j][i]), fp32
// accumulation in input order (acc_in: fp32 running sum or null = 0; it may
// alias out).  Each src fp32 or bf16 (src_bf16[j]); out fp32 or bf16; k may be
// 0 (just scale acc_in) and may exceed kMaxInputs (fp32 out only).  Folding a
// set of inputs in several calls (running sum, scale on the last) gives the
// bitwise-same result as one call over all of them.
void weighted_sum(const void* const* srcs, const int* src_bf16, const float* weights, int k, const float* acc_in,
                  float scale, void* out, int out_bf16, int64_t n, hipStream_t s);

struct AdamParams {
  float lr, beta1, beta2, eps, weight_decay;
  float step_size;     // lr / (1 - beta1^t)
  float inv_sqrt_bc2;  // 1 / sqrt(1 - beta2^t)
  int decoupled;
  // multi-tensor kernel only: when set, t = *t_dev and the two bias
  // corrections above are computed on the device (graph-replayable steps)
  const int* t_dev;
};
void adam_step(float* p, const float* g, float* m, float* v, uint16_t* p_bf16, int64_t n, const AdamParams& h,
               hipStream_t s);

struct SgdParams {
  float lr, momentum, dampening, weight_decay;
  int nesterov, first_step;
};
void sgd_step(float* p, const float* g, float* buf, uint16_t* p_bf16, int64_t n, const SgdParams& h, hipStream_t s);

// Multi-tensor optimizer steps (mixed-precision learners, optim.hip).
constexpr int kMTChunk = 4096;  // elements per block (dense tensors)
constexpr int kMTMaxCL = 4608;  // elements per block of a channels-last tensor staged through LDS
                                // (whole output-channel slabs: the largest ResNet slab is 512 x 3 x 3)
constexpr int kMTGradBf16 = 1;  // gradient tensor is bf16 (else fp32)
constexpr int kMTShadow = 2;    // also write the bf16 shadow of the weight
constexpr int kMTPermCL = 4;    // grad + shadow in channels-last (O, kh, kw, I) order; fp32 state OIHW.
                                // flags bits 8..31 = I, bits 32..55 = kh * kw
// Tables built by p2pfl_amd/learning/optim.py mt_tables(): chunks are int32
// (tensor, first element) pairs; a block covers [first, first + min(chunk, n - first)).
struct MTTensor {
  int64_t off;    // element offset in the flat arenas
  int64_t n;      // elements
  int64_t flags;
  int64_t chunk;  // elements per block (kMTChunk, or whole (I, kh, kw) slabs for the LDS-staged path)
};
void adam_mt_step(float* p, float* m, float* v, uint16_t* p_bf16, const MTTensor* tens, const int2* chunks,
                  int n_chunks, const uint64_t* grad_ptrs, const AdamParams& h, hipStream_t s);
void sgd_mt_step(float* p, float* buf, uint16_t* p_bf16, const MTTensor* tens, const int2* chunks, int n_chunks,
                 const uint64_t* grad_ptrs, const SgdParams& h, hipStream_t s);

}  // namespace p2
