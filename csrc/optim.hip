// Whole-arena fused optimizer steps (Adam / AdamW / SGD-momentum).
//
// torch.optim (and the reference's Lightning loop, cnn.py:89-91) update each
// parameter tensor with its own kernel(s).  With parameters, gradients and
// optimizer state laid out as flat arenas the full update is one streaming
// pass: float4 loads of p, g, m, v; fp32 math; float4 stores; optional bf16
// shadow copy of p for bf16 MFMA consumers (saves a separate cast kernel).
#include "common.h"
#include "kernels.h"

namespace p2 {

__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v,
                                                   uint16_t* __restrict__ pbf, int64_t n4, AdamParams h) {
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 pp = reinterpret_cast<float4*>(p)[i];
    float4 gg = reinterpret_cast<const float4*>(g)[i];
    float4 mm = reinterpret_cast<float4*>(m)[i];
    float4 vv = reinterpret_cast<float4*>(v)[i];
    float* P = &pp.x;
    float* G = &gg.x;
    float* M = &mm.x;
    float* V = &vv.x;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float gj = G[j];
      if (h.weight_decay != 0.f) {
        if (h.decoupled)
          P[j] *= (1.f - h.lr * h.weight_decay);
        else
          gj = fmaf(h.weight_decay, P[j], gj);
      }
      M[j] = fmaf(h.beta1, M[j], (1.f - h.beta1) * gj);
      V[j] = fmaf(h.beta2, V[j], (1.f - h.beta2) * gj * gj);
      const float denom = sqrtf(V[j]) * h.inv_sqrt_bc2 + h.eps;
      P[j] = P[j] - h.step_size * (M[j] / denom);
    }
    reinterpret_cast<float4*>(p)[i] = pp;
    reinterpret_cast<float4*>(m)[i] = mm;
    reinterpret_cast<float4*>(v)[i] = vv;
    if (pbf) {
      uint2 o;
      o.x = pack_bf16x2(pp.x, pp.y);
      o.y = pack_bf16x2(pp.z, pp.w);
      reinterpret_cast<uint2*>(pbf)[i] = o;
    }
  }
}

__global__ __launch_bounds__(256) void sgd_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                  float* __restrict__ buf, uint16_t* __restrict__ pbf,
                                                  int64_t n4, SgdParams h) {
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 pp = reinterpret_cast<float4*>(p)[i];
    float4 gg = reinterpret_cast<const float4*>(g)[i];
    float4 bb = buf ? reinterpret_cast<float4*>(buf)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    float* P = &pp.x;
    float* G = &gg.x;
    float* B = &bb.x;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float d = G[j];
      if (h.weight_decay != 0.f) d = fmaf(h.weight_decay, P[j], d);
      if (buf) {
        B[j] = h.first_step ? d : fmaf(h.momentum, B[j], (1.f - h.dampening) * d);
        d = h.nesterov ? fmaf(h.momentum, B[j], d) : B[j];
      }
      P[j] = fmaf(-h.lr, d, P[j]);
    }
    reinterpret_cast<float4*>(p)[i] = pp;
    if (buf) reinterpret_cast<float4*>(buf)[i] = bb;
    if (pbf) {
      uint2 o;
      o.x = pack_bf16x2(pp.x, pp.y);
      o.y = pack_bf16x2(pp.z, pp.w);
      reinterpret_cast<uint2*>(pbf)[i] = o;
    }
  }
}

void adam_step(float* p, const float* g, float* m, float* v, uint16_t* pbf, int64_t n, const AdamParams& h,
               hipStream_t s) {
  const int64_t n4 = n / 4;  // arenas are padded to 64 elements
  hipLaunchKernelGGL(adam_kernel, dim3(stream_grid(n4, 256)), dim3(256), 0, s, p, g, m, v, pbf, n4, h);
}

void sgd_step(float* p, const float* g, float* buf, uint16_t* pbf, int64_t n, const SgdParams& h, hipStream_t s) {
  const int64_t n4 = n / 4;
  hipLaunchKernelGGL(sgd_kernel, dim3(stream_grid(n4, 256)), dim3(256), 0, s, p, g, buf, pbf, n4, h);
}

}  // namespace p2
