// Whole-arena fused optimizer steps (Adam / AdamW / SGD-momentum).
//
// torch.optim (and the reference's Lightning loop, cnn.py:89-91) update each
// parameter tensor with its own kernel(s).  With parameters, gradients and
// optimizer state laid out as flat arenas the full update is one streaming
// pass: float4 loads of p, g, m, v; fp32 math; float4 stores; optional bf16
// shadow copy of p for bf16 MFMA consumers (saves a separate cast kernel).
#include <cstdlib>
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

// ---------------------------------------------------------------------------
// Multi-tensor variants for mixed-precision learners.  The module's matrix
// weights are bf16 views of a shadow arena (the GEMMs read them directly, no
// per-step cast kernels) and autograd leaves each gradient in its own tensor
// (bf16 for bf16 weights, fp32 for the rest): no per-parameter grad
// accumulate / zero-fill launches.  One launch updates every tensor: a static
// chunk table maps each block to (tensor, start); the per-step table holds
// the gradient pointers (null = no grad this step: the tensor is skipped, as
// torch.optim does).  Master weights and state stay fp32 flat arenas, so
// FedAvg / gossip / checkpoints are unchanged.
// ---------------------------------------------------------------------------
P2_DEVICE void load_grad4(const void* g, bool bf, int64_t i, float (&o)[4]) {
  if (bf) {
    const uint2 u = *reinterpret_cast<const uint2*>(static_cast<const uint16_t*>(g) + i);
    o[0] = __uint_as_float(u.x << 16);
    o[1] = __uint_as_float(u.x & 0xffff0000u);
    o[2] = __uint_as_float(u.y << 16);
    o[3] = __uint_as_float(u.y & 0xffff0000u);
  } else {
    const float4 f = *reinterpret_cast<const float4*>(static_cast<const float*>(g) + i);
    o[0] = f.x; o[1] = f.y; o[2] = f.z; o[3] = f.w;
  }
}
P2_DEVICE float load_grad1(const void* g, bool bf, int64_t i) {
  return bf ? bf16_to_f32(static_cast<const uint16_t*>(g)[i]) : static_cast<const float*>(g)[i];
}

// Memory position, in a channels-last (O, kh, kw, I) tensor, of logical
// OIHW element ``i``.  32-bit math: one tensor stays below 2^31 elements.
P2_DEVICE uint32_t cl_index(uint32_t i, uint32_t C, uint32_t HW) {
  const uint32_t per_o = C * HW, o = i / per_o, r = i - o * per_o, c = r / HW, s = r - c * HW;
  return o * per_o + s * C + c;
}
// n / d by multiply-high (n < 2^31): the magic numbers are computed once per block
// (uniform), so the per-element channels-last index costs two v_mul_hi instead of
// two ~25-instruction integer divisions
struct FastDivU {
  uint32_t d, mul, shift;
};
P2_DEVICE FastDivU make_fastdiv_u(uint32_t d) {
  const uint32_t l = d <= 1 ? 0u : 32u - __clz(d - 1);
  const uint64_t mul = ((uint64_t(1) << 32) * ((uint64_t(1) << l) - d)) / d + 1;
  return FastDivU{d, uint32_t(mul), l};
}
P2_DEVICE uint32_t fdivu(uint32_t n, const FastDivU& f) { return (__umulhi(n, f.mul) + n) >> f.shift; }
P2_DEVICE uint32_t cl_index_fast(uint32_t i, uint32_t C, const FastDivU& per_o, const FastDivU& hw) {
  const uint32_t o = fdivu(i, per_o), r = i - o * per_o.d, c = fdivu(r, hw), s = r - c * hw.d;
  return o * per_o.d + s * C + c;
}
P2_DEVICE uint32_t cl_c(int64_t flags) { return uint32_t((flags >> 8) & 0xFFFFFF); }
P2_DEVICE uint32_t cl_hw(int64_t flags) { return uint32_t((flags >> 32) & 0xFFFFFF); }

// ---- channels-last chunks staged through LDS ---------------------------------
// A chunk of whole output-channel slabs covers the SAME element range in the
// OIHW state and in the (O, kh, kw, I) gradient / shadow, only permuted inside
// each slab.  So every global access can be contiguous: the gradient is read
// as 8 / 16-byte vectors into LDS (one pad word after every I-run, so the
// OIHW-order reads that follow -- I-runs apart -- hit distinct banks), the
// fp32 state is streamed in OIHW order as 16-byte vectors, and the new bf16
// weights go back through LDS to 8-byte stores.  The per-element gather /
// scatter of the fallback path below (2-byte gradient loads and shadow stores
// at channels-last positions) ran sgd_mt at 50-65 % of HBM roofline on
// ResNet-18 (profiles/r4_resnet18_steady_state.md).
constexpr int kMTClPad = kMTMaxCL + kMTMaxCL / 4;  // gradient words incl. pads (I >= 4)
struct ClStage {
  float g[kMTClPad];
  uint16_t sh[kMTMaxCL];
};
// Staged only when the chunk is whole slabs: ops.optim's layout gives whole-slab chunks
// only to tensors whose slab C x HW fits kMTMaxCL; a larger slab is cut into plain
// chunks that start mid-slab, which the slab-local permutation cannot map (gather path).
P2_DEVICE bool cl_staged(uint32_t C, uint32_t HW, int64_t len) {
  return HW > 1 && C % 4 == 0 && len <= kMTMaxCL && C * HW <= uint32_t(kMTMaxCL);
}
// LDS word of channels-last element j (one pad word per I-run of C elements)
P2_DEVICE uint32_t cl_pad(uint32_t j, const FastDivU& fc) { return j + fdivu(j, fc); }
P2_DEVICE void cl_load_grad(ClStage& st, const void* g, bool gbf, int64_t first, int len, const FastDivU& fc) {
  for (int j = threadIdx.x * 4; j < len; j += 1024) {
    float v[4];
    load_grad4(g, gbf, first + j, v);
    const uint32_t q = cl_pad(uint32_t(j), fc);  // the 4 share one I-run (I % 4 == 0)
#pragma unroll
    for (int e = 0; e < 4; ++e) st.g[q + e] = v[e];
  }
}
// channels-last position (within the chunk) of OIHW element i
P2_DEVICE uint32_t cl_local(uint32_t i, uint32_t C, const FastDivU& per_o, const FastDivU& hw) {
  const uint32_t o = fdivu(i, per_o), r = i - o * per_o.d, c = fdivu(r, hw), s = r - c * hw.d;
  return o * per_o.d + s * C + c;
}
P2_DEVICE void cl_store_shadow(const ClStage& st, uint16_t* __restrict__ sb, int len) {
  for (int j = threadIdx.x * 4; j < len; j += 1024)
    *reinterpret_cast<uint2*>(sb + j) = *reinterpret_cast<const uint2*>(st.sh + j);
}

P2_DEVICE void adam_elem(float& p, float g, float& m, float& v, const AdamParams& h) {
  if (h.weight_decay != 0.f) {
    if (h.decoupled)
      p *= (1.f - h.lr * h.weight_decay);
    else
      g = fmaf(h.weight_decay, p, g);
  }
  m = fmaf(h.beta1, m, (1.f - h.beta1) * g);
  v = fmaf(h.beta2, v, (1.f - h.beta2) * g * g);
  p = p - h.step_size * (m / (sqrtf(v) * h.inv_sqrt_bc2 + h.eps));
}

template <bool FD>
__global__ __launch_bounds__(256) void adam_mt_kernel(float* __restrict__ p, float* __restrict__ m,
                                                      float* __restrict__ v, uint16_t* __restrict__ pbf,
                                                      const MTTensor* __restrict__ tens, const int2* __restrict__ chunks,
                                                      const uint64_t* __restrict__ gptr, AdamParams h) {
  if (h.t_dev) {
    const float t = float(*h.t_dev);
    h.step_size = h.lr / (1.f - powf(h.beta1, t));
    h.inv_sqrt_bc2 = rsqrtf(1.f - powf(h.beta2, t));
  }
  __shared__ ClStage st;
  const int2 ch = chunks[blockIdx.x];
  const void* g = reinterpret_cast<const void*>(gptr[ch.x]);
  if (g == nullptr) return;
  const MTTensor T = tens[ch.x];
  const bool gbf = T.flags & kMTGradBf16, shadow = (T.flags & kMTShadow) && pbf;
  const int64_t start = ch.y;
  const int64_t len = T.n - start < T.chunk ? T.n - start : T.chunk;
  const int64_t len4 = len & ~int64_t(3);
  float* P = p + T.off + start;
  float* M = m + T.off + start;
  float* V = v + T.off + start;
  uint16_t* PB = shadow ? pbf + T.off + start : nullptr;
  if ((T.flags & kMTPermCL) && cl_staged(cl_c(T.flags), cl_hw(T.flags), len)) {
    const uint32_t C = cl_c(T.flags), HW = cl_hw(T.flags);
    const FastDivU fpo = make_fastdiv_u(C * HW), fhw = make_fastdiv_u(HW), fc = make_fastdiv_u(C);
    cl_load_grad(st, g, gbf, start, int(len), fc);
    __syncthreads();
    for (int i = threadIdx.x * 4; i < len; i += 1024) {
      float4 pp = *reinterpret_cast<float4*>(P + i), mm = *reinterpret_cast<float4*>(M + i),
             vv = *reinterpret_cast<float4*>(V + i);
      uint32_t j[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) j[e] = cl_local(uint32_t(i + e), C, fpo, fhw);
      adam_elem(pp.x, st.g[cl_pad(j[0], fc)], mm.x, vv.x, h);
      adam_elem(pp.y, st.g[cl_pad(j[1], fc)], mm.y, vv.y, h);
      adam_elem(pp.z, st.g[cl_pad(j[2], fc)], mm.z, vv.z, h);
      adam_elem(pp.w, st.g[cl_pad(j[3], fc)], mm.w, vv.w, h);
      *reinterpret_cast<float4*>(P + i) = pp;
      *reinterpret_cast<float4*>(M + i) = mm;
      *reinterpret_cast<float4*>(V + i) = vv;
      if (PB) {
        st.sh[j[0]] = f32_to_bf16(pp.x);
        st.sh[j[1]] = f32_to_bf16(pp.y);
        st.sh[j[2]] = f32_to_bf16(pp.z);
        st.sh[j[3]] = f32_to_bf16(pp.w);
      }
    }
    if (PB) {
      __syncthreads();
      cl_store_shadow(st, PB, int(len));
    }
    return;
  }
  if (T.flags & kMTPermCL) {
    // fp32 state in logical (coalesced) order; the bf16 gradient and shadow
    // are gathered / scattered at their channels-last positions (the whole
    // slab of an output channel is L2-resident while its block runs)
    const uint32_t C = cl_c(T.flags), HW = cl_hw(T.flags);
    FastDivU fpo{}, fhw{};
    if (FD) fpo = make_fastdiv_u(C * HW), fhw = make_fastdiv_u(HW);
    uint16_t* SB = shadow ? pbf + T.off : nullptr;
    // 4 elements per thread in flight (state loads + gradient gathers issued
    // together): one dependent round trip per element made this loop latency-bound
    for (int64_t i0 = threadIdx.x; i0 < len; i0 += 4 * 256) {
      float pv[4], gv[4], mv[4], vv[4];
      uint32_t j[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t i = i0 + u * 256;
        if (i < len) {
          j[u] = FD ? cl_index_fast(uint32_t(start + i), C, fpo, fhw) : cl_index(uint32_t(start + i), C, HW);
          pv[u] = P[i];
          mv[u] = M[i];
          vv[u] = V[i];
          gv[u] = load_grad1(g, gbf, j[u]);
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t i = i0 + u * 256;
        if (i < len) {
          adam_elem(pv[u], gv[u], mv[u], vv[u], h);
          P[i] = pv[u];
          M[i] = mv[u];
          V[i] = vv[u];
          if (SB) SB[j[u]] = f32_to_bf16(pv[u]);
        }
      }
    }
    return;
  }
  for (int64_t i = int64_t(threadIdx.x) * 4; i < len4; i += 256 * 4) {
    float gg[4];
    load_grad4(g, gbf, start + i, gg);
    float4 pp = *reinterpret_cast<float4*>(P + i), mm = *reinterpret_cast<float4*>(M + i),
           vv = *reinterpret_cast<float4*>(V + i);
    adam_elem(pp.x, gg[0], mm.x, vv.x, h);
    adam_elem(pp.y, gg[1], mm.y, vv.y, h);
    adam_elem(pp.z, gg[2], mm.z, vv.z, h);
    adam_elem(pp.w, gg[3], mm.w, vv.w, h);
    *reinterpret_cast<float4*>(P + i) = pp;
    *reinterpret_cast<float4*>(M + i) = mm;
    *reinterpret_cast<float4*>(V + i) = vv;
    if (PB) {
      uint2 o;
      o.x = pack_bf16x2(pp.x, pp.y);
      o.y = pack_bf16x2(pp.z, pp.w);
      *reinterpret_cast<uint2*>(PB + i) = o;
    }
  }
  for (int64_t i = len4 + threadIdx.x; i < len; i += 256) {
    adam_elem(P[i], load_grad1(g, gbf, start + i), M[i], V[i], h);
    if (PB) PB[i] = f32_to_bf16(P[i]);
  }
}

// register form (a pointer to a local would put the momentum on the stack)
P2_DEVICE float sgd_regs(float& p, float g, float& b, bool has_b, const SgdParams& h) {
  if (h.weight_decay != 0.f) g = fmaf(h.weight_decay, p, g);
  if (has_b) {
    b = h.first_step ? g : fmaf(h.momentum, b, (1.f - h.dampening) * g);
    g = h.nesterov ? fmaf(h.momentum, b, g) : b;
  }
  p = fmaf(-h.lr, g, p);
  return p;
}

P2_DEVICE float sgd_elem(float& p, float g, float* b, const SgdParams& h) {
  if (h.weight_decay != 0.f) g = fmaf(h.weight_decay, p, g);
  if (b) {
    *b = h.first_step ? g : fmaf(h.momentum, *b, (1.f - h.dampening) * g);
    g = h.nesterov ? fmaf(h.momentum, *b, g) : *b;
  }
  p = fmaf(-h.lr, g, p);
  return p;
}

template <bool FD>
__global__ __launch_bounds__(256) void sgd_mt_kernel(float* __restrict__ p, float* __restrict__ buf,
                                                     uint16_t* __restrict__ pbf, const MTTensor* __restrict__ tens,
                                                     const int2* __restrict__ chunks, const uint64_t* __restrict__ gptr,
                                                     SgdParams h) {
  __shared__ ClStage st;
  const int2 ch = chunks[blockIdx.x];
  const void* g = reinterpret_cast<const void*>(gptr[ch.x]);
  if (g == nullptr) return;
  const MTTensor T = tens[ch.x];
  const bool gbf = T.flags & kMTGradBf16, shadow = (T.flags & kMTShadow) && pbf;
  const int64_t start = ch.y;
  const int64_t len = T.n - start < T.chunk ? T.n - start : T.chunk;
  float* P = p + T.off + start;
  float* B = buf ? buf + T.off + start : nullptr;
  uint16_t* PB = shadow ? pbf + T.off + start : nullptr;
  if ((T.flags & kMTPermCL) && cl_staged(cl_c(T.flags), cl_hw(T.flags), len)) {  // see adam_mt_kernel
    const uint32_t C = cl_c(T.flags), HW = cl_hw(T.flags);
    const FastDivU fpo = make_fastdiv_u(C * HW), fhw = make_fastdiv_u(HW), fc = make_fastdiv_u(C);
    cl_load_grad(st, g, gbf, start, int(len), fc);
    __syncthreads();
    for (int i = threadIdx.x * 4; i < len; i += 1024) {
      float4 pp = *reinterpret_cast<float4*>(P + i);
      float4 bb = B ? *reinterpret_cast<float4*>(B + i) : float4{0.f, 0.f, 0.f, 0.f};
      uint32_t j[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) j[e] = cl_local(uint32_t(i + e), C, fpo, fhw);
      sgd_regs(pp.x, st.g[cl_pad(j[0], fc)], bb.x, B != nullptr, h);
      sgd_regs(pp.y, st.g[cl_pad(j[1], fc)], bb.y, B != nullptr, h);
      sgd_regs(pp.z, st.g[cl_pad(j[2], fc)], bb.z, B != nullptr, h);
      sgd_regs(pp.w, st.g[cl_pad(j[3], fc)], bb.w, B != nullptr, h);
      *reinterpret_cast<float4*>(P + i) = pp;
      if (B) *reinterpret_cast<float4*>(B + i) = bb;
      if (PB) {
        st.sh[j[0]] = f32_to_bf16(pp.x);
        st.sh[j[1]] = f32_to_bf16(pp.y);
        st.sh[j[2]] = f32_to_bf16(pp.z);
        st.sh[j[3]] = f32_to_bf16(pp.w);
      }
    }
    if (PB) {
      __syncthreads();
      cl_store_shadow(st, PB, int(len));
    }
    return;
  }
  if (T.flags & kMTPermCL) {  // gather path (4 elements per thread in flight, see adam_mt_kernel)
    const uint32_t C = cl_c(T.flags), HW = cl_hw(T.flags);
    FastDivU fpo{}, fhw{};
    if (FD) fpo = make_fastdiv_u(C * HW), fhw = make_fastdiv_u(HW);
    uint16_t* SB = shadow ? pbf + T.off : nullptr;
    for (int64_t i0 = threadIdx.x; i0 < len; i0 += 4 * 256) {
      float pv[4], gv[4], bv[4];
      uint32_t j[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t i = i0 + u * 256;
        if (i < len) {
          j[u] = FD ? cl_index_fast(uint32_t(start + i), C, fpo, fhw) : cl_index(uint32_t(start + i), C, HW);
          pv[u] = P[i];
          bv[u] = B ? B[i] : 0.f;
          gv[u] = load_grad1(g, gbf, j[u]);
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t i = i0 + u * 256;
        if (i < len) {
          const float np = sgd_regs(pv[u], gv[u], bv[u], B != nullptr, h);
          P[i] = np;
          if (B) B[i] = bv[u];
          if (SB) SB[j[u]] = f32_to_bf16(np);
        }
      }
    }
    return;
  }
  // contiguous tensors: 16-B vectors, as adam_mt_kernel
  const int64_t len4 = (reinterpret_cast<uintptr_t>(P) & 15) == 0 ? (len & ~int64_t(3)) : 0;
  for (int64_t i = int64_t(threadIdx.x) * 4; i < len4; i += 256 * 4) {
    float gg[4];
    load_grad4(g, gbf, start + i, gg);
    float4 pp = *reinterpret_cast<float4*>(P + i);
    float4 bb = B ? *reinterpret_cast<float4*>(B + i) : float4{0.f, 0.f, 0.f, 0.f};
    sgd_regs(pp.x, gg[0], bb.x, B != nullptr, h);
    sgd_regs(pp.y, gg[1], bb.y, B != nullptr, h);
    sgd_regs(pp.z, gg[2], bb.z, B != nullptr, h);
    sgd_regs(pp.w, gg[3], bb.w, B != nullptr, h);
    *reinterpret_cast<float4*>(P + i) = pp;
    if (B) *reinterpret_cast<float4*>(B + i) = bb;
    if (PB) {
      uint2 o;
      o.x = pack_bf16x2(pp.x, pp.y);
      o.y = pack_bf16x2(pp.z, pp.w);
      *reinterpret_cast<uint2*>(PB + i) = o;
    }
  }
  for (int64_t i = len4 + threadIdx.x; i < len; i += 256) {
    const float np = sgd_elem(P[i], load_grad1(g, gbf, start + i), B ? B + i : nullptr, h);
    if (PB) PB[i] = f32_to_bf16(np);
  }
}

// channels-last index by multiply-high (default) or by integer division (P2_MT_FASTDIV=0; A/B knob, read once)
static bool mt_fastdiv() {
  static const bool on = [] {
    const char* e = getenv("P2_MT_FASTDIV");
    return !e || atoi(e) != 0;
  }();
  return on;
}

void adam_mt_step(float* p, float* m, float* v, uint16_t* pbf, const MTTensor* tens, const int2* chunks,
                  int n_chunks, const uint64_t* gptr, const AdamParams& h, hipStream_t s) {
  if (n_chunks <= 0) return;
  if (mt_fastdiv())
    hipLaunchKernelGGL(adam_mt_kernel<true>, dim3(n_chunks), dim3(256), 0, s, p, m, v, pbf, tens, chunks, gptr, h);
  else
    hipLaunchKernelGGL(adam_mt_kernel<false>, dim3(n_chunks), dim3(256), 0, s, p, m, v, pbf, tens, chunks, gptr, h);
}

void sgd_mt_step(float* p, float* buf, uint16_t* pbf, const MTTensor* tens, const int2* chunks, int n_chunks,
                 const uint64_t* gptr, const SgdParams& h, hipStream_t s) {
  if (n_chunks <= 0) return;
  if (mt_fastdiv())
    hipLaunchKernelGGL(sgd_mt_kernel<true>, dim3(n_chunks), dim3(256), 0, s, p, buf, pbf, tens, chunks, gptr, h);
  else
    hipLaunchKernelGGL(sgd_mt_kernel<false>, dim3(n_chunks), dim3(256), 0, s, p, buf, pbf, tens, chunks, gptr, h);
}

}  // namespace p2
