// Classification head of the CNN families in two launches (gfx950): global
// average pool -> Linear (N <= 64 classes) -> softmax cross-entropy, forward and
// backward.  On PyTorch-ROCm this tail is a dozen launches per training step
// (adaptive_avg_pool2d, the Linear GEMM + bias on hipBLASLt, log_softmax,
// nll_loss, their backward kernels, the bias-gradient reduction, the pooling
// broadcast) for a few KFLOP of work.
//
//   forward  (grid B): workgroup b pools sample b's [HW][C] channels-last feature
//            map in fp32, computes its N logits (per-thread channel partials,
//            fixed-order LDS reduction), its log-sum-exp loss and argmax hit; the
//            last workgroup to arrive (relaxed ticket, sc1 partials) writes the
//            batch-mean loss and accuracy in fixed sample order.
//   backward (grid B + ceil(N C / 256)): workgroup b < B writes dF[b] =
//            (dL/dlogits_b . W) / HW broadcast over its HW pixels (bf16,
//            channels-last); the others compute dW = dlogits^T pooled, one element
//            per thread, and db = column sums of dlogits.
//
// The reference's heads: nn.Linear + CrossEntropyLoss in
// /root/reference/p2pfl/learning/pytorch/mnist_examples/models/cnn.py:71-98.
#include "common.h"
#include <cstdlib>

namespace p2head {
using namespace p2;

constexpr int kT = 256;
constexpr int kMaxN = 64;

template <typename TW>
P2_DEVICE float ldw(const TW* w, int64_t i);
template <>
P2_DEVICE float ldw<float>(const float* w, int64_t i) { return w[i]; }
template <>
P2_DEVICE float ldw<uint16_t>(const uint16_t* w, int64_t i) { return bf16_to_f32(w[i]); }

// 8 consecutive weights as fp32 (16-B aligned: C % 8 == 0)
template <typename TW>
P2_DEVICE void ldw8(const TW* w, int64_t i, float (&o)[8]);
template <>
P2_DEVICE void ldw8<float>(const float* w, int64_t i, float (&o)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(w + i), b = *reinterpret_cast<const float4*>(w + i + 4);
  o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w;
  o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
}
template <>
P2_DEVICE void ldw8<uint16_t>(const uint16_t* w, int64_t i, float (&o)[8]) {
  const uint4 u = *reinterpret_cast<const uint4*>(w + i);
  const uint32_t x[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    o[2 * j] = __uint_as_float(x[j] << 16);
    o[2 * j + 1] = __uint_as_float(x[j] & 0xffff0000u);
  }
}
P2_DEVICE void add8(float (&q)[8], uint4 u) {
  const uint32_t x[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    q[2 * j] += __uint_as_float(x[j] << 16);
    q[2 * j + 1] += __uint_as_float(x[j] & 0xffff0000u);
  }
}

P2_DEVICE void st_sc1f(float* p, float v) {
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(p, 0, 4, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rs, 0, 0, 16);
}
P2_DEVICE float ld_sc1f(const float* p) {
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), 0, 4, 0x00020000);
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, 0, 0, 16));
}

// f: [B][HW][C] bf16; w: [N][C]; bias [N] fp32 (or null); y [B] int64 (or null: logits only)
template <typename TW>
__global__ __launch_bounds__(kT) void head_fwd_kernel(const uint16_t* __restrict__ f, const TW* __restrict__ w,
                                                      const float* __restrict__ bias, const int64_t* __restrict__ y,
                                                      float* __restrict__ pooled, float* __restrict__ logits,
                                                      float* __restrict__ loss_rows, float* __restrict__ loss_out, float* __restrict__ acc_out,
                                                      int* __restrict__ ctr, int B, int HW, int C, int N, int vec) {
  __shared__ float red[kMaxN][kT / 64];
  __shared__ float lg[kMaxN];
  __shared__ int last;
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float inv = 1.f / float(HW);
  float part[kMaxN];
#pragma unroll
  for (int n = 0; n < kMaxN; ++n) part[n] = 0.f;
  const uint16_t* fb = f + int64_t(b) * HW * C;
  if (vec == 2) {
    // narrow features (C / 8 divides the 256 threads): G channel groups x P pixel phases, so
    // every wave loads -- phase ph sums pixels ph, ph + P, ... of 8 channels (16-B loads, all in
    // flight), the P phase sums are combined in LDS in fixed order by the phase-0 threads
    __shared__ float psum[kT * 8];
    const int G = C / 8, P = kT / G, g = tid % G, ph = tid / G;
    float q[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int p = ph; p < HW; p += P) add8(q, *reinterpret_cast<const uint4*>(fb + int64_t(p) * C + g * 8));
#pragma unroll
    for (int j = 0; j < 8; ++j) psum[(ph * G + g) * 8 + j] = q[j];
    __syncthreads();
    if (ph == 0) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float t = 0.f;
        for (int k = 0; k < P; ++k) t += psum[(k * G + g) * 8 + j];
        q[j] = t * inv;
      }
      float4* pd = reinterpret_cast<float4*>(pooled + int64_t(b) * C + g * 8);
      pd[0] = make_float4(q[0], q[1], q[2], q[3]);
      pd[1] = make_float4(q[4], q[5], q[6], q[7]);
#pragma unroll
      for (int n = 0; n < kMaxN; ++n)
        if (n < N) {
          float wv[8];
          ldw8<TW>(w, int64_t(n) * C + g * 8, wv);
#pragma unroll
          for (int j = 0; j < 8; ++j) part[n] = fmaf(q[j], wv[j], part[n]);
        }
    }
  } else if (vec) {
    // 8 consecutive channels per thread, 16-B loads: a pixel's 8 channels in one load and
    // 8 pixels' loads in flight together (one channel per thread per iteration took a
    // dependent round trip per channel group: 53 us at ResNet-50's C = 2048)
    for (int c8 = tid * 8; c8 < C; c8 += kT * 8) {
      float q[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      int p = 0;
      for (; p + 8 <= HW; p += 8) {
        uint4 u[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) u[k] = *reinterpret_cast<const uint4*>(fb + int64_t(p + k) * C + c8);
#pragma unroll
        for (int k = 0; k < 8; ++k) add8(q, u[k]);
      }
      for (; p < HW; ++p) add8(q, *reinterpret_cast<const uint4*>(fb + int64_t(p) * C + c8));
#pragma unroll
      for (int j = 0; j < 8; ++j) q[j] *= inv;
      float4* pd = reinterpret_cast<float4*>(pooled + int64_t(b) * C + c8);
      pd[0] = make_float4(q[0], q[1], q[2], q[3]);
      pd[1] = make_float4(q[4], q[5], q[6], q[7]);
#pragma unroll
      for (int n = 0; n < kMaxN; ++n)
        if (n < N) {
          float wv[8];
          ldw8<TW>(w, int64_t(n) * C + c8, wv);
#pragma unroll
          for (int j = 0; j < 8; ++j) part[n] = fmaf(q[j], wv[j], part[n]);
        }
    }
  } else
  for (int c = tid; c < C; c += kT) {
    // 8 independent partial sums: the pixel loads of one channel are all in flight
    // at once instead of one dependent L2 round trip per pixel (HW = 16..49)
    float q[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    int p = 0;
    for (; p + 8 <= HW; p += 8) {
#pragma unroll
      for (int u = 0; u < 8; ++u) q[u] += bf16_to_f32(fb[int64_t(p + u) * C + c]);
    }
    for (int u = 0; p < HW; ++p, ++u) q[u] += bf16_to_f32(fb[int64_t(p) * C + c]);
    float s = ((q[0] + q[1]) + (q[2] + q[3])) + ((q[4] + q[5]) + (q[6] + q[7]));
    s *= inv;
    pooled[int64_t(b) * C + c] = s;
#pragma unroll
    for (int n = 0; n < kMaxN; ++n)
      if (n < N) part[n] = fmaf(s, ldw<TW>(w, int64_t(n) * C + c), part[n]);
  }
  // fixed-order reduction: wave sums, then the 4 waves in order
#pragma unroll
  for (int n = 0; n < kMaxN; ++n) {
    if (n < N) {  // (no early exit: keeps the loop unrolled and part[] in registers)
      const float v = wave_sum(part[n]);
      if (lane == 0) red[n][wave] = v;
    }
  }
  __syncthreads();
  if (tid < N) {
    float z = red[tid][0] + red[tid][1] + red[tid][2] + red[tid][3];
    if (bias) z += bias[tid];
    lg[tid] = z;
    logits[int64_t(b) * N + tid] = z;
  }
  __syncthreads();
  if (!y) return;
  if (tid == 0) {
    float mx = lg[0];
    int arg = 0;
    for (int n = 1; n < N; ++n)
      if (lg[n] > mx) {
        mx = lg[n];
        arg = n;
      }
    float se = 0.f;
    for (int n = 0; n < N; ++n) se += __expf(lg[n] - mx);
    // a label outside [0, N) (F.cross_entropy raises; ignore_index is not
    // supported here) makes the loss NaN instead of a finite wrong value
    const int64_t yl = y[b];
    const bool ok = yl >= 0 && yl < N;
    const int yy = ok ? int(yl) : 0;
    const float lv = ok ? (logf(se) + mx) - lg[yy] : __builtin_nanf("");
    st_sc1f(loss_rows + b, lv);
    st_sc1f(loss_rows + B + b, arg == yy ? 1.f : 0.f);
  }
  // last arrival writes [mean loss, accuracy] in sample order
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const int old = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = old == B - 1;
    if (last) __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!last || tid != 0) return;
  float sl = 0.f, sa = 0.f;
  for (int i = 0; i < B; ++i) {
    sl += ld_sc1f(loss_rows + i);
    sa += ld_sc1f(loss_rows + B + i);
  }
  loss_out[0] = sl / float(B);
  acc_out[0] = sa / float(B);
}

// dl[n] of sample b: (softmax(logits_b)[n] - [n == y_b]) * gscale
P2_DEVICE void dlogits(const float* lg, int64_t yl, int N, float gscale, float* dl) {
  if (yl < 0 || yl >= N) {  // out-of-range label: NaN gradient, never a silently wrong one
    for (int n = 0; n < N; ++n) dl[n] = __builtin_nanf("");
    return;
  }
  const int yy = int(yl);
  float mx = lg[0];
  for (int n = 1; n < N; ++n) mx = fmaxf(mx, lg[n]);
  float se = 0.f;
  for (int n = 0; n < N; ++n) se += __expf(lg[n] - mx);
  const float r = 1.f / se;
  for (int n = 0; n < N; ++n) dl[n] = (__expf(lg[n] - mx) * r - (n == yy ? 1.f : 0.f)) * gscale;
}

template <typename TW>
__global__ __launch_bounds__(kT) void head_bwd_kernel(const float* __restrict__ gloss, const float* __restrict__ logits,
                                                      const int64_t* __restrict__ y, const float* __restrict__ pooled,
                                                      const TW* __restrict__ w, uint16_t* __restrict__ df,
                                                      TW* __restrict__ dw, float* __restrict__ db, int B, int HW,
                                                      int C, int N, int vec) {
  __shared__ float dl[kMaxN];
  const int b = blockIdx.x, tid = threadIdx.x;
  const float gscale = gloss[0] / float(B);
  if (b < B) {
    if (tid == 0) dlogits(logits + int64_t(b) * N, y[b], N, gscale, dl);
    __syncthreads();
    const float inv = 1.f / float(HW);
    uint16_t* out = df + int64_t(b) * HW * C;
    if (vec) {  // 8 channels per thread: 16-B weight loads and 16-B pixel stores
      // (vec == 2, narrow features: G channel groups x P pixel phases, each phase storing
      // every P-th pixel of its group)
      const int G = vec == 2 ? C / 8 : kT, P = vec == 2 ? kT / G : 1;
      const int g = tid % G, ph = tid / G;
      for (int c8 = g * 8; c8 < C; c8 += G * 8) {
        float sv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int n = 0; n < kMaxN; ++n)
          if (n < N) {
            float wv[8];
            ldw8<TW>(w, int64_t(n) * C + c8, wv);
#pragma unroll
            for (int j = 0; j < 8; ++j) sv[j] = fmaf(dl[n], wv[j], sv[j]);
          }
        const uint4 v = make_uint4(pack_bf16x2(sv[0] * inv, sv[1] * inv), pack_bf16x2(sv[2] * inv, sv[3] * inv),
                                   pack_bf16x2(sv[4] * inv, sv[5] * inv), pack_bf16x2(sv[6] * inv, sv[7] * inv));
        for (int p = ph; p < HW; p += P) *reinterpret_cast<uint4*>(out + int64_t(p) * C + c8) = v;
      }
      return;
    }
    for (int c = tid; c < C; c += kT) {
      float s = 0.f;
#pragma unroll
      for (int n = 0; n < kMaxN; ++n)  // unrolled + predicated: the N weight loads issue together
        if (n < N) s = fmaf(dl[n], ldw<TW>(w, int64_t(n) * C + c), s);
      const uint16_t v = f32_to_bf16(s * inv);
      for (int p = 0; p < HW; ++p) out[int64_t(p) * C + c] = v;
    }
    return;
  }
  // workgroups B.. : one thread per dW element, dW[n][c] = sum_b dl_b[n] pooled[b][c]
  // (samples in order, loads unrolled so they are in flight together); the first
  // of them also writes db[n] = sum_b dl_b[n].  (One workgroup looping over all
  // N x C elements spent ~70 us on dependent pooled loads for ResNet-18.)
  __shared__ float dla[64][kMaxN];  // dl of up to 64 samples per chunk
  const int e = (b - B) * kT + tid;
  const int n = e / C, c = e - n * C;
  const bool live = e < N * C;
  float s = 0.f, sb = 0.f;
  for (int b0 = 0; b0 < B; b0 += 64) {
    const int nb = min(64, B - b0);
    __syncthreads();
    if (tid < nb) dlogits(logits + int64_t(b0 + tid) * N, y[b0 + tid], N, gscale, dla[tid]);
    __syncthreads();
    if (live) {
      int i = 0;
      for (; i + 8 <= nb; i += 8) {
        float pv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) pv[u] = pooled[int64_t(b0 + i + u) * C + c];
#pragma unroll
        for (int u = 0; u < 8; ++u) s = fmaf(dla[i + u][n], pv[u], s);
      }
      for (; i < nb; ++i) s = fmaf(dla[i][n], pooled[int64_t(b0 + i) * C + c], s);
    }
    if (b == B && tid < N)
      for (int i = 0; i < nb; ++i) sb += dla[i][tid];
  }
  if (live) {
    if constexpr (sizeof(TW) == 4)
      dw[e] = s;
    else
      dw[e] = f32_to_bf16(s);
  }
  if (b == B && tid < N) db[tid] = sb;
}

}  // namespace p2head

namespace p2 {

// P2PFL_HEAD_VEC=0: the scalar one-channel-per-thread loops everywhere (A/B knob)
static bool head_vec_enabled() {
  static const bool on = [] {
    const char* e = getenv("P2PFL_HEAD_VEC");
    return !(e && e[0] == '0');
  }();
  return on;
}

void head_fwd(const uint16_t* f, const void* w, int w_bf16, const float* bias, const int64_t* y, float* pooled,
              float* logits, float* loss_rows, float* loss, float* acc, int* ctr, int B, int HW, int C, int N,
              hipStream_t s) {
  using namespace p2head;
  // 16-B vector paths: whole 8-channel groups and 16-B aligned features / weights (a weight
  // inside a shadow arena need not be).  vec 1 (C >= 1024): 8 channels per thread; vec 2
  // (C / 8 divides the block): channel groups x pixel phases, so all four waves load -- with
  // 8 channels per thread alone, C = 512 (ResNet-18) left 3 of 4 waves idle and measured no
  // faster (scripts/ab_head_vec.sh)
  const bool al = head_vec_enabled() && C % 8 == 0 && reinterpret_cast<uintptr_t>(f) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(w) % 16 == 0 && reinterpret_cast<uintptr_t>(pooled) % 16 == 0;
  const int vec = !al ? 0 : (C >= 1024 ? 1 : (C >= 64 && kT % (C / 8) == 0 ? 2 : 0));
  if (w_bf16)
    hipLaunchKernelGGL(head_fwd_kernel<uint16_t>, dim3(B), dim3(kT), 0, s, f, static_cast<const uint16_t*>(w), bias, y,
                       pooled, logits, loss_rows, loss, acc, ctr, B, HW, C, N, vec);
  else
    hipLaunchKernelGGL(head_fwd_kernel<float>, dim3(B), dim3(kT), 0, s, f, static_cast<const float*>(w), bias, y,
                       pooled, logits, loss_rows, loss, acc, ctr, B, HW, C, N, vec);
}

void head_bwd(const float* gloss, const float* logits, const int64_t* y, const float* pooled, const void* w, int w_bf16,
              uint16_t* df, void* dw, float* db, int B, int HW, int C, int N, hipStream_t s) {
  using namespace p2head;
  const bool al = head_vec_enabled() && C % 8 == 0 && reinterpret_cast<uintptr_t>(df) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(w) % 16 == 0;
  const int vec = !al ? 0 : (C >= 1024 ? 1 : (C >= 64 && kT % (C / 8) == 0 ? 2 : 0));
  if (w_bf16)
    hipLaunchKernelGGL(head_bwd_kernel<uint16_t>, dim3(B + (N * C + kT - 1) / kT), dim3(kT), 0, s, gloss, logits, y, pooled,
                       static_cast<const uint16_t*>(w), df, static_cast<uint16_t*>(dw), db, B, HW, C, N, vec);
  else
    hipLaunchKernelGGL(head_bwd_kernel<float>, dim3(B + (N * C + kT - 1) / kT), dim3(kT), 0, s, gloss, logits, y, pooled,
                       static_cast<const float*>(w), df, static_cast<float*>(dw), db, B, HW, C, N, vec);
}

}  // namespace p2
