// Fused BatchNorm (+ residual add) (+ ReLU) for MI355X (gfx950, wave64), on
// channels-last activations viewed as [M, C] (M = N*H*W rows of C channels).
//
// What it replaces in a ResNet block (PyTorch-ROCm, NHWC bf16):
//   forward   MIOpen BN training kernel(s) + residual add + ReLU     (3+ passes)
//   backward  ReLU threshold_backward + MIOpen BN backward           (3+ passes)
// Here, per BN:
//   forward   stats (1 read of x)  -> finalize (C threads) -> apply (read x [+res], write y)
//   backward  stats (read dy, y, x) -> finalize              -> apply (read dy, y, x, write dx [+dres])
//
// Column statistics: every thread owns 8 consecutive channels (one 16-B bf16
// load per row), a 256-thread block covers `tpr` threads per row x `rp` row
// phases, row splits go over gridDim.y.  Per-block sums are combined across
// row phases in LDS in fixed order and written as [S, C] partials; the
// finalize kernel reduces the S partials in fixed order (for small bf16
// activations both run as one launch, bn_stats_fin_kernel / bn_bwd_stats_fin_
// kernel, the last block to arrive doing the finalize).  No float atomics:
// results are bitwise reproducible run to run.  Forward statistics use sums
// shifted by the first row's value (x - x[0][c]) so the variance does not
// cancel for activations with a large mean.
#include "batchnorm.h"
#include "common.h"

namespace p2bn {
using namespace p2;

template <typename T>
struct V8;
template <>
struct V8<uint16_t> {
  static P2_DEVICE void load(const uint16_t* p, float (&v)[8]) {
    const uint4 u = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[2 * j] = __uint_as_float(w[j] << 16);
      v[2 * j + 1] = __uint_as_float(w[j] & 0xffff0000u);
    }
  }
  static P2_DEVICE void store(uint16_t* p, const float (&v)[8]) {
    uint4 u;
    u.x = pack_bf16x2(v[0], v[1]);
    u.y = pack_bf16x2(v[2], v[3]);
    u.z = pack_bf16x2(v[4], v[5]);
    u.w = pack_bf16x2(v[6], v[7]);
    *reinterpret_cast<uint4*>(p) = u;
  }
  static P2_DEVICE float one(const uint16_t* p) { return bf16_to_f32(*p); }
};
template <>
struct V8<float> {
  static P2_DEVICE void load(const float* p, float (&v)[8]) {
    const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
  static P2_DEVICE void store(float* p, const float (&v)[8]) {
    reinterpret_cast<float4*>(p)[0] = make_float4(v[0], v[1], v[2], v[3]);
    reinterpret_cast<float4*>(p)[1] = make_float4(v[4], v[5], v[6], v[7]);
  }
  static P2_DEVICE float one(const float* p) { return *p; }
};
P2_DEVICE void ld8f(const float* p, float (&v)[8]) { V8<float>::load(p, v); }

constexpr int kThreads = 256;
constexpr int kRedCols = kThreads * 8;  // LDS columns of one phase-reduction slab
constexpr int kInFlight = 4;             // rows per thread in flight in the statistics passes

// ---------------------------------------------------------------------------
// Block-level fixed-order reduction of two per-thread [8] accumulators over
// the rp row phases, written as row blockIdx.y of the [S, C] partials a / b.
// ---------------------------------------------------------------------------
P2_DEVICE void phase_reduce_store(float (&s1)[8], float (&s2)[8], bool active, int tg, int ph, int tpr, int rp,
                                  float* __restrict__ part, int C) {
  __shared__ float red[2][kRedCols];
  const int width = tpr * 8;  // columns of this block
  if (active) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[0][ph * width + tg * 8 + j] = s1[j];
      red[1][ph * width + tg * 8 + j] = s2[j];
    }
  }
  __syncthreads();
  const int S = gridDim.y;
  for (int i = threadIdx.x; i < width; i += kThreads) {
    const int c = blockIdx.x * width + i;
    if (c >= C) continue;
    float a = 0.f, b = 0.f;
    for (int p = 0; p < rp; ++p) {
      a += red[0][p * width + i];
      b += red[1][p * width + i];
    }
    part[size_t(blockIdx.y) * C + c] = a;
    part[size_t(S + blockIdx.y) * C + c] = b;
  }
}

// forward statistics: sum (x - x0) and sum (x - x0)^2 per channel
template <typename T>
__global__ __launch_bounds__(kThreads) void bn_stats_kernel(const T* __restrict__ x, float* __restrict__ part, int M,
                                                            int C, int tpr, int rp) {
  const int tg = threadIdx.x % tpr, ph = threadIdx.x / tpr;
  const int c = (blockIdx.x * tpr + tg) * 8;
  const bool active = ph < rp && c < C;
  float s1[8], s2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s1[j] = s2[j] = 0.f;
  if (active) {
    float sh[8];
    V8<T>::load(x + c, sh);
    const int step = rp * gridDim.y;
    // kInFlight rows per iteration, loaded unconditionally (rows past M re-read
    // row 0 and count zero): a load under a branch gets its own vmcnt(0), which
    // serialised the rows one memory round trip at a time
    for (int r = blockIdx.y * rp + ph; r < M; r += kInFlight * step) {
      float v[kInFlight][8];
#pragma unroll
      for (int u = 0; u < kInFlight; ++u) {
        const int ru = r + u * step;
        V8<T>::load(x + size_t(ru < M ? ru : 0) * C + c, v[u]);
      }
#pragma unroll
      for (int u = 0; u < kInFlight; ++u) {
        const bool in = r + u * step < M;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = in ? v[u][j] - sh[j] : 0.f;
          s1[j] += d;
          s2[j] = fmaf(d, d, s2[j]);
        }
      }
    }
  }
  phase_reduce_store(s1, s2, active, tg, ph, tpr, rp, part, C);
}

// backward statistics: sum dz and sum dz * (x - mean) per channel.  dy2 (or null):
// a second gradient of the same output, summed on load -- a residual block's
// input feeds two branches, and the two gradients never need an add pass
template <typename T, bool RELU>
__global__ __launch_bounds__(kThreads) void bn_bwd_stats_kernel(const T* __restrict__ dy, const T* __restrict__ dy2,
                                                                const T* __restrict__ y,
                                                                const T* __restrict__ x,
                                                                const float* __restrict__ mean,
                                                                float* __restrict__ part, int M, int C, int tpr,
                                                                int rp) {
  const int tg = threadIdx.x % tpr, ph = threadIdx.x / tpr;
  const int c = (blockIdx.x * tpr + tg) * 8;
  const bool active = ph < rp && c < C;
  float s1[8], s2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s1[j] = s2[j] = 0.f;
  if (active) {
    float mu[8];
    ld8f(mean + c, mu);
    const int step = rp * gridDim.y;
    // kInFlight rows per iteration, loads unconditional (see bn_stats_kernel)
    for (int r = blockIdx.y * rp + ph; r < M; r += kInFlight * step) {
      float g[kInFlight][8], xv[kInFlight][8], yv[kInFlight][8];
#pragma unroll
      for (int u = 0; u < kInFlight; ++u) {
        const int ru = r + u * step;
        const size_t e = size_t(ru < M ? ru : 0) * C + c;
        V8<T>::load(dy + e, g[u]);
        V8<T>::load(x + e, xv[u]);
        if (RELU) V8<T>::load(y + e, yv[u]);
      }
      if (dy2) {
#pragma unroll
        for (int u = 0; u < kInFlight; ++u) {
          const int ru = r + u * step;
          float g2[8];
          V8<T>::load(dy2 + size_t(ru < M ? ru : 0) * C + c, g2);
#pragma unroll
          for (int j = 0; j < 8; ++j) g[u][j] += g2[j];
        }
      }
#pragma unroll
      for (int u = 0; u < kInFlight; ++u) {
        const bool in = r + u * step < M;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float gg = in && (!RELU || yv[u][j] > 0.f) ? g[u][j] : 0.f;
          s1[j] += gg;
          s2[j] = fmaf(gg, xv[u][j] - mu[j], s2[j]);
        }
      }
    }
  }
  phase_reduce_store(s1, s2, active, tg, ph, tpr, rp, part, C);
}

// ---------------------------------------------------------------------------
// Finalize: block = 16 channels x 16 partial-row phases, 8 rows in flight per
// thread (two arrays), then a fixed-order sum over the phases in LDS.  The
// S <= 256 partial rows are read in <= 2 rounds of memory latency (the
// earlier 64 x 4 split needed up to 16 dependent rounds: 5.5 us per call).
// ---------------------------------------------------------------------------
constexpr int kFinCols = 16, kFinPh = kThreads / kFinCols;

P2_DEVICE void reduce_parts(const float* __restrict__ part, int S, int C, int c, float& a, float& b) {
  __shared__ float red[2][kFinPh][kFinCols];
  const int cl = threadIdx.x % kFinCols, q = threadIdx.x / kFinCols;
  float sa = 0.f, sb = 0.f;
  if (c < C) {
    for (int r0 = q; r0 < S; r0 += kFinPh * 8) {
      float ta[8], tb[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int r = r0 + kFinPh * u;
        ta[u] = r < S ? part[size_t(r) * C + c] : 0.f;
        tb[u] = r < S ? part[size_t(S + r) * C + c] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        sa += ta[u];
        sb += tb[u];
      }
    }
  }
  red[0][q][cl] = sa;
  red[1][q][cl] = sb;
  __syncthreads();
  a = 0.f;
  b = 0.f;
  if (q == 0) {
#pragma unroll
    for (int p = 0; p < kFinPh; ++p) {
      a += red[0][p][cl];
      b += red[1][p][cl];
    }
  }
}

template <typename T>
__global__ __launch_bounds__(kThreads) void bn_finalize_fwd_kernel(
    const float* __restrict__ part, int S, const T* __restrict__ x, const float* __restrict__ w,
    const float* __restrict__ b, float* __restrict__ run_mean, float* __restrict__ run_var, int64_t* __restrict__ nbt,
    float momentum, float eps, float* __restrict__ mean_out, float* __restrict__ rstd_out, float* __restrict__ coef,
    int M, int C) {
  const int c = blockIdx.x * kFinCols + (threadIdx.x % kFinCols);
  float s1, s2;
  reduce_parts(part, S, C, c, s1, s2);
  if (threadIdx.x >= kFinCols || c >= C) return;
  const float inv_m = 1.f / float(M);
  const float ms = s1 * inv_m;
  const float var = fmaxf(s2 * inv_m - ms * ms, 0.f);
  const float mu = V8<T>::one(x + c) + ms;
  const float rs = rsqrtf(var + eps);
  mean_out[c] = mu;
  rstd_out[c] = rs;
  coef[c] = mu;
  coef[C + c] = w[c] * rs;
  coef[2 * C + c] = b[c];
  if (run_mean) {
    const float unb = M > 1 ? var * (float(M) / float(M - 1)) : var;
    run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * mu;
    run_var[c] = (1.f - momentum) * run_var[c] + momentum * unb;
  }
  if (nbt && c == 0) nbt[0] += 1;
}


// coef = [A | B | D]: dx = A dz + B (x - mean) + D;  dw = rstd * s2, db = s1
__global__ __launch_bounds__(kThreads) void bn_finalize_bwd_kernel(const float* __restrict__ part, int S,
                                                                   const float* __restrict__ w,
                                                                   const float* __restrict__ rstd,
                                                                   float* __restrict__ dw, float* __restrict__ db,
                                                                   float* __restrict__ coef, int M, int C) {
  const int c = blockIdx.x * kFinCols + (threadIdx.x % kFinCols);
  float s1, s2;
  reduce_parts(part, S, C, c, s1, s2);
  if (threadIdx.x >= kFinCols || c >= C) return;
  const float rs = rstd[c], inv_m = 1.f / float(M);
  const float A = w[c] * rs;
  db[c] = s1;
  dw[c] = s2 * rs;
  coef[c] = A;
  coef[C + c] = -A * rs * rs * s2 * inv_m;
  coef[2 * C + c] = -A * s1 * inv_m;
}

// ---------------------------------------------------------------------------
// Apply passes: 8 channels per thread, grid-stride over the [M, C] matrix.
// ---------------------------------------------------------------------------
template <typename T, bool RELU, bool RES>
__global__ __launch_bounds__(kThreads) void bn_apply_fwd_kernel(const T* __restrict__ x, const T* __restrict__ res,
                                                                const float* __restrict__ c_mean,
                                                                const float* __restrict__ c_scale,
                                                                const float* __restrict__ c_bias,
                                                                const float* __restrict__ run_var, float eps,
                                                                T* __restrict__ y, int64_t n8, int C) {
  // training: (mean, scale, bias) = the finalize kernel's coefficients;
  // inference (run_var != null): (running_mean, weight, bias), scale = w * rsqrt(running_var + eps)
  for (int64_t i = blockIdx.x * int64_t(kThreads) + threadIdx.x; i < n8; i += int64_t(gridDim.x) * kThreads) {
    const int64_t e = i * 8;
    const int c = int(e % C);
    float v[8], mu[8], sc[8], bb[8];
    V8<T>::load(x + e, v);
    ld8f(c_mean + c, mu);
    ld8f(c_scale + c, sc);
    ld8f(c_bias + c, bb);
    if (run_var) {
      float rv[8];
      ld8f(run_var + c, rv);
#pragma unroll
      for (int j = 0; j < 8; ++j) sc[j] *= rsqrtf(rv[j] + eps);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = fmaf(v[j] - mu[j], sc[j], bb[j]);
    if (RES) {
      float r[8];
      V8<T>::load(res + e, r);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += r[j];
    }
    if (RELU) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = fmaxf(v[j], 0.f);
    }
    V8<T>::store(y + e, v);
  }
}

template <typename T, bool RELU, bool RES>
__global__ __launch_bounds__(kThreads) void bn_apply_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ dy2,
                                                                const T* __restrict__ y,
                                                                const T* __restrict__ x,
                                                                const float* __restrict__ mean,
                                                                const float* __restrict__ coef, T* __restrict__ dx,
                                                                T* __restrict__ dres, int64_t n8, int C) {
  for (int64_t i = blockIdx.x * int64_t(kThreads) + threadIdx.x; i < n8; i += int64_t(gridDim.x) * kThreads) {
    const int64_t e = i * 8;
    const int c = int(e % C);
    float g[8], xv[8], mu[8], A[8], B[8], D[8];
    V8<T>::load(dy + e, g);
    V8<T>::load(x + e, xv);
    if (dy2) {
      float g2[8];
      V8<T>::load(dy2 + e, g2);
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] += g2[j];
    }
    if (RELU) {
      float yv[8];
      V8<T>::load(y + e, yv);
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = yv[j] > 0.f ? g[j] : 0.f;
    }
    ld8f(mean + c, mu);
    ld8f(coef + c, A);
    ld8f(coef + C + c, B);
    ld8f(coef + 2 * C + c, D);
    if (RES) V8<T>::store(dres + e, g);
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = fmaf(A[j], g[j], fmaf(B[j], xv[j] - mu[j], D[j]));
    V8<T>::store(dx + e, o);
  }
}

// ---------------------------------------------------------------------------
// Statistics + finalize in ONE launch (bf16, C <= 2048, small activations).
// On the ResNet CIFAR shapes each BN pass above is a few us of latency (a
// handful of dependent memory rounds, ~5 us per launch in
// profiles/r3_resnet18_native_steady_state.md), not of bandwidth, so the
// separate finalize launch costs as much as the statistics pass itself.  Here
// every thread loads all kFuseRows of its rows at once, the block writes its
// partial-sum row with sc1 (write-through) stores, and the LAST block to
// arrive (relaxed agent-scope ticket, the split-K hand-off of gemm_core.h: no
// fences) reduces the [S, C] partials in fixed order (sc1 loads) and writes
// the statistics and the apply coefficients.  No block ever waits for
// another (no grid barrier, nothing to deadlock against concurrent streams);
// the apply pass stays its own launch.  Counter: 1 int, zero on entry and on
// exit (ops/splitk.py ring).
// ---------------------------------------------------------------------------
constexpr int kFuseRows = 8;          // rows per thread, all in flight
constexpr int kFuseMaxPart = 16384;   // S * C: the last block reads <= 128 KB of partials

P2_DEVICE __amdgpu_buffer_rsrc_t f32_rsrc(const float* p, int n) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), 0, n * 4, 0x00020000);
}

// Block phase reduction of (s1, s2) written as partial row blockIdx.y with sc1 stores.
P2_DEVICE void fused_partial_store(const float (&s1)[8], const float (&s2)[8], bool active, int tg, int ph, int rp,
                                   float* part, int S, int C) {
  __shared__ float red[2][kRedCols];
  if (active) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[0][ph * C + tg * 8 + j] = s1[j];
      red[1][ph * C + tg * 8 + j] = s2[j];
    }
  }
  __syncthreads();
  const auto rs = f32_rsrc(part, 2 * S * C);
  for (int c = threadIdx.x; c < C; c += kThreads) {
    float a = 0.f, b = 0.f;
    for (int p = 0; p < rp; ++p) {
      a += red[0][p * C + c];
      b += red[1][p * C + c];
    }
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(a), rs, (blockIdx.y * C + c) * 4, 0, 16);
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(b), rs, ((S + blockIdx.y) * C + c) * 4, 0, 16);
  }
}

// Ticket: true in the one block that arrived last (every block drained its
// sc1 partial stores before taking its ticket); it resets the counter.
P2_DEVICE bool fused_arrive(int* ctr, int total) {
  __shared__ int last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const int old = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = old == total - 1;
    if (last) __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  return last;
}

// Fixed-order sum of the S partial rows of (a, b), 4 consecutive columns per
// thread and pq row phases, 8 rows per phase in flight; calls fn(c0, a, b)
// once per 4-column group.
template <class Fn>
P2_DEVICE void fused_reduce_parts(const float* part, int S, int C, Fn&& fn) {
  __shared__ f32x4 red[2][kThreads];
  const auto rs = f32_rsrc(part, 2 * S * C);
  const int nc4 = C / 4;
  const bool narrow = nc4 <= kThreads;
  const int pq = narrow ? kThreads / nc4 : 1;
  const int cl = narrow ? threadIdx.x % nc4 : threadIdx.x, q = narrow ? threadIdx.x / nc4 : 0;
  for (int base = 0; base < nc4; base += kThreads) {  // a second round only when C > 1024
    const int c4 = base + cl;
    const bool on = q < pq && c4 < nc4;
    f32x4 a = {0.f, 0.f, 0.f, 0.f}, b = a;
    if (on) {
      for (int r0 = q; r0 < S; r0 += 8 * pq) {
        f32x4 ta[8], tb[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int r = r0 + u * pq;
          const bool in = r < S;
          ta[u] = in ? __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (r * C + 4 * c4) * 4, 0, 16))
                     : f32x4{0.f, 0.f, 0.f, 0.f};
          tb[u] = in ? __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, ((S + r) * C + 4 * c4) * 4, 0, 16))
                     : f32x4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          a += ta[u];
          b += tb[u];
        }
      }
    }
    __syncthreads();
    red[0][threadIdx.x] = a;
    red[1][threadIdx.x] = b;
    __syncthreads();
    if (on && q == 0) {
      f32x4 sa = {0.f, 0.f, 0.f, 0.f}, sb = sa;
      for (int p = 0; p < pq; ++p) {
        sa += red[0][p * nc4 + cl];
        sb += red[1][p * nc4 + cl];
      }
      fn(4 * c4, sa, sb);
    }
  }
}

P2_DEVICE void unpack8(const uint4& u, float (&v)[8]) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[2 * j] = __uint_as_float(w[j] << 16);
    v[2 * j + 1] = __uint_as_float(w[j] & 0xffff0000u);
  }
}

// forward: statistics + finalize (coef / mean / rstd / running stats as bn_finalize_fwd_kernel)
__global__ __launch_bounds__(kThreads) void bn_stats_fin_kernel(
    const uint16_t* __restrict__ x, const float* __restrict__ w, const float* __restrict__ b,
    float* __restrict__ run_mean, float* __restrict__ run_var, int64_t* __restrict__ nbt, float momentum, float eps,
    float* __restrict__ mean_out, float* __restrict__ rstd_out, float* __restrict__ coef, float* part, int* ctr, int M,
    int C, int tpr, int rp) {
  const int tg = threadIdx.x % tpr, ph = threadIdx.x / tpr, c = tg * 8, S = gridDim.y;
  const bool active = ph < rp;
  const int r0 = blockIdx.y * rp * kFuseRows + ph;
  float s1[8], s2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s1[j] = s2[j] = 0.f;
  if (active) {
    float sh[8];
    V8<uint16_t>::load(x + c, sh);
    uint4 xv[kFuseRows];
#pragma unroll
    for (int k = 0; k < kFuseRows; ++k) {
      const int r = r0 + k * rp;
      xv[k] = r < M ? *reinterpret_cast<const uint4*>(x + size_t(r) * C + c) : uint4{0, 0, 0, 0};
    }
#pragma unroll
    for (int k = 0; k < kFuseRows; ++k) {
      if (r0 + k * rp >= M) continue;
      float v[8];
      unpack8(xv[k], v);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = v[j] - sh[j];
        s1[j] += d;
        s2[j] = fmaf(d, d, s2[j]);
      }
    }
  }
  fused_partial_store(s1, s2, active, tg, ph, rp, part, S, C);
  if (!fused_arrive(ctr, S)) return;
  const float inv_m = 1.f / float(M);
  fused_reduce_parts(part, S, C, [&](int c0, const f32x4& sa, const f32x4& sb) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int cc = c0 + e;
      const float ms = sa[e] * inv_m;
      const float var = fmaxf(sb[e] * inv_m - ms * ms, 0.f);
      const float mu = bf16_to_f32(x[cc]) + ms;
      const float rsd = rsqrtf(var + eps);
      mean_out[cc] = mu;
      rstd_out[cc] = rsd;
      coef[cc] = mu;
      coef[C + cc] = w[cc] * rsd;
      coef[2 * C + cc] = b[cc];
      if (run_mean) {
        const float unb = M > 1 ? var * (float(M) / float(M - 1)) : var;
        run_mean[cc] = (1.f - momentum) * run_mean[cc] + momentum * mu;
        run_var[cc] = (1.f - momentum) * run_var[cc] + momentum * unb;
      }
    }
  });
  if (nbt && threadIdx.x == 0) nbt[0] += 1;
}

// backward: statistics + finalize (dw / db / coef as bn_finalize_bwd_kernel)
template <bool RELU>
__global__ __launch_bounds__(kThreads) void bn_bwd_stats_fin_kernel(
    const uint16_t* __restrict__ dy, const uint16_t* __restrict__ y, const uint16_t* __restrict__ x,
    const float* __restrict__ w, const float* __restrict__ mean, const float* __restrict__ rstd,
    float* __restrict__ dw, float* __restrict__ db, float* __restrict__ coef, float* part, int* ctr, int M, int C,
    int tpr, int rp) {
  const int tg = threadIdx.x % tpr, ph = threadIdx.x / tpr, c = tg * 8, S = gridDim.y;
  const bool active = ph < rp;
  const int r0 = blockIdx.y * rp * kFuseRows + ph;
  float s1[8], s2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s1[j] = s2[j] = 0.f;
  if (active) {
    float mu[8];
    ld8f(mean + c, mu);
    uint4 gv[kFuseRows], xv[kFuseRows], yv[kFuseRows];
#pragma unroll
    for (int k = 0; k < kFuseRows; ++k) {
      const int r = r0 + k * rp;
      const bool in = r < M;
      gv[k] = in ? *reinterpret_cast<const uint4*>(dy + size_t(r) * C + c) : uint4{0, 0, 0, 0};
      xv[k] = in ? *reinterpret_cast<const uint4*>(x + size_t(r) * C + c) : uint4{0, 0, 0, 0};
      if (RELU) yv[k] = in ? *reinterpret_cast<const uint4*>(y + size_t(r) * C + c) : uint4{0, 0, 0, 0};
    }
#pragma unroll
    for (int k = 0; k < kFuseRows; ++k) {
      float g[8], xf[8];
      unpack8(gv[k], g);
      unpack8(xv[k], xf);
      if (RELU) {
        float yf[8];
        unpack8(yv[k], yf);
#pragma unroll
        for (int j = 0; j < 8; ++j) g[j] = yf[j] > 0.f ? g[j] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s1[j] += g[j];
        s2[j] = fmaf(g[j], xf[j] - mu[j], s2[j]);
      }
    }
  }
  fused_partial_store(s1, s2, active, tg, ph, rp, part, S, C);
  if (!fused_arrive(ctr, S)) return;
  const float inv_m = 1.f / float(M);
  fused_reduce_parts(part, S, C, [&](int c0, const f32x4& sa, const f32x4& sb) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int cc = c0 + e;
      const float rsd = rstd[cc], A = w[cc] * rsd;
      db[cc] = sa[e];
      dw[cc] = sb[e] * rsd;
      coef[cc] = A;
      coef[C + cc] = -A * rsd * rsd * sb[e] * inv_m;
      coef[2 * C + cc] = -A * sa[e] * inv_m;
    }
  });
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
BnPlan bn_fused_plan(int M, int C) {
  BnPlan p{};
  const int groups = C / 8;
  if (C % 8 || groups > kThreads) return p;  // S = 0: not eligible
  p.tpr = groups;
  p.rp = kThreads / groups;
  p.gx = 1;
  const int64_t S = (int64_t(M) + int64_t(p.rp) * kFuseRows - 1) / (int64_t(p.rp) * kFuseRows);
  if (S < 1 || S * C > kFuseMaxPart) return p;
  p.S = int(S);
  return p;
}

BnPlan bn_plan(int M, int C) {
  BnPlan p{};
  const int groups = C / 8;
  p.tpr = groups < kThreads ? groups : kThreads;
  p.rp = kThreads / p.tpr;
  p.gx = (groups + p.tpr - 1) / p.tpr;
  // >= 4 rows per thread, <= 256 row splits, <= ~1024 blocks in total
  int S = (M + 4 * p.rp - 1) / (4 * p.rp);
  const int cap = 1024 / p.gx > 256 ? 256 : (1024 / p.gx < 1 ? 1 : 1024 / p.gx);
  if (S > cap) S = cap;
  p.S = S < 1 ? 1 : S;
  return p;
}

template <typename T>
static void apply_fwd(const T* x, const T* r, const float* coef, T* y, int M, int C, bool relu, hipStream_t s) {
  const int64_t n8 = int64_t(M) * C / 8;
  const dim3 grid(stream_grid(n8, kThreads)), blk(kThreads);
  if (relu && r)
    hipLaunchKernelGGL((bn_apply_fwd_kernel<T, true, true>), grid, blk, 0, s, x, r, coef, coef + C, coef + 2 * C, nullptr, 0.f, y, n8, C);
  else if (relu)
    hipLaunchKernelGGL((bn_apply_fwd_kernel<T, true, false>), grid, blk, 0, s, x, r, coef, coef + C, coef + 2 * C, nullptr, 0.f, y, n8, C);
  else if (r)
    hipLaunchKernelGGL((bn_apply_fwd_kernel<T, false, true>), grid, blk, 0, s, x, r, coef, coef + C, coef + 2 * C, nullptr, 0.f, y, n8, C);
  else
    hipLaunchKernelGGL((bn_apply_fwd_kernel<T, false, false>), grid, blk, 0, s, x, r, coef, coef + C, coef + 2 * C, nullptr, 0.f, y, n8, C);
}

template <typename T>
static void apply_bwd(const T* dy, const T* dy2, const T* y, const T* x, const float* mean, const float* coef, T* dx,
                      T* dres, int M, int C, bool relu, hipStream_t s) {
  const int64_t n8 = int64_t(M) * C / 8;
  const dim3 grid(stream_grid(n8, kThreads)), blk(kThreads);
  if (relu && dres)
    hipLaunchKernelGGL((bn_apply_bwd_kernel<T, true, true>), grid, blk, 0, s, dy, dy2, y, x, mean, coef, dx, dres, n8, C);
  else if (relu)
    hipLaunchKernelGGL((bn_apply_bwd_kernel<T, true, false>), grid, blk, 0, s, dy, dy2, y, x, mean, coef, dx, dres, n8, C);
  else if (dres)
    hipLaunchKernelGGL((bn_apply_bwd_kernel<T, false, true>), grid, blk, 0, s, dy, dy2, y, x, mean, coef, dx, dres, n8, C);
  else
    hipLaunchKernelGGL((bn_apply_bwd_kernel<T, false, false>), grid, blk, 0, s, dy, dy2, y, x, mean, coef, dx, dres, n8, C);
}

template <typename T>
static void fwd_train_t(const void* xv, const void* rv, const float* w, const float* b, float* rm, float* rvar,
                        int64_t* nbt, float momentum, float eps, void* yv, float* mean, float* rstd, float* coef,
                        float* part, int* ctr, int M, int C, bool relu, hipStream_t s) {
  const T* x = static_cast<const T*>(xv);
  const T* r = static_cast<const T*>(rv);
  T* y = static_cast<T*>(yv);
  if constexpr (sizeof(T) == 2) {
    const BnPlan f = bn_fused_plan(M, C);
    if (ctr && f.S > 0) {
      hipLaunchKernelGGL(bn_stats_fin_kernel, dim3(1, f.S), dim3(kThreads), 0, s, x, w, b, rm, rvar, nbt, momentum, eps,
                         mean, rstd, coef, part, ctr, M, C, f.tpr, f.rp);
      apply_fwd(x, r, coef, y, M, C, relu, s);
      return;
    }
  }
  const BnPlan p = bn_plan(M, C);
  hipLaunchKernelGGL(bn_stats_kernel<T>, dim3(p.gx, p.S), dim3(kThreads), 0, s, x, part, M, C, p.tpr, p.rp);
  hipLaunchKernelGGL(bn_finalize_fwd_kernel<T>, dim3((C + kFinCols - 1) / kFinCols), dim3(kThreads), 0, s, part, p.S, x, w, b, rm,
                     rvar, nbt, momentum, eps, mean, rstd, coef, M, C);
  apply_fwd(x, r, coef, y, M, C, relu, s);
}

void bn_fwd_train(bool bf16, const void* x, const void* res, const float* w, const float* b, float* run_mean,
                  float* run_var, int64_t* nbt, float momentum, float eps, void* y, float* mean, float* rstd,
                  float* coef, float* part, int* ctr, int M, int C, bool relu, hipStream_t s) {
  if (bf16)
    fwd_train_t<uint16_t>(x, res, w, b, run_mean, run_var, nbt, momentum, eps, y, mean, rstd, coef, part, ctr, M, C, relu, s);
  else
    fwd_train_t<float>(x, res, w, b, run_mean, run_var, nbt, momentum, eps, y, mean, rstd, coef, part, nullptr, M, C, relu, s);
}

template <typename T>
static void fwd_eval_t(const void* xv, const void* rv, const float* w, const float* b, const float* rm,
                       const float* rvar, float eps, void* yv, float* coef, int M, int C, bool relu, hipStream_t s) {
  const T* x = static_cast<const T*>(xv);
  const T* r = static_cast<const T*>(rv);
  T* y = static_cast<T*>(yv);
  const int64_t n8 = int64_t(M) * C / 8;
  const dim3 grid(stream_grid(n8, kThreads)), blk(kThreads);
  if (relu && r)
    hipLaunchKernelGGL((bn_apply_fwd_kernel<T, true, true>), grid, blk, 0, s, x, r, rm, w, b, rvar, eps, y, n8, C);
  else if (relu)
    hipLaunchKernelGGL((bn_apply_fwd_kernel<T, true, false>), grid, blk, 0, s, x, r, rm, w, b, rvar, eps, y, n8, C);
  else if (r)
    hipLaunchKernelGGL((bn_apply_fwd_kernel<T, false, true>), grid, blk, 0, s, x, r, rm, w, b, rvar, eps, y, n8, C);
  else
    hipLaunchKernelGGL((bn_apply_fwd_kernel<T, false, false>), grid, blk, 0, s, x, r, rm, w, b, rvar, eps, y, n8, C);
}

void bn_apply_train(bool bf16, const void* x, const void* res, const float* coef, void* y, int M, int C, bool relu,
                    hipStream_t s) {
  if (bf16)
    apply_fwd<uint16_t>(static_cast<const uint16_t*>(x), static_cast<const uint16_t*>(res), coef, static_cast<uint16_t*>(y),
                        M, C, relu, s);
  else
    apply_fwd<float>(static_cast<const float*>(x), static_cast<const float*>(res), coef, static_cast<float*>(y), M, C,
                     relu, s);
}

void bn_apply_bwd_only(const void* dy, const void* y, const void* x, const float* mean, const float* coef, void* dx,
                       int M, int C, bool relu, hipStream_t s) {
  apply_bwd<uint16_t>(static_cast<const uint16_t*>(dy), nullptr, static_cast<const uint16_t*>(y), static_cast<const uint16_t*>(x),
                      mean, coef, static_cast<uint16_t*>(dx), nullptr, M, C, relu, s);
}

void bn_fwd_eval(bool bf16, const void* x, const void* res, const float* w, const float* b, const float* run_mean,
                 const float* run_var, float eps, void* y, float* coef, int M, int C, bool relu, hipStream_t s) {
  if (bf16)
    fwd_eval_t<uint16_t>(x, res, w, b, run_mean, run_var, eps, y, coef, M, C, relu, s);
  else
    fwd_eval_t<float>(x, res, w, b, run_mean, run_var, eps, y, coef, M, C, relu, s);
}

template <typename T>
static void bwd_t(const void* dyv, const void* dy2v, const void* yv, const void* xv, const float* w, const float* mean,
                  const float* rstd, void* dxv, void* dresv, float* dw, float* db, float* coef, float* part, int* ctr,
                  int M, int C, bool relu, hipStream_t s) {
  const T* dy = static_cast<const T*>(dyv);
  const T* dy2 = static_cast<const T*>(dy2v);
  const T* y = static_cast<const T*>(yv);
  const T* x = static_cast<const T*>(xv);
  T* dx = static_cast<T*>(dxv);
  T* dres = static_cast<T*>(dresv);
  if constexpr (sizeof(T) == 2) {
    const BnPlan f = bn_fused_plan(M, C);
    if (ctr && f.S > 0 && !dy2) {
      if (relu)
        hipLaunchKernelGGL(bn_bwd_stats_fin_kernel<true>, dim3(1, f.S), dim3(kThreads), 0, s, dy, y, x, w, mean, rstd, dw,
                           db, coef, part, ctr, M, C, f.tpr, f.rp);
      else
        hipLaunchKernelGGL(bn_bwd_stats_fin_kernel<false>, dim3(1, f.S), dim3(kThreads), 0, s, dy, y, x, w, mean, rstd, dw,
                           db, coef, part, ctr, M, C, f.tpr, f.rp);
      apply_bwd(dy, dy2, y, x, mean, coef, dx, dres, M, C, relu, s);
      return;
    }
  }
  const BnPlan p = bn_plan(M, C);
  const dim3 sgrid(p.gx, p.S), blk(kThreads);
  if (relu)
    hipLaunchKernelGGL((bn_bwd_stats_kernel<T, true>), sgrid, blk, 0, s, dy, dy2, y, x, mean, part, M, C, p.tpr, p.rp);
  else
    hipLaunchKernelGGL((bn_bwd_stats_kernel<T, false>), sgrid, blk, 0, s, dy, dy2, y, x, mean, part, M, C, p.tpr, p.rp);
  hipLaunchKernelGGL(bn_finalize_bwd_kernel, dim3((C + kFinCols - 1) / kFinCols), blk, 0, s, part, p.S, w, rstd, dw, db, coef, M, C);
  apply_bwd(dy, dy2, y, x, mean, coef, dx, dres, M, C, relu, s);
}

void bn_bwd(bool bf16, const void* dy, const void* dy2, const void* y, const void* x, const float* w, const float* mean,
            const float* rstd, void* dx, void* dres, float* dw, float* db, float* coef, float* part, int* ctr, int M,
            int C, bool relu, hipStream_t s) {
  if (bf16)
    bwd_t<uint16_t>(dy, dy2, y, x, w, mean, rstd, dx, dres, dw, db, coef, part, ctr, M, C, relu, s);
  else
    bwd_t<float>(dy, dy2, y, x, w, mean, rstd, dx, dres, dw, db, coef, part, nullptr, M, C, relu, s);
}

}  // namespace p2bn
