// Fused BatchNorm (+ residual add) (+ ReLU) for MI355X (gfx950, wave64), on
// channels-last activations viewed as [M, C] (M = N*H*W rows of C channels).
//
// What it replaces in a ResNet block (PyTorch-ROCm, NHWC bf16):
//   forward   MIOpen BN training kernel(s) + residual add + ReLU     (3+ passes)
//   backward  ReLU threshold_backward + MIOpen BN backward           (3+ passes)
// Here, per BN, two launches each way (one for inference):
//   forward   stats+finalize (1 read of x)   -> apply (read x [+res], write y)
//   backward  stats+finalize (read dy, y, x) -> apply (read dy, y, x, write dx [+dres])
//   eval      apply with the running statistics
//
// Column statistics: every thread owns 8 consecutive channels (one 16-B bf16
// load per row, 8 rows in flight), a 256-thread block covers `tpr` threads
// per row x `rp` row phases, row splits go over gridDim.y.  Each block sums
// its row phases in LDS in fixed order and stores one [S, C] partial row.
// The LAST block of a column slice to finish (per-slice arrival counter)
// reduces the S partial rows in fixed order and writes the per-channel
// coefficients, so no separate finalize launch is needed.  The hand-off
// follows the MI355X inter-workgroup rules (XCD L2s are not coherent):
// partials are stored write-through (`sc1`), every storing wave drains its
// stores before the block barrier, one lane adds to the agent-scope counter,
// and the last block reads the partials with `sc1` loads.  The last block
// resets its counter, so the counters (owned by the BatchNorm module, zeroed
// once) stay valid across launches and HIP-graph replays.  No float atomics:
// results are bitwise reproducible run to run.
//
// Forward statistics use sums shifted by the first row's value (x - x[0][c])
// so the variance does not cancel for activations with a large mean; the
// apply pass computes (x - mean) * scale + b for the same reason.
#include "batchnorm.h"
#include "common.h"

namespace p2bn {
using namespace p2;

typedef __attribute__((address_space(1))) float gf32;
typedef __attribute__((address_space(1))) int gi32;

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
constexpr int kMaxCols = 256;      // channels per column slice (<= 32 threads per row)
constexpr int kRowsInFlight = 8;   // rows loaded per thread per iteration
constexpr int kGroup = 16;         // partial rows per level-1 group
constexpr int kMaxSplits = 256;    // partial rows (16 groups of 16)

P2_DEVICE void st_sc1(float* p, float v) { __hip_atomic_store((gf32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
P2_DEVICE float ld_sc1(const float* p) {
  return __hip_atomic_load((gf32*)const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Partial-row storage of one launch: rows [0, S) per block, rows [S, S + 16)
// per level-1 group; array b follows array a.
struct Parts {
  float* a;
  float* b;
};
P2_DEVICE Parts parts(float* part, int C) {
  const int R = gridDim.y + kGroup;
  return Parts{part, part + size_t(R) * C};
}

// Columns of this slice: lane group tg of the block owns 8 of them.
P2_DEVICE int slice_width(int tpr) { return tpr * 8; }

// Store this block's per-column sums (LDS res[2][W]) as partial row `row`
// (write-through), drain, and arrive on `ctr` (agent-scope atomic by one
// lane after the barrier).  Returns true in the block that arrived last
// (which resets the counter for the next launch).
P2_DEVICE bool publish_arrive(const float* res, int row, int W, int C, Parts pt, int* ctr, int expected) {
  __shared__ int s_last;
  for (int i = threadIdx.x; i < W; i += kThreads) {
    const int c = blockIdx.x * W + i;
    if (c < C) {
      st_sc1(pt.a + size_t(row) * C + c, res[i]);
      st_sc1(pt.b + size_t(row) * C + c, res[kMaxCols + i]);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains first
  __syncthreads();
  if (threadIdx.x == 0) {
    const int prev = __hip_atomic_fetch_add((gi32*)ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool last = prev == expected - 1;
    if (last) __hip_atomic_store((gi32*)ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = last;
  }
  __syncthreads();
  return s_last;
}

// res[.][i] = sum of partial rows [r0, r0 + n) of column slice i (fixed order,
// sc1 loads).  P = 256 / W row phases per column, combined in LDS in order.
P2_DEVICE void reduce_rows(Parts pt, int r0, int n, int W, int C, float* red, float* res) {
  const int P = kThreads / W;
  const int i = threadIdx.x;
  if (i < W * P) {
    const int cl = i % W, ph = i / W, c = blockIdx.x * W + cl;
    float a = 0.f, b = 0.f;
    if (c < C) {
      float ta[kGroup], tb[kGroup];
#pragma unroll
      for (int u = 0; u < kGroup; ++u) {
        const int r = ph + u * P;
        ta[u] = r < n ? ld_sc1(pt.a + size_t(r0 + r) * C + c) : 0.f;
        tb[u] = r < n ? ld_sc1(pt.b + size_t(r0 + r) * C + c) : 0.f;
      }
#pragma unroll
      for (int u = 0; u < kGroup; ++u) {
        a += ta[u];
        b += tb[u];
      }
    }
    red[ph * W + cl] = a;
    red[kThreads + ph * W + cl] = b;
  }
  __syncthreads();
  for (int cl = threadIdx.x; cl < W; cl += kThreads) {
    float a = 0.f, b = 0.f;
    for (int p = 0; p < P; ++p) {
      a += red[p * W + cl];
      b += red[kThreads + p * W + cl];
    }
    res[cl] = a;
    res[kMaxCols + cl] = b;
  }
  __syncthreads();
}

// Block sums -> level-1 partial row -> (last of its group) level-2 row ->
// (last group) final per-column sums in res.  Returns true in the one block
// that then finalises the slice.
P2_DEVICE bool fan_in(float (&s1)[8], float (&s2)[8], bool active, int tg, int ph, int tpr, int rp, float* part,
                      int C, int* ctr, float* red, float* res) {
  const int W = slice_width(tpr), S = gridDim.y;
  const Parts pt = parts(part, C);
  // 1. fixed-order sum over this block's row phases
  if (active) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[ph * W + tg * 8 + j] = s1[j];
      red[kThreads * 8 + ph * W + tg * 8 + j] = s2[j];
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < W; i += kThreads) {
    float a = 0.f, b = 0.f;
    for (int p = 0; p < rp; ++p) {
      a += red[p * W + i];
      b += red[kThreads * 8 + p * W + i];
    }
    res[i] = a;
    res[kMaxCols + i] = b;
  }
  __syncthreads();
  const int G = (S + kGroup - 1) / kGroup, grp = blockIdx.y / kGroup;
  const int in_grp = min(kGroup, S - grp * kGroup);
  int* c1 = ctr + blockIdx.x * (1 + kGroup);
  // 2. level 1: one partial row per block, the group's last block reduces them
  if (!publish_arrive(res, blockIdx.y, W, C, pt, c1 + 1 + grp, in_grp)) return false;
  reduce_rows(pt, grp * kGroup, in_grp, W, C, red, res);
  if (G == 1) return true;
  // 3. level 2: one row per group, the last group reduces them
  if (!publish_arrive(res, S + grp, W, C, pt, c1, G)) return false;
  reduce_rows(pt, S, G, W, C, red, res);
  return true;
}

// ---------------------------------------------------------------------------
// forward statistics + finalize.  coef = [mean | scale | bias] for the apply pass.
// ---------------------------------------------------------------------------
struct FwdFin {
  const float* w;
  const float* b;
  float* run_mean;
  float* run_var;
  int64_t* nbt;
  float momentum, eps;
  float* mean_out;
  float* rstd_out;
  float* coef;
};

template <typename T>
__global__ __launch_bounds__(kThreads) void bn_stats_kernel(const T* __restrict__ x, float* __restrict__ part,
                                                            int* __restrict__ counter, FwdFin f, int M, int C, int tpr,
                                                            int rp) {
  __shared__ float red[2 * kThreads * 8];
  __shared__ float res[2 * kMaxCols];
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
    for (int r0 = blockIdx.y * rp + ph; r0 < M; r0 += kRowsInFlight * step) {
      float v[kRowsInFlight][8];
#pragma unroll
      for (int u = 0; u < kRowsInFlight; ++u) {
        const int r = r0 + u * step;
        if (r < M) {
          V8<T>::load(x + size_t(r) * C + c, v[u]);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[u][j] = sh[j];  // contributes 0
        }
      }
#pragma unroll
      for (int u = 0; u < kRowsInFlight; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = v[u][j] - sh[j];
          s1[j] += d;
          s2[j] = fmaf(d, d, s2[j]);
        }
    }
  }
  if (!fan_in(s1, s2, active, tg, ph, tpr, rp, part, C, counter, red, res)) return;
  const float inv_m = 1.f / float(M);
  const int W = slice_width(tpr);
  for (int cl = threadIdx.x; cl < W; cl += kThreads) {
    const int cc = blockIdx.x * W + cl;
    if (cc >= C) continue;
    const float a = res[cl], b = res[kMaxCols + cl];
    const float ms = a * inv_m;
    const float var = fmaxf(b * inv_m - ms * ms, 0.f);
    const float mu = V8<T>::one(x + cc) + ms;
    const float rs = rsqrtf(var + f.eps);
    f.mean_out[cc] = mu;
    f.rstd_out[cc] = rs;
    f.coef[cc] = mu;
    f.coef[C + cc] = f.w[cc] * rs;
    f.coef[2 * C + cc] = f.b[cc];
    if (f.run_mean) {
      const float unb = M > 1 ? var * (float(M) / float(M - 1)) : var;
      f.run_mean[cc] = (1.f - f.momentum) * f.run_mean[cc] + f.momentum * mu;
      f.run_var[cc] = (1.f - f.momentum) * f.run_var[cc] + f.momentum * unb;
    }
    if (f.nbt && cc == 0) f.nbt[0] += 1;
  }
}

// ---------------------------------------------------------------------------
// backward statistics + finalize: sum dz and sum dz * (x - mean) per channel.
// coef = [A | B | D | mean]: dx = A dz + B (x - mean) + D;  dw = rstd * s2, db = s1
// ---------------------------------------------------------------------------
struct BwdFin {
  const float* w;
  const float* mean;
  const float* rstd;
  float* dw;
  float* db;
  float* coef;
};

template <typename T, bool RELU>
__global__ __launch_bounds__(kThreads) void bn_bwd_stats_kernel(const T* __restrict__ dy, const T* __restrict__ y,
                                                                const T* __restrict__ x, float* __restrict__ part,
                                                                int* __restrict__ counter, BwdFin f, int M, int C,
                                                                int tpr, int rp) {
  __shared__ float red[2 * kThreads * 8];
  __shared__ float res[2 * kMaxCols];
  const int tg = threadIdx.x % tpr, ph = threadIdx.x / tpr;
  const int c = (blockIdx.x * tpr + tg) * 8;
  const bool active = ph < rp && c < C;
  float s1[8], s2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s1[j] = s2[j] = 0.f;
  if (active) {
    float mu[8];
    ld8f(f.mean + c, mu);
    const int step = rp * gridDim.y;
    constexpr int U = kRowsInFlight / 2;  // three streams per row
    for (int r0 = blockIdx.y * rp + ph; r0 < M; r0 += U * step) {
      float g[U][8], xv[U][8];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int r = r0 + u * step;
        if (r < M) {
          const size_t e = size_t(r) * C + c;
          V8<T>::load(dy + e, g[u]);
          V8<T>::load(x + e, xv[u]);
          if (RELU) {
            float yv[8];
            V8<T>::load(y + e, yv);
#pragma unroll
            for (int j = 0; j < 8; ++j) g[u][j] = yv[j] > 0.f ? g[u][j] : 0.f;
          }
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) g[u][j] = xv[u][j] = 0.f;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          s1[j] += g[u][j];
          s2[j] = fmaf(g[u][j], xv[u][j] - mu[j], s2[j]);
        }
    }
  }
  if (!fan_in(s1, s2, active, tg, ph, tpr, rp, part, C, counter, red, res)) return;
  const float inv_m = 1.f / float(M);
  const int W = slice_width(tpr);
  for (int cl = threadIdx.x; cl < W; cl += kThreads) {
    const int cc = blockIdx.x * W + cl;
    if (cc >= C) continue;
    const float a = res[cl], b = res[kMaxCols + cl];
    const float rs = f.rstd[cc];
    const float A = f.w[cc] * rs;
    f.db[cc] = a;
    f.dw[cc] = b * rs;
    f.coef[cc] = A;
    f.coef[C + cc] = -A * rs * rs * b * inv_m;
    f.coef[2 * C + cc] = -A * a * inv_m;
    f.coef[3 * C + cc] = f.mean[cc];
  }
}

// ---------------------------------------------------------------------------
// Apply passes: the block stages its per-channel coefficients in LDS, then
// 8 channels per thread, grid-stride over the [M, C] matrix.
// ---------------------------------------------------------------------------
template <typename T, bool RELU, bool RES>
__global__ __launch_bounds__(kThreads) void bn_apply_fwd_kernel(const T* __restrict__ x, const T* __restrict__ res,
                                                                const float* __restrict__ coef,
                                                                const float* __restrict__ ew,
                                                                const float* __restrict__ eb,
                                                                const float* __restrict__ erm,
                                                                const float* __restrict__ erv, float eps,
                                                                T* __restrict__ y, int64_t n8, int C) {
  extern __shared__ __attribute__((aligned(16))) float lc[];  // [3][C]: mean, scale, bias
  for (int c = threadIdx.x; c < C; c += kThreads) {
    if (coef) {
      lc[c] = coef[c];
      lc[C + c] = coef[C + c];
      lc[2 * C + c] = coef[2 * C + c];
    } else {  // inference: running statistics
      lc[c] = erm[c];
      lc[C + c] = ew[c] * rsqrtf(erv[c] + eps);
      lc[2 * C + c] = eb[c];
    }
  }
  __syncthreads();
  for (int64_t i = blockIdx.x * int64_t(kThreads) + threadIdx.x; i < n8; i += int64_t(gridDim.x) * kThreads) {
    const int64_t e = i * 8;
    const int c = int(e % C);
    float v[8], mu[8], sc[8], bb[8];
    V8<T>::load(x + e, v);
    ld8f(lc + c, mu);
    ld8f(lc + C + c, sc);
    ld8f(lc + 2 * C + c, bb);
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
__global__ __launch_bounds__(kThreads) void bn_apply_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ y,
                                                                const T* __restrict__ x,
                                                                const float* __restrict__ coef, T* __restrict__ dx,
                                                                T* __restrict__ dres, int64_t n8, int C) {
  extern __shared__ __attribute__((aligned(16))) float lc[];  // [4][C]: A, B, D, mean
  for (int c = threadIdx.x; c < 4 * C; c += kThreads) lc[c] = coef[c];
  __syncthreads();
  for (int64_t i = blockIdx.x * int64_t(kThreads) + threadIdx.x; i < n8; i += int64_t(gridDim.x) * kThreads) {
    const int64_t e = i * 8;
    const int c = int(e % C);
    float g[8], xv[8], A[8], B[8], D[8], mu[8];
    V8<T>::load(dy + e, g);
    V8<T>::load(x + e, xv);
    if (RELU) {
      float yv[8];
      V8<T>::load(y + e, yv);
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = yv[j] > 0.f ? g[j] : 0.f;
    }
    ld8f(lc + c, A);
    ld8f(lc + C + c, B);
    ld8f(lc + 2 * C + c, D);
    ld8f(lc + 3 * C + c, mu);
    if (RES) V8<T>::store(dres + e, g);
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = fmaf(A[j], g[j], fmaf(B[j], xv[j] - mu[j], D[j]));
    V8<T>::store(dx + e, o);
  }
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
BnPlan bn_plan(int M, int C) {
  BnPlan p{};
  const int groups = C / 8;
  p.tpr = groups < kMaxCols / 8 ? groups : kMaxCols / 8;
  p.rp = kThreads / p.tpr;
  p.gx = (groups + p.tpr - 1) / p.tpr;
  // one round of 8 loads in flight per thread, <= 256 partial rows, <= 2048 blocks
  int S = (M + kRowsInFlight * p.rp - 1) / (kRowsInFlight * p.rp);
  const int cap = 2048 / p.gx < kMaxSplits ? 2048 / p.gx : kMaxSplits;
  if (S > cap) S = cap;
  p.S = S < 1 ? 1 : S;
  return p;
}

int bn_counters(int C) {
  const BnPlan p = bn_plan(1, C);
  return p.gx * (1 + kGroup);
}

int bn_part_rows(int S) { return S + kGroup; }

static int apply_grid(int64_t n8) {
  // >= 2 items per thread so staging the coefficients is amortised
  int64_t g = (n8 + kThreads * 2 - 1) / (kThreads * 2);
  return int(g < 1 ? 1 : (g > 2048 ? 2048 : g));
}

template <typename T>
static void launch_apply_fwd(const T* x, const T* r, const float* coef, const float* w, const float* b,
                             const float* rm, const float* rv, float eps, T* y, int M, int C, bool relu,
                             hipStream_t s) {
  const int64_t n8 = int64_t(M) * C / 8;
  const dim3 grid(apply_grid(n8)), blk(kThreads);
  const size_t lds = size_t(3) * C * sizeof(float);
  if (relu && r)
    hipLaunchKernelGGL((bn_apply_fwd_kernel<T, true, true>), grid, blk, lds, s, x, r, coef, w, b, rm, rv, eps, y, n8, C);
  else if (relu)
    hipLaunchKernelGGL((bn_apply_fwd_kernel<T, true, false>), grid, blk, lds, s, x, r, coef, w, b, rm, rv, eps, y, n8, C);
  else if (r)
    hipLaunchKernelGGL((bn_apply_fwd_kernel<T, false, true>), grid, blk, lds, s, x, r, coef, w, b, rm, rv, eps, y, n8, C);
  else
    hipLaunchKernelGGL((bn_apply_fwd_kernel<T, false, false>), grid, blk, lds, s, x, r, coef, w, b, rm, rv, eps, y, n8, C);
}

template <typename T>
static void fwd_train_t(const void* xv, const void* rv, const float* w, const float* b, float* rm, float* rvar,
                        int64_t* nbt, float momentum, float eps, void* yv, float* mean, float* rstd, float* coef,
                        float* part, int* counters, int M, int C, bool relu, hipStream_t s) {
  const T* x = static_cast<const T*>(xv);
  const BnPlan p = bn_plan(M, C);
  const FwdFin f{w, b, rm, rvar, nbt, momentum, eps, mean, rstd, coef};
  hipLaunchKernelGGL(bn_stats_kernel<T>, dim3(p.gx, p.S), dim3(kThreads), 0, s, x, part, counters, f, M, C, p.tpr,
                     p.rp);
  launch_apply_fwd<T>(x, static_cast<const T*>(rv), coef, nullptr, nullptr, nullptr, nullptr, 0.f, static_cast<T*>(yv),
                      M, C, relu, s);
}

void bn_fwd_train(bool bf16, const void* x, const void* res, const float* w, const float* b, float* run_mean,
                  float* run_var, int64_t* nbt, float momentum, float eps, void* y, float* mean, float* rstd,
                  float* coef, float* part, int* counters, int M, int C, bool relu, hipStream_t s) {
  if (bf16)
    fwd_train_t<uint16_t>(x, res, w, b, run_mean, run_var, nbt, momentum, eps, y, mean, rstd, coef, part, counters, M,
                          C, relu, s);
  else
    fwd_train_t<float>(x, res, w, b, run_mean, run_var, nbt, momentum, eps, y, mean, rstd, coef, part, counters, M, C,
                       relu, s);
}

void bn_fwd_eval(bool bf16, const void* x, const void* res, const float* w, const float* b, const float* run_mean,
                 const float* run_var, float eps, void* y, int M, int C, bool relu, hipStream_t s) {
  if (bf16)
    launch_apply_fwd<uint16_t>(static_cast<const uint16_t*>(x), static_cast<const uint16_t*>(res), nullptr, w, b,
                               run_mean, run_var, eps, static_cast<uint16_t*>(y), M, C, relu, s);
  else
    launch_apply_fwd<float>(static_cast<const float*>(x), static_cast<const float*>(res), nullptr, w, b, run_mean,
                            run_var, eps, static_cast<float*>(y), M, C, relu, s);
}

template <typename T>
static void bwd_t(const void* dyv, const void* yv, const void* xv, const float* w, const float* mean,
                  const float* rstd, void* dxv, void* dresv, float* dw, float* db, float* coef, float* part,
                  int* counters, int M, int C, bool relu, hipStream_t s) {
  const T* dy = static_cast<const T*>(dyv);
  const T* y = static_cast<const T*>(yv);
  const T* x = static_cast<const T*>(xv);
  T* dx = static_cast<T*>(dxv);
  T* dres = static_cast<T*>(dresv);
  const BnPlan p = bn_plan(M, C);
  const dim3 sgrid(p.gx, p.S), blk(kThreads);
  const BwdFin f{w, mean, rstd, dw, db, coef};
  if (relu)
    hipLaunchKernelGGL((bn_bwd_stats_kernel<T, true>), sgrid, blk, 0, s, dy, y, x, part, counters, f, M, C, p.tpr, p.rp);
  else
    hipLaunchKernelGGL((bn_bwd_stats_kernel<T, false>), sgrid, blk, 0, s, dy, y, x, part, counters, f, M, C, p.tpr,
                       p.rp);
  const int64_t n8 = int64_t(M) * C / 8;
  const dim3 grid(apply_grid(n8));
  const size_t lds = size_t(4) * C * sizeof(float);
  if (relu && dres)
    hipLaunchKernelGGL((bn_apply_bwd_kernel<T, true, true>), grid, blk, lds, s, dy, y, x, coef, dx, dres, n8, C);
  else if (relu)
    hipLaunchKernelGGL((bn_apply_bwd_kernel<T, true, false>), grid, blk, lds, s, dy, y, x, coef, dx, dres, n8, C);
  else if (dres)
    hipLaunchKernelGGL((bn_apply_bwd_kernel<T, false, true>), grid, blk, lds, s, dy, y, x, coef, dx, dres, n8, C);
  else
    hipLaunchKernelGGL((bn_apply_bwd_kernel<T, false, false>), grid, blk, lds, s, dy, y, x, coef, dx, dres, n8, C);
}

void bn_bwd(bool bf16, const void* dy, const void* y, const void* x, const float* w, const float* mean,
            const float* rstd, void* dx, void* dres, float* dw, float* db, float* coef, float* part, int* counters,
            int M, int C, bool relu, hipStream_t s) {
  if (bf16)
    bwd_t<uint16_t>(dy, y, x, w, mean, rstd, dx, dres, dw, db, coef, part, counters, M, C, relu, s);
  else
    bwd_t<float>(dy, y, x, w, mean, rstd, dx, dres, dw, db, coef, part, counters, M, C, relu, s);
}

}  // namespace p2bn
