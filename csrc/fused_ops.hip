// Fused transformer / classifier ops for MI355X (gfx950, wave64):
//   LayerNorm forward / backward, bias + GELU forward / backward,
//   softmax cross-entropy forward / backward.
// Activations are bf16 or fp32 (T), parameters and statistics fp32.  Every
// row-wise op gives one row to one wave (64 lanes x 16-B vector loads), keeps
// the row in registers between its passes, and reduces with cross-lane
// shuffles.  Column reductions (LayerNorm dgamma/dbeta, GELU dbias) are
// per-block partial rows summed by col_reduce in fixed order: no float
// atomics, bitwise-reproducible results.
#include "common.h"
#include "fused_ops.h"

namespace p2fused {
using namespace p2;

// ---- 8-element vector load/store for bf16 (16 B) and fp32 (2 x 16 B) ----
template <typename T>
struct Vec8;
template <>
struct Vec8<uint16_t> {
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
};
template <>
struct Vec8<float> {
  static P2_DEVICE void load(const float* p, float (&v)[8]) {
    const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
  static P2_DEVICE void store(float* p, const float (&v)[8]) {
    reinterpret_cast<float4*>(p)[0] = make_float4(v[0], v[1], v[2], v[3]);
    reinterpret_cast<float4*>(p)[1] = make_float4(v[4], v[5], v[6], v[7]);
  }
};
P2_DEVICE void load8f(const float* p, float (&v)[8]) { Vec8<float>::load(p, v); }
// round fp32 values to what a T tensor holds (bf16: RNE; fp32: identity)
template <typename T>
P2_DEVICE void round_to(float (&v)[8]);
template <>
P2_DEVICE void round_to<uint16_t>(float (&v)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = bf16_to_f32(f32_to_bf16(v[j]));
}
template <>
P2_DEVICE void round_to<float>(float (&)[8]) {}

// ---------------------------------------------------------------------------
// LayerNorm forward: y = (x - mean) * rstd * w + b over the last dim C.
// One wave per row, R rows per wave with every row's loads issued before the
// first reduction (one memory round trip for R rows instead of R: one row per
// wave left the ViT-sized call latency-bound at ~1.4 TB/s).  The rows
// (C <= 512 * K elements, C <= 2048) stay in registers between the mean and
// the variance pass (two-pass variance: no cancellation).  Saves mean / rstd
// for the backward.
// ---------------------------------------------------------------------------
template <typename T, int K, int R, bool RES>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const T* __restrict__ x, const T* __restrict__ res,
                                                     const float* __restrict__ w, const float* __restrict__ b,
                                                     T* __restrict__ y, T* __restrict__ sum_out,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                     int N, int C, float eps) {
  const int lane = threadIdx.x & 63;
  const int nw = gridDim.x * 4;
  // affine parameters are the same for every row: loaded once
  // Loads are unconditional (column clamped to a valid chunk, unused values
  // masked at use; residual presence is a template parameter): a load under
  // a branch gets its own s_waitcnt vmcnt(0), which serialised the rows.
  float wv[K][8], bv[K][8];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int c = (lane + 64 * k) * 8, cc = c < C ? c : 0;
    load8f(w + cc, wv[k]);
    load8f(b + cc, bv[k]);
  }
  for (int row0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * R; row0 < N; row0 += nw * R) {
    float v[R][K][8], rv[R][K][8];
#pragma unroll
    for (int q = 0; q < R; ++q) {
      const int row = row0 + q < N ? row0 + q : N - 1;  // clamped: duplicates are not stored
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int c = (lane + 64 * k) * 8, cc = c < C ? c : 0;
        Vec8<T>::load(x + size_t(row) * C + cc, v[q][k]);
        if constexpr (RES) Vec8<T>::load(res + size_t(row) * C + cc, rv[q][k]);
      }
    }
    if constexpr (RES) {  // fused residual: s = x + r (rounded to T, as a separate add would store it)
#pragma unroll
      for (int q = 0; q < R; ++q)
#pragma unroll
        for (int k = 0; k < K; ++k) {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[q][k][j] += rv[q][k][j];
          round_to<T>(v[q][k]);
        }
    }
#pragma unroll
    for (int q = 0; q < R; ++q) {
      const int row = row0 + q;
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int c = (lane + 64 * k) * 8;
        if (c < C) {
          if constexpr (RES)
            if (row < N) Vec8<T>::store(sum_out + size_t(row) * C + c, v[q][k]);
#pragma unroll
          for (int j = 0; j < 8; ++j) s += v[q][k][j];
        }
      }
      const float mean = wave_sum(s) / float(C);
      float sq = 0.f;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int c = (lane + 64 * k) * 8;
        if (c < C)
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float d = v[q][k][j] - mean;
            sq = fmaf(d, d, sq);
          }
      }
      const float rstd = rsqrtf(wave_sum(sq) / float(C) + eps);
      if (row >= N) continue;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int c = (lane + 64 * k) * 8;
        if (c < C) {
          float o[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = fmaf((v[q][k][j] - mean) * rstd, wv[k][j], bv[k][j]);
          Vec8<T>::store(y + size_t(row) * C + c, o);
        }
      }
      if (lane == 0) {
        mean_out[row] = mean;
        rstd_out[row] = rstd;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// LayerNorm backward.  Per row (xhat = (x - mean) * rstd, g = dy * w):
//   dx = rstd * (g - mean(g) - xhat * mean(g * xhat))
// and per-block partial column sums of dy * xhat (dgamma) and dy (dbeta),
// combined across the block's 4 waves in fixed order through LDS.
// ---------------------------------------------------------------------------
template <typename T, int K, bool GS>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                     const float* __restrict__ w, const float* __restrict__ mean_in,
                                                     const float* __restrict__ rstd_in, const T* __restrict__ gs,
                                                     T* __restrict__ dx,
                                                     float* __restrict__ part_dw, float* __restrict__ part_db, int N,
                                                     int C) {
  extern __shared__ float sred[];  // [2][C]
  constexpr int R = 2;  // rows per wave whose loads are in flight together
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nw = gridDim.x * 4;
  float adw[K][8], adb[K][8];
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) adw[k][j] = adb[k][j] = 0.f;
  // Loads are unconditional (columns clamped to a valid chunk, unused values
  // masked at use; the residual branch is a template parameter): a load
  // under a branch gets its own s_waitcnt vmcnt(0), serialising the row.
  float wk[K][8];  // same for every row: loaded once
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int c = (lane + 64 * k) * 8;
    load8f(w + (c < C ? c : 0), wk[k]);
  }
  for (int row0 = (blockIdx.x * 4 + wave) * R; row0 < N; row0 += nw * R) {
    float xv[R][K][8], dv[R][K][8], gv[R][K][8], mean[R], rstd[R];
#pragma unroll
    for (int q = 0; q < R; ++q) {
      const int row = row0 + q < N ? row0 + q : N - 1;  // clamped: duplicates add nothing, store nothing
      mean[q] = mean_in[row];
      rstd[q] = rstd_in[row];
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int c = (lane + 64 * k) * 8, cc = c < C ? c : 0;
        Vec8<T>::load(x + size_t(row) * C + cc, xv[q][k]);
        Vec8<T>::load(dy + size_t(row) * C + cc, dv[q][k]);
        if constexpr (GS) Vec8<T>::load(gs + size_t(row) * C + cc, gv[q][k]);
      }
    }
#pragma unroll
    for (int q = 0; q < R; ++q) {
      const int row = row0 + q;
      const bool live = row < N;
      float xh[K][8], g[K][8];
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int c = (lane + 64 * k) * 8;
        if (c < C && live) {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            xh[k][j] = (xv[q][k][j] - mean[q]) * rstd[q];
            g[k][j] = dv[q][k][j] * wk[k][j];
            s1 += g[k][j];
            s2 = fmaf(g[k][j], xh[k][j], s2);
            adw[k][j] = fmaf(dv[q][k][j], xh[k][j], adw[k][j]);
            adb[k][j] += dv[q][k][j];
          }
        }
      }
      const float m1 = wave_sum(s1) / float(C), m2 = wave_sum(s2) / float(C);
      if (!live) continue;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int c = (lane + 64 * k) * 8;
        if (c < C) {
          float o[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = rstd[q] * (g[k][j] - m1 - xh[k][j] * m2);
          if constexpr (GS) {  // fused residual branch: dx += gradient arriving at the sum directly
#pragma unroll
            for (int j = 0; j < 8; ++j) o[j] += gv[q][k][j];
          }
          Vec8<T>::store(dx + size_t(row) * C + c, o);
        }
      }
    }
  }
  // fixed-order cross-wave sum of the column partials
  for (int wv = 0; wv < 4; ++wv) {
    if (wave == wv) {
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int c = (lane + 64 * k) * 8;
        if (c < C)
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            sred[c + j] = (wv == 0 ? 0.f : sred[c + j]) + adw[k][j];
            sred[C + c + j] = (wv == 0 ? 0.f : sred[C + c + j]) + adb[k][j];
          }
      }
    }
    __syncthreads();
  }
  for (int c = threadIdx.x; c < C; c += 256) {
    part_dw[size_t(blockIdx.x) * C + c] = sred[c];
    part_db[size_t(blockIdx.x) * C + c] = sred[C + c];
  }
}

// out[c] = sum_r part[r][c] (fixed order), for one or two partial arrays.
// Block = 16 columns x 16 row phases; each thread keeps 8 rows x 2 arrays of
// loads in flight, so R <= 384 partial rows take <= 3 rounds of memory
// latency (the previous 64 x 4 split needed up to 13: 6.7 us per call at
// the ViT sizes); the 16 phase partials are combined in LDS in fixed order.
constexpr int kCrCols = 16, kCrPh = 256 / kCrCols;
P2_DEVICE void col_reduce_body(const float* __restrict__ a, float* __restrict__ oa, const float* __restrict__ b,
                               float* __restrict__ ob, int R, int C, uint16_t* __restrict__ oa_bf, int cblock) {
  __shared__ float red[2][kCrPh][kCrCols];
  const int cl = threadIdx.x % kCrCols, q = threadIdx.x / kCrCols;
  const int c = cblock * kCrCols + cl;
  float sa = 0.f, sb = 0.f;
  if (c < C) {
    for (int r0 = q; r0 < R; r0 += kCrPh * 8) {
      float ta[8], tb[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int r = r0 + kCrPh * u;
        ta[u] = r < R ? a[size_t(r) * C + c] : 0.f;
        tb[u] = (b && r < R) ? b[size_t(r) * C + c] : 0.f;
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
  if (q == 0 && c < C) {
    float xa = 0.f, xb = 0.f;
#pragma unroll
    for (int p = 0; p < kCrPh; ++p) {
      xa += red[0][p][cl];
      xb += red[1][p][cl];
    }
    if (oa_bf)  // bf16 result (a bf16 parameter's gradient): no separate cast kernel
      oa_bf[c] = f32_to_bf16(xa);
    else
      oa[c] = xa;
    if (b) ob[c] = xb;
  }
}

__global__ __launch_bounds__(256) void col_reduce_kernel(const float* __restrict__ a, float* __restrict__ oa,
                                                         const float* __restrict__ b, float* __restrict__ ob, int R,
                                                         int C, uint16_t* __restrict__ oa_bf = nullptr) {
  col_reduce_body(a, oa, b, ob, R, C, oa_bf, blockIdx.x);
}

// Many column reductions in one launch (the parameter gradients whose reduction a
// training step defers to the end of its backward: LayerNorm dgamma / dbeta, bias
// gradients): the job table rides in the kernel arguments, a block takes the job
// whose block range holds blockIdx.x and runs exactly the col_reduce_kernel body,
// so every result is bitwise the separate launch's.
__global__ __launch_bounds__(256) void col_reduce_multi_kernel(CrJobs jobs) {
  int j = 0;
  while (j + 1 < jobs.n && int(blockIdx.x) >= jobs.j[j + 1].blk0) ++j;  // block-uniform
  const CrJob& t = jobs.j[j];
  col_reduce_body(t.a, t.oa, t.b, t.ob, t.R, t.C, t.oa_bf, int(blockIdx.x) - t.blk0);
}

void col_reduce_multi(CrJobs& jobs, hipStream_t s) {
  int blocks = 0;
  for (int i = 0; i < jobs.n; ++i) {
    jobs.j[i].blk0 = blocks;
    blocks += (jobs.j[i].C + kCrCols - 1) / kCrCols;
  }
  if (blocks > 0) hipLaunchKernelGGL(col_reduce_multi_kernel, dim3(blocks), dim3(256), 0, s, jobs);
}

// ---------------------------------------------------------------------------
// bias + GELU (exact erf form, = torch.nn.functional.gelu default)
// ---------------------------------------------------------------------------
// erf for the exact (erf) GELU, branch-free: Abramowitz & Stegun 7.1.26,
// |error| <= 1.5e-7 (plus fp32 rounding), i.e. far below the bf16 output
// rounding and inside the fp32 tests' 1e-5.  ~12 VALU instructions against
// ~80 for the library erff, which made the bias+GELU kernels VALU-bound.
P2_DEVICE float erf_as(float x) {
  const float a = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, a, 1.f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  const float r = 1.f - p * t * __expf(-a * a);
  return copysignf(r, x);
}
P2_DEVICE float gelu_f(float z) { return 0.5f * z * (1.f + erf_as(z * 0.70710678118654752f)); }
P2_DEVICE float gelu_grad(float z) {
  return 0.5f * (1.f + erf_as(z * 0.70710678118654752f)) + z * 0.39894228040143268f * __expf(-0.5f * z * z);
}

template <typename T>
__global__ __launch_bounds__(256) void bias_gelu_fwd_kernel(const T* __restrict__ x, const float* __restrict__ b,
                                                            T* __restrict__ y, int64_t n8, int H) {
  // two chunks per iteration, both loads issued before the (erf-heavy) math,
  // so each thread keeps a second chunk in flight while it computes
  const int64_t stride = int64_t(gridDim.x) * 256;
  for (int64_t i = blockIdx.x * int64_t(256) + threadIdx.x; i < n8; i += 2 * stride) {
    const int64_t i1 = i + stride < n8 ? i + stride : i;
    const int64_t e0 = i * 8, e1 = i1 * 8;
    float v[2][8], bv[2][8];
    Vec8<T>::load(x + e0, v[0]);
    Vec8<T>::load(x + e1, v[1]);
    load8f(b + int(e0 % H), bv[0]);
    load8f(b + int(e1 % H), bv[1]);
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int j = 0; j < 8; ++j) v[u][j] = gelu_f(v[u][j] + bv[u][j]);
    Vec8<T>::store(y + e0, v[0]);
    if (i1 != i) Vec8<T>::store(y + e1, v[1]);
  }
}

// dx = dy * gelu'(x + b); per-block partial column sums of dx (dbias).
// Grid (ceil(H / 512), S): 64 lanes x 8 columns per block, 4 row phases,
// rows strided by 4 * S.
template <typename T>
__global__ __launch_bounds__(256) void bias_gelu_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                            const float* __restrict__ b, T* __restrict__ dx,
                                                            float* __restrict__ part_db, int N, int H) {
  __shared__ float red[4][512];
  const int lane = threadIdx.x & 63, ph = threadIdx.x >> 6;
  const int c = (blockIdx.x * 64 + lane) * 8;
  const int S = gridDim.y;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c < H) {
    float bv[8];
    load8f(b + c, bv);
    // two rows per iteration, all four loads issued before the math (the
    // rows of a thread are otherwise one serial load -> compute chain)
    for (int r = blockIdx.y * 4 + ph; r < N; r += 8 * S) {
      const int r1 = r + 4 * S;
      const bool two = r1 < N;
      const int rr1 = two ? r1 : r;
      float xv[2][8], dv[2][8];
      Vec8<T>::load(x + size_t(r) * H + c, xv[0]);
      Vec8<T>::load(dy + size_t(r) * H + c, dv[0]);
      Vec8<T>::load(x + size_t(rr1) * H + c, xv[1]);
      Vec8<T>::load(dy + size_t(rr1) * H + c, dv[1]);
      float o[2][8];
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) o[u][j] = dv[u][j] * gelu_grad(xv[u][j] + bv[j]);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += o[0][j];
      Vec8<T>::store(dx + size_t(r) * H + c, o[0]);
      if (two) {
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += o[1][j];
        Vec8<T>::store(dx + size_t(r1) * H + c, o[1]);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[ph][lane * 8 + j] = acc[j];
  __syncthreads();
  for (int i = threadIdx.x; i < 512; i += 256) {
    const int cc = blockIdx.x * 512 + i;
    if (cc < H) part_db[size_t(blockIdx.y) * H + cc] = (red[0][i] + red[1][i]) + (red[2][i] + red[3][i]);
  }
}

// db[c] = sum_r dy[r][c] (bias gradient of a linear layer): same grid and
// fixed-order partials as bias_gelu_bwd, without the GELU and the dx write.
template <typename T>
P2_DEVICE void colsum_body(const T* __restrict__ dy, float* __restrict__ part, int N, int H, int bx, int by, int S) {
  __shared__ float red[4][512];
  const int lane = threadIdx.x & 63, ph = threadIdx.x >> 6;
  const int c = (bx * 64 + lane) * 8;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c < H) {
    for (int r = by * 4 + ph; r < N; r += 4 * S) {
      float dv[8];
      Vec8<T>::load(dy + size_t(r) * H + c, dv);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += dv[j];
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[ph][lane * 8 + j] = acc[j];
  __syncthreads();
  for (int i = threadIdx.x; i < 512; i += 256) {
    const int cc = bx * 512 + i;
    if (cc < H) part[size_t(by) * H + cc] = (red[0][i] + red[1][i]) + (red[2][i] + red[3][i]);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void colsum_kernel(const T* __restrict__ dy, float* __restrict__ part, int N, int H) {
  colsum_body<T>(dy, part, N, H, blockIdx.x, blockIdx.y, gridDim.y);
}

// The [S, H] column partials of many bf16 activations in one launch (the deferred bias
// gradients of a training step): block -> (job, column block, row split) through the job
// table in the kernel arguments; each block runs exactly colsum_kernel's body.
__global__ __launch_bounds__(256) void colsum_multi_kernel(CsJobs jobs) {
  int j = 0;
  while (j + 1 < jobs.n && int(blockIdx.x) >= jobs.j[j + 1].blk0) ++j;  // block-uniform
  const CsJob& t = jobs.j[j];
  const int nbx = (t.H + 511) / 512, lid = int(blockIdx.x) - t.blk0;
  colsum_body<uint16_t>(t.x, t.part, t.N, t.H, lid % nbx, lid / nbx, t.S);
}

void colsum_multi(CsJobs& jobs, hipStream_t s) {
  int blocks = 0;
  for (int i = 0; i < jobs.n; ++i) {
    jobs.j[i].blk0 = blocks;
    blocks += (jobs.j[i].H + 511) / 512 * jobs.j[i].S;
  }
  if (blocks > 0) hipLaunchKernelGGL(colsum_multi_kernel, dim3(blocks), dim3(256), 0, s, jobs);
}

// ---------------------------------------------------------------------------
// Softmax cross-entropy: loss_r = logsumexp(z_r) - z_r[y_r]; one wave per
// row, online max/sum per lane then combined across the wave.
// Backward: dz = (softmax(z) - onehot(y)) * (*gscale) / N, with the upstream
// gradient read from device memory (no host sync).
// ---------------------------------------------------------------------------
template <typename T>
P2_DEVICE float ld1(const T* p);
template <>
P2_DEVICE float ld1<uint16_t>(const uint16_t* p) { return bf16_to_f32(*p); }
template <>
P2_DEVICE float ld1<float>(const float* p) { return *p; }
template <typename T>
P2_DEVICE void st1(T* p, float v);
template <>
P2_DEVICE void st1<uint16_t>(uint16_t* p, float v) { *p = f32_to_bf16(v); }
template <>
P2_DEVICE void st1<float>(float* p, float v) { *p = v; }

template <typename T>
__global__ __launch_bounds__(256) void xent_fwd_kernel(const T* __restrict__ z, const int64_t* __restrict__ y,
                                                       float* __restrict__ loss, float* __restrict__ lse_out, int N,
                                                       int K) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= N) return;
  const T* zr = z + size_t(row) * K;
  float m = -INFINITY, s = 0.f;
  for (int k = lane; k < K; k += 64) {
    const float v = ld1<T>(zr + k);
    if (v > m) {
      s = s * __expf(m - v) + 1.f;
      m = v;
    } else {
      s += __expf(v - m);
    }
  }
  const float gm = wave_max(m);
  s = (m == -INFINITY) ? 0.f : s * __expf(m - gm);
  const float lse = gm + __logf(wave_sum(s));
  if (lane == 0) {
    const int64_t t = y[row];
    lse_out[row] = lse;
    loss[row] = (t >= 0 && t < K) ? lse - ld1<T>(zr + t) : 0.f;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void xent_bwd_kernel(const T* __restrict__ z, const int64_t* __restrict__ y,
                                                       const float* __restrict__ lse, const float* __restrict__ gscale,
                                                       T* __restrict__ dz, int N, int K, float inv_n) {
  const int64_t total = int64_t(N) * K;
  const float g = *gscale * inv_n;
  for (int64_t e = blockIdx.x * int64_t(256) + threadIdx.x; e < total; e += int64_t(gridDim.x) * 256) {
    const int row = int(e / K), k = int(e % K);
    const float p = __expf(ld1<T>(z + e) - lse[row]);
    st1<T>(dz + e, (p - (y[row] == k ? 1.f : 0.f)) * g);
  }
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
static int rows_grid(int N) {
  int g = (N + 3) / 4;
  return g > 4096 ? 4096 : (g < 1 ? 1 : g);
}

// ---------------------------------------------------------------------------
// ViT embedding: patchify of the uint8 batch, token concat + position embedding
// ---------------------------------------------------------------------------
// One thread per 8 consecutive patch-row elements (same channel and patch row,
// 8 adjacent pixels): one 8-byte load, one 16-byte store.  Replaces the float
// cast, the /255 multiply, the patch permute copy and the bf16 cast of the
// model's eager prologue (4 launches over the fp32 image).
__global__ __launch_bounds__(256) void patchify_u8_kernel(const uint8_t* __restrict__ x, uint16_t* __restrict__ out,
                                                          int B, int C, int H, int W, int P) {
  const int gw = W / P, np = (H / P) * gw, cols = C * P * P, c8 = cols / 8;
  const int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (i >= int64_t(B) * np * c8) return;
  const int64_t prow = i / c8;
  const int k = int(i - prow * c8) * 8;  // column within the patch row
  const int b = int(prow / np), pi = int(prow - int64_t(b) * np), py = pi / gw, px = pi - py * gw;
  const int c = k / (P * P), rem = k - c * P * P, iy = rem / P, ix = rem - iy * P;
  const uint2 u = *reinterpret_cast<const uint2*>(x + ((int64_t(b) * C + c) * H + py * P + iy) * W + px * P + ix);
  const uint32_t w[2] = {u.x, u.y};
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = float((w[j >> 2] >> (8 * (j & 3))) & 0xffu) * (1.f / 255.f);
  Vec8<uint16_t>::store(out + prow * cols + k, v);
}

void patchify_u8(const uint8_t* x, uint16_t* out, int B, int C, int H, int W, int P, hipStream_t s) {
  const int64_t n = int64_t(B) * (H / P) * (W / P) * (C * P * P / 8);
  hipLaunchKernelGGL(patchify_u8_kernel, dim3(int((n + 255) / 256)), dim3(256), 0, s, x, out, B, C, H, W, P);
}

// h = cat(cls, y) + pos, rounded once to bf16 (what the bf16 cat + add stored)
__global__ __launch_bounds__(256) void embed_tokens_fwd_kernel(const uint16_t* __restrict__ y,
                                                               const uint16_t* __restrict__ cls,
                                                               const uint16_t* __restrict__ pos, uint16_t* __restrict__ h,
                                                               int B, int N, int D) {
  const int d8 = D / 8;
  const int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (i >= int64_t(B) * (N + 1) * d8) return;
  const int64_t row = i / d8;
  const int k = int(i - row * d8) * 8;
  const int b = int(row / (N + 1)), t = int(row - int64_t(b) * (N + 1));
  float a[8], p[8];
  Vec8<uint16_t>::load(t == 0 ? cls + k : y + (int64_t(b) * N + t - 1) * D + k, a);
  Vec8<uint16_t>::load(pos + int64_t(t) * D + k, p);
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] += p[j];
  Vec8<uint16_t>::store(h + row * D + k, a);
}

// One thread per (token, 8 channels): the batch sum of dh in fixed order (fp32,
// rounded to the bf16 parameter gradient), and the patch tokens' rows copied out
// contiguously for the patch-embedding GEMM's backward -- all B loads in flight.
__global__ __launch_bounds__(256) void embed_tokens_bwd_kernel(const uint16_t* __restrict__ dh,
                                                               uint16_t* __restrict__ dy,
                                                               uint16_t* __restrict__ dpos,
                                                               uint16_t* __restrict__ dcls, int B, int N, int D) {
  const int d8 = D / 8;
  const int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (i >= int64_t(N + 1) * d8) return;
  const int t = int(i / d8), k = int(i - int64_t(t) * d8) * 8;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  constexpr int kU = 8;
  for (int b0 = 0; b0 < B; b0 += kU) {
    uint4 u[kU];
#pragma unroll
    for (int q = 0; q < kU; ++q)
      u[q] = b0 + q < B ? *reinterpret_cast<const uint4*>(dh + ((int64_t(b0 + q) * (N + 1)) + t) * D + k)
                        : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int q = 0; q < kU; ++q) {
      if (b0 + q >= B) break;
      if (t > 0) *reinterpret_cast<uint4*>(dy + (int64_t(b0 + q) * N + t - 1) * D + k) = u[q];
      const uint32_t w[4] = {u[q].x, u[q].y, u[q].z, u[q].w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[2 * j] += __uint_as_float(w[j] << 16);
        acc[2 * j + 1] += __uint_as_float(w[j] & 0xffff0000u);
      }
    }
  }
  Vec8<uint16_t>::store(dpos + int64_t(t) * D + k, acc);
  if (t == 0) Vec8<uint16_t>::store(dcls + k, acc);
}

void embed_tokens_fwd(const uint16_t* y, const uint16_t* cls, const uint16_t* pos, uint16_t* h, int B, int N, int D,
                      hipStream_t s) {
  const int64_t n = int64_t(B) * (N + 1) * (D / 8);
  hipLaunchKernelGGL(embed_tokens_fwd_kernel, dim3(int((n + 255) / 256)), dim3(256), 0, s, y, cls, pos, h, B, N, D);
}

void embed_tokens_bwd(const uint16_t* dh, uint16_t* dy, uint16_t* dpos, uint16_t* dcls, int B, int N, int D,
                      hipStream_t s) {
  const int64_t n = int64_t(N + 1) * (D / 8);
  hipLaunchKernelGGL(embed_tokens_bwd_kernel, dim3(int((n + 255) / 256)), dim3(256), 0, s, dh, dy, dpos, dcls, B, N, D);
}

template <typename T>
static void ln_fwd_t(const void* x, const void* r, const float* w, const float* b, void* y, void* sum, float* mean,
                     float* rstd, int N, int C, float eps, hipStream_t s) {
  // Rows per wave: R = 4 (all loads of 4 rows in flight, 394 blocks at ViT's
  // 6304 rows) measured 14.3 us per residual call in the ViT graph vs ~12 us
  // with one row per wave (1576 blocks): the per-row reductions of a wave
  // run serially, so more waves beat deeper per-wave batches here.  Kept
  // selectable; the default is one row per wave.
  constexpr int R = 4;
  const bool multi = false;
  const dim3 grid(multi ? (N + 4 * R - 1) / (4 * R) : rows_grid(N)), blk(256);
  const T* xp = static_cast<const T*>(x);
  const T* rp = static_cast<const T*>(r);
  T* yp = static_cast<T*>(y);
  T* sp = static_cast<T*>(sum);
#define P2_LN_FWD(KK, RR)                                                                                    \
  do {                                                                                                      \
    if (rp)                                                                                                 \
      hipLaunchKernelGGL((ln_fwd_kernel<T, KK, RR, true>), grid, blk, 0, s, xp, rp, w, b, yp, sp, mean, rstd, N, C, \
                         eps);                                                                              \
    else                                                                                                    \
      hipLaunchKernelGGL((ln_fwd_kernel<T, KK, RR, false>), grid, blk, 0, s, xp, rp, w, b, yp, sp, mean, rstd, N, \
                         C, eps);                                                                           \
  } while (0)
  if (C <= 512) {
    if (multi) P2_LN_FWD(1, R); else P2_LN_FWD(1, 1);
  } else if (C <= 1024) {
    if (multi) P2_LN_FWD(2, R); else P2_LN_FWD(2, 1);
  } else {
    if (multi) P2_LN_FWD(4, 2); else P2_LN_FWD(4, 1);
  }
#undef P2_LN_FWD
}

void layer_norm_fwd(bool bf16, const void* x, const void* residual, const float* w, const float* b, void* y,
                    void* sum, float* mean, float* rstd, int N, int C, float eps, hipStream_t s) {
  if (bf16)
    ln_fwd_t<uint16_t>(x, residual, w, b, y, sum, mean, rstd, N, C, eps, s);
  else
    ln_fwd_t<float>(x, residual, w, b, y, sum, mean, rstd, N, C, eps, s);
}

int layer_norm_bwd_blocks(int N) {
  // ~4 rows per wave: enough blocks to fill 256 CUs at ViT sizes (6304 rows ->
  // 394 blocks; the previous 16 rows per wave gave 99 blocks, 42 us/call),
  // while the [G, C] partials the column reduction reads stay a few MB.
  int g = (N + 15) / 16;
  return g > 1024 ? 1024 : (g < 1 ? 1 : g);
}

template <typename T>
static void ln_bwd_t(const void* dy, const void* x, const float* w, const float* mean, const float* rstd,
                     const void* gsum, void* dx, float* pdw, float* pdb, float* dw, float* db, int N, int C,
                     hipStream_t s) {
  const T* gp = static_cast<const T*>(gsum);
  const int G = layer_norm_bwd_blocks(N);
  const dim3 grid(G), blk(256);
  const size_t lds = size_t(2) * C * sizeof(float);
  const T* dyp = static_cast<const T*>(dy);
  const T* xp = static_cast<const T*>(x);
  T* dxp = static_cast<T*>(dx);
#define P2_LN_BWD(KK)                                                                                            \
  do {                                                                                                          \
    if (gp)                                                                                                     \
      hipLaunchKernelGGL((ln_bwd_kernel<T, KK, true>), grid, blk, lds, s, dyp, xp, w, mean, rstd, gp, dxp, pdw, pdb, N, \
                         C);                                                                                    \
    else                                                                                                        \
      hipLaunchKernelGGL((ln_bwd_kernel<T, KK, false>), grid, blk, lds, s, dyp, xp, w, mean, rstd, gp, dxp, pdw, pdb, \
                         N, C);                                                                                 \
  } while (0)
  if (C <= 512)
    P2_LN_BWD(1);
  else if (C <= 1024)
    P2_LN_BWD(2);
  else
    P2_LN_BWD(4);
#undef P2_LN_BWD
  if (dw) hipLaunchKernelGGL(col_reduce_kernel, dim3((C + kCrCols - 1) / kCrCols), blk, 0, s, pdw, dw, pdb, db, G, C);
}

void layer_norm_bwd(bool bf16, const void* dy, const void* x, const float* w, const float* mean, const float* rstd,
                    const void* gsum, void* dx, float* pdw, float* pdb, float* dw, float* db, int N, int C,
                    hipStream_t s) {
  if (bf16)
    ln_bwd_t<uint16_t>(dy, x, w, mean, rstd, gsum, dx, pdw, pdb, dw, db, N, C, s);
  else
    ln_bwd_t<float>(dy, x, w, mean, rstd, gsum, dx, pdw, pdb, dw, db, N, C, s);
}

void bias_gelu_fwd(bool bf16, const void* x, const float* b, void* y, int64_t n, int H, hipStream_t s) {
  const int64_t n8 = n / 8;
  const dim3 grid(stream_grid(n8, 256)), blk(256);
  if (bf16)
    hipLaunchKernelGGL(bias_gelu_fwd_kernel<uint16_t>, grid, blk, 0, s, static_cast<const uint16_t*>(x), b,
                       static_cast<uint16_t*>(y), n8, H);
  else
    hipLaunchKernelGGL(bias_gelu_fwd_kernel<float>, grid, blk, 0, s, static_cast<const float*>(x), b,
                       static_cast<float*>(y), n8, H);
}

int bias_gelu_bwd_splits(int N) {
  int S = (N + 31) / 32;
  return S > 128 ? 128 : (S < 1 ? 1 : S);
}

void bias_gelu_bwd(bool bf16, const void* dy, const void* x, const float* b, void* dx, float* pdb, float* db, int N,
                   int H, hipStream_t s) {
  const int S = bias_gelu_bwd_splits(N);
  const dim3 grid((H + 511) / 512, S), blk(256);
  if (bf16)
    hipLaunchKernelGGL(bias_gelu_bwd_kernel<uint16_t>, grid, blk, 0, s, static_cast<const uint16_t*>(dy),
                       static_cast<const uint16_t*>(x), b, static_cast<uint16_t*>(dx), pdb, N, H);
  else
    hipLaunchKernelGGL(bias_gelu_bwd_kernel<float>, grid, blk, 0, s, static_cast<const float*>(dy),
                       static_cast<const float*>(x), b, static_cast<float*>(dx), pdb, N, H);
  if (db)
    hipLaunchKernelGGL(col_reduce_kernel, dim3((H + kCrCols - 1) / kCrCols), blk, 0, s, pdb, db, nullptr, nullptr, S, H);
}

void column_sum(bool bf16, const void* dy, float* part, float* out, uint16_t* out_bf, int N, int H, hipStream_t s) {
  const int S = bias_gelu_bwd_splits(N);
  const dim3 grid((H + 511) / 512, S), blk(256);
  if (bf16)
    hipLaunchKernelGGL(colsum_kernel<uint16_t>, grid, blk, 0, s, static_cast<const uint16_t*>(dy), part, N, H);
  else
    hipLaunchKernelGGL(colsum_kernel<float>, grid, blk, 0, s, static_cast<const float*>(dy), part, N, H);
  if (out || out_bf)
    hipLaunchKernelGGL(col_reduce_kernel, dim3((H + kCrCols - 1) / kCrCols), blk, 0, s, part, out, nullptr, nullptr, S,
                       H, out_bf);
}

// ---------------------------------------------------------------------------
// out[i] = bf16(sum_s parts[s][i]), fp32 accumulation in fixed s order: the
// reduction of split-K weight-gradient partials (one pass; replaces a generic
// reduce kernel + a float->bf16 cast kernel).  n % 8 == 0, 16-B accesses.
// ---------------------------------------------------------------------------
// ---------------------------------------------------------------------------
// Multi-region device copy: up to kMaxCopies (dst, src, bytes) regions in ONE
// launch (a weight snapshot of several tensors was one blit kernel per region,
// ~5 us each on the learner's stream).  Workgroups stride over the regions'
// 16-byte chunks; a region's dword tail is copied by its first workgroup.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void multi_copy_kernel(p2fused::CopyList cl) {
  const int64_t stride = int64_t(gridDim.x) * 256;
  for (int r = 0; r < cl.n; ++r) {
    const int64_t n16 = cl.bytes[r] >> 4;
    const uint4* __restrict__ s16 = reinterpret_cast<const uint4*>(cl.src[r]);
    uint4* __restrict__ d16 = reinterpret_cast<uint4*>(cl.dst[r]);
    for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n16; i += stride) d16[i] = s16[i];
    const int64_t tail = (cl.bytes[r] & 15) >> 2;
    if (blockIdx.x == 0 && threadIdx.x < tail)
      reinterpret_cast<uint32_t*>(cl.dst[r])[n16 * 4 + threadIdx.x] = reinterpret_cast<const uint32_t*>(cl.src[r])[n16 * 4 + threadIdx.x];
  }
}

__global__ __launch_bounds__(256) void split_sum_bf16_kernel(const uint16_t* __restrict__ parts,
                                                             uint16_t* __restrict__ out, int64_t n8, int S) {
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n8; i += stride) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int sp = 0; sp < S; ++sp) {
      const uint4 u = reinterpret_cast<const uint4*>(parts + size_t(sp) * size_t(n8) * 8)[i];
      const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        acc[2 * k] += __uint_as_float(w[k] << 16);
        acc[2 * k + 1] += __uint_as_float(w[k] & 0xffff0000u);
      }
    }
    uint4 o;
    o.x = pack_bf16x2(acc[0], acc[1]);
    o.y = pack_bf16x2(acc[2], acc[3]);
    o.z = pack_bf16x2(acc[4], acc[5]);
    o.w = pack_bf16x2(acc[6], acc[7]);
    reinterpret_cast<uint4*>(out)[i] = o;
  }
}

void split_sum_bf16(const uint16_t* parts, uint16_t* out, int64_t n, int S, hipStream_t s) {
  const int64_t n8 = n / 8;
  hipLaunchKernelGGL(split_sum_bf16_kernel, dim3(stream_grid(n8, 256)), dim3(256), 0, s, parts, out, n8, S);
}

void multi_copy(const CopyList& cl, hipStream_t s) {
  int64_t chunks = 0;
  for (int r = 0; r < cl.n; ++r) chunks = std::max<int64_t>(chunks, cl.bytes[r] >> 4);
  const int grid = int(std::min<int64_t>(std::max<int64_t>((chunks + 255) / 256, 1), 2048));
  hipLaunchKernelGGL(multi_copy_kernel, dim3(grid), dim3(256), 0, s, cl);
}

void xent_fwd(bool bf16, const void* z, const int64_t* y, float* loss, float* lse, int N, int K, hipStream_t s) {
  const dim3 grid((N + 3) / 4), blk(256);
  if (bf16)
    hipLaunchKernelGGL(xent_fwd_kernel<uint16_t>, grid, blk, 0, s, static_cast<const uint16_t*>(z), y, loss, lse, N, K);
  else
    hipLaunchKernelGGL(xent_fwd_kernel<float>, grid, blk, 0, s, static_cast<const float*>(z), y, loss, lse, N, K);
}

void xent_bwd(bool bf16, const void* z, const int64_t* y, const float* lse, const float* gscale, void* dz, int N, int K,
              hipStream_t s) {
  const dim3 grid(stream_grid(int64_t(N) * K, 256)), blk(256);
  const float inv_n = 1.f / float(N);
  if (bf16)
    hipLaunchKernelGGL(xent_bwd_kernel<uint16_t>, grid, blk, 0, s, static_cast<const uint16_t*>(z), y, lse, gscale,
                       static_cast<uint16_t*>(dz), N, K, inv_n);
  else
    hipLaunchKernelGGL(xent_bwd_kernel<float>, grid, blk, 0, s, static_cast<const float*>(z), y, lse, gscale,
                       static_cast<float*>(dz), N, K, inv_n);
}

}  // namespace p2fused
