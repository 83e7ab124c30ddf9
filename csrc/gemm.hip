// Hand-written bf16 MFMA GEMM for the Linear layers (ViT blocks, MLP), gfx950.
//
// One kernel covers the three products of a Linear layer -- forward
// (x . W^T), input gradient (dY . W) and weight gradient (dY^T . x) -- by
// letting each operand be "k-major" (the reduction index contiguous in
// memory) or "mn-major" (the row/column index contiguous), so no operand is
// ever transposed in memory:
//
// * 128 x 128 output tile per 256-thread workgroup, 4 waves as 2 x 2, each
//   wave 64 x 64 = 2 x 2 tiles of v_mfma_f32_32x32x16_bf16, BK = 64;
// * operands go HBM -> LDS with global_load_lds (16 B per lane, no VGPR
//   round trip) into a double buffer: the next K-tile's loads are issued
//   before the current tile's MFMAs (one vmcnt(0) + barrier per K-tile);
// * k-major tiles are [128 rows][64 k] (128-B rows) read with ds_read_b128,
//   chunk XOR-swizzled by (row >> 1) & 7 (conflict-free 16-lane reads);
//   mn-major tiles are [64 k][128] (256-B rows) read with the gfx950
//   transpose read ds_read_b64_tr_b16, chunk XOR-swizzled by
//   ((row & 3) << 2 | (row >> 2) & 3) -- the swizzle is applied to the
//   per-lane GLOBAL address so the LDS image stays lane-linear for the DMA;
// * the MFMA is issued as (B, A) so the accumulator holds C with m on the
//   lane and 4 consecutive n per register group: the epilogue writes 8-B
//   (bf16) / 16-B (fp32) vectors along rows, with bias, GELU (+ its
//   pre-activation) and residual add fused;
// * workgroups are remapped so each XCD gets a contiguous run of tiles
//   (bijective for any grid size), and consecutive tiles share a B panel;
// * split-K (fp32 slabs) fills the chip when M x N has few tiles (weight
//   gradients reduce over the 6304 token rows).
//
// The reference has no GEMM of its own (Lightning/torch.nn.Linear); shapes
// from /root/reference/p2pfl/learning/pytorch/mnist_examples/models/mlp.py:53-69
// and the ViT-B config of BASELINE.json.
#include "common.h"
#include "gemm.h"

namespace p2gemm {
using namespace p2;

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

constexpr int BM = 128, BN = 128, BK = 64, NT = 256;
constexpr int TILE = BM * BK * 2;  // bytes per operand tile (16 KB)

P2_DEVICE f32x16 mfma(uint4 a, uint4 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c,
                                                  0, 0, 0);
}

P2_DEVICE int swz_k(int row) { return (row >> 1) & 7; }                       // k-major: 8 chunks / 128-B row
P2_DEVICE int swz_mn(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }  // mn-major: 16 chunks / 256-B row

// Issue the DMA of one operand tile (rows r0.. of the M or N dimension,
// reduction indices k0..k0+63) into `lds`.  Every lane loads 16 B four times;
// out-of-range rows / k are clamped onto valid memory (their products are
// masked in the epilogue / zeroed in the last K-tile).
template <bool KMAJ>
P2_DEVICE void stage(const uint16_t* __restrict__ g, int64_t ld, int nrows, int r0, int k0, int K, char* lds, int tid) {
  const int wave = tid >> 6;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int cid = i * NT + tid;
    char* dst = lds + (i * NT + wave * 64) * 16;  // wave-uniform; lane L writes dst + 16 L
    const uint16_t* src;
    if constexpr (KMAJ) {
      const int row = cid >> 3, c = (cid & 7) ^ swz_k(row);
      int gr = r0 + row;
      gr = gr < nrows ? gr : nrows - 1;
      int gk = k0 + 8 * c;
      gk = gk < K ? gk : K - 8;
      src = g + gr * ld + gk;
    } else {
      const int row = cid >> 4, ch = (cid & 15) ^ swz_mn(row);
      int gk = k0 + row;
      gk = gk < K ? gk : K - 1;
      int gc = r0 + 8 * ch;
      gc = gc < nrows ? gc : nrows - 8;
      src = g + gk * ld + gc;
    }
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
  }
}

// Fragment of a 32-row block (rows rb..rb+31 of the tile) for k-substep ks
// (k = 16 ks .. 16 ks + 15): lane l holds element (rb + (l & 31), 16 ks + 8 (l >> 5) + j), j = 0..7.
template <bool KMAJ>
P2_DEVICE uint4 frag(const char* lds, int rb, int ks, int lane) {
  if constexpr (KMAJ) {
    const int row = rb + (lane & 31), c = 2 * ks + (lane >> 5);
    return *reinterpret_cast<const uint4*>(lds + row * 128 + ((c ^ swz_k(row)) << 4));
  } else {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int col = rb + 16 * (g & 1) + 4 * p;  // this lane supplies 4 columns of row q
    const int ch = col >> 3, sub = (col & 7) * 2;
    uint4 out;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int row = 16 * ks + 8 * (g >> 1) + 4 * t + q;
      const char* addr = lds + row * 256 + ((ch ^ swz_mn(row)) << 4) + sub;
      const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) s16x4*)(addr));
      const uint2 u = __builtin_bit_cast(uint2, v);
      if (t == 0) {
        out.x = u.x;
        out.y = u.y;
      } else {
        out.z = u.x;
        out.w = u.y;
      }
    }
    return out;
  }
}

P2_DEVICE float gelu_f(float z) { return 0.5f * z * (1.f + erff(z * 0.70710678118654752f)); }

template <bool AK, bool BKM>
__global__ __launch_bounds__(NT, 2) void gemm_kernel(GemmParams p, int tiles_m, int tiles_n) {
  __shared__ __attribute__((aligned(16))) char smem[4 * TILE];  // [buf][A | B]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  // XCD-aware bijective remap: blocks that share an XCD get consecutive tile ids
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig % 8, q = nwg / 8, r = nwg % 8;
  const int bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
  const int tiles = tiles_m * tiles_n;
  const int split = bid / tiles, t = bid % tiles;
  const int tm = t % tiles_m, tn = t / tiles_m;  // consecutive tiles share the B panel
  const int m0 = tm * BM, n0 = tn * BN;
  int kper = (p.K + p.splits - 1) / p.splits;
  kper = (kper + BK - 1) / BK * BK;
  const int kb = split * kper, ke = min(p.K, kb + kper);
  const int nt = ke > kb ? (ke - kb + BK - 1) / BK : 0;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  if (nt > 0) {
    stage<AK>(p.a, p.lda, p.M, m0, kb, p.K, smem, tid);
    stage<BKM>(p.b, p.ldb, p.N, n0, kb, p.K, smem + TILE, tid);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  for (int it = 0; it < nt; ++it) {
    const int cur = it & 1;
    const char* sa = smem + cur * 2 * TILE;
    const char* sb = sa + TILE;
    if (it + 1 < nt) {
      char* na = smem + (cur ^ 1) * 2 * TILE;
      stage<AK>(p.a, p.lda, p.M, m0, kb + (it + 1) * BK, p.K, na, tid);
      stage<BKM>(p.b, p.ldb, p.N, n0, kb + (it + 1) * BK, p.K, na + TILE, tid);
    }
    const int kvalid = ke - (kb + it * BK);  // < BK only in the last tile of a ragged K
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      uint4 fa[2], fb[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) fa[i] = frag<AK>(sa, wm * 64 + i * 32, ks, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j) fb[j] = frag<BKM>(sb, wn * 64 + j * 32, ks, lane);
      if (kvalid < BK) {  // zero the A elements past K (B there is finite clamped data)
        const int k8 = 16 * ks + 8 * (lane >> 5);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          if (k8 >= kvalid) fa[i].x = fa[i].y = 0u;
          if (k8 + 4 >= kvalid) fa[i].z = fa[i].w = 0u;
        }
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma(fb[j], fa[i], acc[i][j]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ---- epilogue: lane holds C[m][n0 + ... + 8 g + 4 h + e] for its m
  const int h = lane >> 5;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = m0 + wm * 64 + i * 32 + (lane & 31);
    if (m >= p.M) continue;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int n = n0 + wn * 64 + j * 32 + 8 * g + 4 * h;
        if (n >= p.N) continue;  // N is a multiple of 4: a group is all in or all out
        float v[4] = {acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]};
        if (p.splits > 1) {
          float* slab = reinterpret_cast<float*>(p.c) + int64_t(split) * p.M * p.N + int64_t(m) * p.N + n;
          *reinterpret_cast<f32x4*>(slab) = f32x4{v[0], v[1], v[2], v[3]};
          continue;
        }
        if (p.bias) {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            v[e] += p.bias_bf16 ? bf16_to_f32(reinterpret_cast<const uint16_t*>(p.bias)[n + e])
                                : reinterpret_cast<const float*>(p.bias)[n + e];
        }
        const int64_t off = int64_t(m) * p.ldc + n;
        if (p.gelu) {
          if (p.z) *reinterpret_cast<uint2*>(p.z + off) = uint2{pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3])};
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = gelu_f(v[e]);
        }
        if (p.residual) {
          const uint2 rr = *reinterpret_cast<const uint2*>(p.residual + off);
          v[0] += __uint_as_float(rr.x << 16);
          v[1] += __uint_as_float(rr.x & 0xffff0000u);
          v[2] += __uint_as_float(rr.y << 16);
          v[3] += __uint_as_float(rr.y & 0xffff0000u);
        }
        if (p.c_bf16) {
          *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(p.c) + off) =
              uint2{pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3])};
        } else {
          *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(p.c) + off) = f32x4{v[0], v[1], v[2], v[3]};
        }
      }
    }
  }
}

}  // namespace p2gemm

namespace p2 {

void gemm_bf16(const GemmParams& p, hipStream_t s) {
  using namespace p2gemm;
  const int tiles_m = (p.M + BM - 1) / BM, tiles_n = (p.N + BN - 1) / BN;
  const int grid = tiles_m * tiles_n * (p.splits > 1 ? p.splits : 1);
  GemmParams q = p;
  if (q.splits < 1) q.splits = 1;
  if (p.a_kmajor && p.b_kmajor)
    hipLaunchKernelGGL((gemm_kernel<true, true>), dim3(grid), dim3(NT), 0, s, q, tiles_m, tiles_n);
  else if (p.a_kmajor)
    hipLaunchKernelGGL((gemm_kernel<true, false>), dim3(grid), dim3(NT), 0, s, q, tiles_m, tiles_n);
  else if (p.b_kmajor)
    hipLaunchKernelGGL((gemm_kernel<false, true>), dim3(grid), dim3(NT), 0, s, q, tiles_m, tiles_n);
  else
    hipLaunchKernelGGL((gemm_kernel<false, false>), dim3(grid), dim3(NT), 0, s, q, tiles_m, tiles_n);
}

}  // namespace p2
