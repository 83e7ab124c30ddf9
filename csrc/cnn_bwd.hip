// Fused MNIST-CNN training step -- backward kernels with fused Adam epilogues.
// Layouts: see cnn_fwd.hip.  Backward buffers:
//   dH     bf16 [mrows][2048]      dLoss/dH (ReLU mask applied), rows >= B are zero
//   dC2m   bf16 [mrows][64][224]   dC2 map, positions laid out 14 rows x 16 cols (cols 14/15 zero)
//   gB     f32  [mrows][3136]      alive-masked dA1 (conv2 bias gradient terms)
//   W2q    bf16 [32][25][64]       conv2 weight, (ic, tap, oc) -- transposed-conv B operand
//   wslab1 f32  [B][7][832]        conv1 weight/bias partials per (image, position tile)
//   wslab2 f32  [ceil(B/2)][25][64][32]  conv2 weight partials per image pair, (tap, oc, ic)
// Every reduction has a fixed order (no float atomics), so a step is bitwise
// reproducible -- required because Adam amplifies last-bit differences in
// near-zero gradients.  Adam's step count is (*adam_t + t_off): a device base
// plus an offset baked into each launch, so a whole epoch is one HIP graph.
#include <cstdlib>

#include "cnn.h"
#include "cnn_fwd_dev.h"
#include "common.h"

namespace p2cnn {
using namespace p2;

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
P2_DEVICE f32x16 mfma32b(uint4 a, uint4 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c,
                                                  0, 0, 0);
}
P2_DEVICE int acc_row_b(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }
P2_DEVICE uint4 pack8(const uint16_t (&v)[8]) {
  uint4 q;
  q.x = uint32_t(v[0]) | (uint32_t(v[1]) << 16);
  q.y = uint32_t(v[2]) | (uint32_t(v[3]) << 16);
  q.z = uint32_t(v[4]) | (uint32_t(v[5]) << 16);
  q.w = uint32_t(v[6]) | (uint32_t(v[7]) << 16);
  return q;
}

struct AdamScal {
  float step_size, inv_sqrt_bc2;
};
P2_DEVICE AdamScal adam_scal(const AdamCfg& c, const int* t, int t_off) {
  const float tt = float(*t + t_off);
  AdamScal s;
  s.step_size = c.lr / (1.f - powf(c.beta1, tt));
  s.inv_sqrt_bc2 = 1.f / sqrtf(1.f - powf(c.beta2, tt));
  return s;
}
// m / (sqrt(v) c + eps) with the hardware square root and reciprocal (v_sqrt_f32,
// v_rcp_f32: 1 ulp each) instead of the correctly rounded sequences (~20 VALU
// instructions per element more: the Adam streams are issue-bound beside their
// memory traffic, profiles/r4_cnn_pmc.md).  The update differs from the IEEE one
// in the last bit of an lr-sized step.
P2_DEVICE float adam_dir(float mv, float vv, float c, float eps) {
  return mv * __builtin_amdgcn_rcpf(fmaf(__builtin_amdgcn_sqrtf(vv), c, eps));
}
// torch.optim.Adam semantics (L2 weight decay added to the gradient), on
// values already in registers (lets a caller batch its loads).
P2_DEVICE void adam_regs(float& pv, float& mv, float& vv, float g, const AdamCfg& c, const AdamScal& s) {
  if (c.weight_decay != 0.f) g = fmaf(c.weight_decay, pv, g);
  mv = fmaf(c.beta1, mv, (1.f - c.beta1) * g);
  vv = fmaf(c.beta2, vv, (1.f - c.beta2) * g * g);
  pv -= s.step_size * adam_dir(mv, vv, s.inv_sqrt_bc2, c.eps);
}
// Same, loading and storing in place.
P2_DEVICE float adam_apply(float* __restrict__ p, float* __restrict__ m, float* __restrict__ v, int64_t e, float g,
                           const AdamCfg& c, const AdamScal& s) {
  float pv = p[e];
  if (c.weight_decay != 0.f) g = fmaf(c.weight_decay, pv, g);
  const float mv = fmaf(c.beta1, m[e], (1.f - c.beta1) * g);
  const float vv = fmaf(c.beta2, v[e], (1.f - c.beta2) * g * g);
  pv -= s.step_size * adam_dir(mv, vv, s.inv_sqrt_bc2, c.eps);
  p[e] = pv;
  m[e] = mv;
  v[e] = vv;
  return pv;
}

// ---------------------------------------------------------------------------
// 5+6. One launch, two independent block roles (both only need the head's
//    outputs, so sharing a launch saves a kernel boundary):
//  * blocks [0, 98): dA1 = dH x W1 on MFMA with the pool2/ReLU backward fused
//    into the epilogue.  32 features per block, 8 waves splitting K = 2048 in
//    64-wide groups (same streaming scheme and k permutation as gemm_skinny),
//    all of a wave's loads issued before its first MFMA, partial tiles reduced
//    in LDS in fixed wave order.  Each output (b, feature) is routed to the
//    argmax of its 2x2 pooling window; all four window positions of the dC2
//    map are written (so it never needs clearing), plus the fp32 alive-masked
//    dA1 (conv2 bias terms).  The block's 32 features are contiguous, so its
//    dC2 rows are shared with at most one neighbour block.
//  * blocks [98, 139): FC2 weight/bias gradient + Adam, one thread per
//    parameter: dW2[c][k] = sum_b dlogits[b][c] H[b][k].
// ---------------------------------------------------------------------------
constexpr int kRouteBlocks = kFeat / 32;                       // 98
constexpr int kFc2Blocks = (kCls * kHid + kCls + 511) / 512;   // 41 (512-thread blocks)

template <int TPB>
P2_DEVICE void fc2_role(int blk, const float* __restrict__ dlogits, const uint16_t* __restrict__ H, int B,
                        float* __restrict__ p, float* __restrict__ m, float* __restrict__ v,
                        float* __restrict__ gdump, const Offsets& off, const int* __restrict__ adam_t, int t_off,
                        const AdamCfg& cfg, uint16_t* __restrict__ w2bf = nullptr) {
  const int e = blk * TPB + threadIdx.x;
  const int nW = kCls * kHid;
  if (e >= nW + kCls) return;
  const int64_t pi = e < nW ? off.l2w + e : off.l2b + (e - nW);
  float pv = p[pi], mv = m[pi], vv = v[pi];  // issued before the reduction's loads
  float g = 0.f;
  if (e < nW) {
    const int c = e / kHid, k = e % kHid;
    for (int b0 = 0; b0 < B; b0 += 8) {
      float t[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        t[u] = b0 + u < B ? dlogits[(b0 + u) * kCls + c] * bf16_to_f32(H[size_t(b0 + u) * kHid + k]) : 0.f;
#pragma unroll
      for (int u = 0; u < 8; ++u) g += t[u];
    }
  } else {
    const int c = e - nW;
    for (int b = 0; b < B; ++b) g += dlogits[b * kCls + c];
  }
  if (gdump) gdump[pi] = g;
  const AdamScal s = adam_scal(cfg, adam_t, t_off);
  adam_regs(pv, mv, vv, g, cfg, s);
  p[pi] = pv;
  m[pi] = mv;
  v[pi] = vv;
  if (w2bf && e < nW) w2bf[e] = f32_to_bf16(pv);  // the head's bf16 copy of W2
}

template <int MT>
__global__ __launch_bounds__(512) void route_fc2_kernel(const uint16_t* __restrict__ dH,
                                                        const uint16_t* __restrict__ w1t,
                                                        const uint8_t* __restrict__ am2, int B,
                                                        uint16_t* __restrict__ dc2m, float* __restrict__ gb,
                                                        const float* __restrict__ dlogits,
                                                        const uint16_t* __restrict__ H, float* __restrict__ p,
                                                        float* __restrict__ m, float* __restrict__ v,
                                                        float* __restrict__ gdump, Offsets off,
                                                        const int* __restrict__ adam_t, int t_off, AdamCfg cfg) {
  const int bid = blockIdx.x;
  if (bid >= kRouteBlocks) {
    fc2_role<512>(bid - kRouteBlocks, dlogits, H, B, p, m, v, gdump, off, adam_t, t_off, cfg);
    return;
  }
  __shared__ float red[8 * MT * 1024];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const int n0 = bid * 32;
  constexpr int K = kHid, NG = K / 64;
  // argmax codes of this thread's epilogue elements (independent of the GEMM)
  uint8_t acode[2 * MT];
#pragma unroll
  for (int q = 0; q < 2 * MT; ++q) {
    const int e = tid + 512 * q;
    const int b = (e >> 10) * 32 + acc_row_b((e >> 6) & 15, (e & 63) >> 5);
    acode[q] = b < B ? am2[size_t(b) * kFeat + n0 + (e & 31)] : uint8_t(4);
  }
  f32x16 acc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x16{};
  const uint16_t* brow = w1t + size_t(n0 + r) * K + 32 * h;
  // all of this wave's loads are issued before the first MFMA (one memory
  // round-trip instead of one per k-group)
  constexpr int NGW = NG / 8;
  uint4 bq[NGW][4], aq[NGW][MT][4];
#pragma unroll
  for (int gi = 0; gi < NGW; ++gi) {
    const int k0 = (wave + 8 * gi) * 64;
#pragma unroll
    for (int q = 0; q < 4; ++q) bq[gi][q] = ld_nt16(brow + k0 + q * 8);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        aq[gi][mt][q] = reinterpret_cast<const uint4*>(dH + size_t(mt * 32 + r) * K + 32 * h + k0)[q];
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int gi = 0; gi < NGW; ++gi)
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) acc[mt] = mfma32b(aq[gi][mt][q], bq[gi][q], acc[mt]);
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int i = 0; i < 16; ++i) red[((wave * MT + mt) * 16 + i) * 64 + lane] = acc[mt][i];
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 2 * MT; ++q) {
    const int e = tid + 512 * q;
    float g = 0.f;
#pragma unroll
    for (int w = 0; w < 8; ++w) g += red[w * MT * 1024 + e];
    const int mt = e >> 10, i = (e >> 6) & 15, ln = e & 63;
    const int b = mt * 32 + acc_row_b(i, ln >> 5), feat = n0 + (ln & 31);
    if (b >= B) continue;
    const uint8_t a = acode[q];
    const int oc = feat / 49, pp = feat % 49, py = pp / 7, px = pp % 7;
    gb[size_t(b) * kFeat + feat] = a < 4 ? g : 0.f;
    const uint16_t gv = f32_to_bf16(g);
    uint16_t* row = dc2m + (size_t(b) * kC2 + oc) * 224 + (2 * py) * 16 + 2 * px;
    // two 4-byte stores: (dy=0: dx 0,1) and (dy=1: dx 0,1)
    const uint32_t top = (a == 0 ? gv : 0u) | (uint32_t(a == 1 ? gv : 0u) << 16);
    const uint32_t bot = (a == 2 ? gv : 0u) | (uint32_t(a == 3 ? gv : 0u) << 16);
    *reinterpret_cast<uint32_t*>(row) = top;
    *reinterpret_cast<uint32_t*>(row + 16) = bot;
  }
}

// Same dA1 routing, reading the row-major FC1 weight W1 [2048][3136] (the
// forward operand) instead of a transposed W1^T shadow, so the FC1 Adam
// stream no longer writes 12.8 MB of W1^T per step.  Each wave DMAs its 256 K
// rows of the block's 32 feature columns (64 B per row) into LDS, and reads
// the B fragments back with ds_read_b64_tr_b16: per 16-lane group 4 rows x 16
// columns delivered column-major.  Same k permutation as the W1^T kernel
// (lane half h, sub-step q -> physical k = k0 + 32 h + 8 q + j), so the A
// fragments (dH rows) are unchanged.  A 32-lane half reads 4 rows x 64 B =
// 256 contiguous bytes: conflict-free.  128 KB of LDS: one block per CU (98
// blocks), the reduction buffer aliases the tile after the MFMAs.
constexpr int kRouteRmLds = kHid * 64;  // 131072 B

// Workgroups are dispatched round-robin over the 8 XCDs; renumber so that
// consecutive logical blocks share an XCD (and its L2): route_rm's blocks 2j
// and 2j+1 read the two 64-B halves of the same 128-B lines of W1.
P2_DEVICE int xcd_local(int orig, int nwg) {
  const int xcd = orig % 8, q = nwg / 8, r = nwg % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

// Write-through (sc1) store / load of a split-K partial: the tile's last
// arriving K-slice reads the others' partials from another CU (possibly another
// XCD), so they bypass the non-coherent L1 / per-XCD L2 (the hand-off of
// gemm_core.h: drain vmcnt, barrier, relaxed agent-scope ticket).
P2_DEVICE void st_sc1f(float* p, float v) {
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(p, 0, 4, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rs, 0, 0, 16);
}
P2_DEVICE float ld_sc1f(const float* p) {
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), 0, 4, 0x00020000);
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, 0, 0, 16));
}

// KS > 1: split-K over KS workgroups per 32-feature tile (98 x KS blocks).  The
// kernel is bound by what one CU can pull (each tile block streams 128 KB of W1
// and re-reads the 128 KB dH: ~11 B/cycle/CU, MI355X_MICROARCH.md), so with 98
// blocks 158 CUs idle; KS = 2 halves the bytes per block.  Each slice reduces its
// 8 waves in LDS, stores its fp32 partial (sc1), and the last slice to take the
// tile's ticket sums the KS partials in slice order (deterministic, whichever
// slice arrives last) and runs the routing epilogue.  ws: [98][KS][MT*1024] fp32,
// ctr: [98] int, zero between launches (the last arriver resets its entry).
template <int MT, int KS>
__global__ __launch_bounds__(512) void route_rm_kernel(const uint16_t* __restrict__ dH,
                                                       const uint16_t* __restrict__ w1,
                                                       const uint8_t* __restrict__ am2, int B,
                                                       uint16_t* __restrict__ dc2m, float* __restrict__ gb,
                                                       const float* __restrict__ dlogits,
                                                       const uint16_t* __restrict__ H, float* __restrict__ p,
                                                       float* __restrict__ m, float* __restrict__ v,
                                                       float* __restrict__ gdump, Offsets off,
                                                       const int* __restrict__ adam_t, int t_off, AdamCfg cfg,
                                                       float* __restrict__ ws, int* __restrict__ ctr, int xa) {
  constexpr int NB = kRouteBlocks * KS;
  // xa > 0 (KS = 1): 8 x xa routing blocks, block b on XCD b % 8 takes feature tile
  // (b % 8) xa + b / 8 -- the tiles of FC1 split b % 8, whose W1 columns the skinny
  // GEMM's blocks on that XCD just read into its L2 (gemm_skinny_kernel XA)
  const int nbl = xa ? 8 * xa : NB;
  if (int(blockIdx.x) >= nbl) {
    fc2_role<512>(blockIdx.x - nbl, dlogits, H, B, p, m, v, gdump, off, adam_t, t_off, cfg);
    return;
  }
  int bid;
  if (xa) {
    const int x = blockIdx.x & 7, r = blockIdx.x >> 3;
    bid = x * xa + r;
    if (bid >= NB) return;
  } else {
    bid = xcd_local(blockIdx.x, NB);
  }
  const int tile = bid / KS, split = bid % KS;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  static_assert(8 * MT * 1024 * 4 <= kRouteRmLds / KS, "reduction buffer must fit the tile");
  float* red = reinterpret_cast<float*>(smem);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const int n0 = tile * 32;
  constexpr int K = kHid, NG = K / 64, NGW = NG / 8 / KS;
  const int gbase = split * (NG / KS);  // first 64-wide k-group of this slice
  uint8_t acode[2 * MT];
#pragma unroll
  for (int q = 0; q < 2 * MT; ++q) {
    const int e = tid + 512 * q;
    const int b = (e >> 10) * 32 + acc_row_b((e >> 6) & 15, (e & 63) >> 5);
    acode[q] = b < B ? am2[size_t(b) * kFeat + n0 + (e & 31)] : uint8_t(4);
  }
  // W1 rows of this wave's k-groups -> LDS [k - kbase][32 features] (64-B rows):
  // one wave instruction = 16 rows x 4 lanes x 16 B
#pragma unroll
  for (int gi = 0; gi < NGW; ++gi) {
    const int kl = (wave + 8 * gi) * 64, k0 = gbase * 64 + kl;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int row = k0 + 16 * c + (lane >> 2);
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(w1 + size_t(row) * kFeat + n0 + (lane & 3) * 8),
          (__attribute__((address_space(3))) void*)(smem + (kl + 16 * c) * 64), 16, 0, 0);
    }
  }
  uint4 aq[NGW][MT][4];
#pragma unroll
  for (int gi = 0; gi < NGW; ++gi) {
    const int k0 = (gbase + wave + 8 * gi) * 64;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        aq[gi][mt][q] = reinterpret_cast<const uint4*>(dH + size_t(mt * 32 + r) * K + 32 * h + k0)[q];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  f32x16 acc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x16{};
  const int g = lane >> 4, qq = (lane >> 2) & 3, col = 16 * (g & 1) + 4 * (lane & 3);
#pragma unroll
  for (int gi = 0; gi < NGW; ++gi) {
    const int kl = (wave + 8 * gi) * 64;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      uint4 bq;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int row = kl + 32 * (g >> 1) + 8 * q + 4 * t + qq;
        const s16x4 w = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4*)(smem + row * 64 + col * 2));
        const uint2 u = __builtin_bit_cast(uint2, w);
        if (t == 0) {
          bq.x = u.x;
          bq.y = u.y;
        } else {
          bq.z = u.x;
          bq.w = u.y;
        }
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) acc[mt] = mfma32b(aq[gi][mt][q], bq, acc[mt]);
    }
  }
  __syncthreads();  // tile dead -> reduction buffer
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int i = 0; i < 16; ++i) red[((wave * MT + mt) * 16 + i) * 64 + lane] = acc[mt][i];
  __syncthreads();
  float part[2 * MT];
#pragma unroll
  for (int q = 0; q < 2 * MT; ++q) {
    const int e = tid + 512 * q;
    float gsum = 0.f;
#pragma unroll
    for (int w = 0; w < 8; ++w) gsum += red[w * MT * 1024 + e];
    part[q] = gsum;
  }
  if (KS > 1) {
    float* slab = ws + size_t(tile) * KS * (MT * 1024);
#pragma unroll
    for (int q = 0; q < 2 * MT; ++q) st_sc1f(slab + split * (MT * 1024) + tid + 512 * q, part[q]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // every wave's partial written; the reduction buffer is dead
    int* flag = reinterpret_cast<int*>(smem);
    if (tid == 0) {
      const int old = __hip_atomic_fetch_add(ctr + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      flag[0] = old == KS - 1;
      if (old == KS - 1) __hip_atomic_store(ctr + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!flag[0]) return;
#pragma unroll
    for (int q = 0; q < 2 * MT; ++q) {
      float t = 0.f;
#pragma unroll
      for (int s2 = 0; s2 < KS; ++s2) t += s2 == split ? part[q] : ld_sc1f(slab + s2 * (MT * 1024) + tid + 512 * q);
      part[q] = t;
    }
  }
#pragma unroll
  for (int q = 0; q < 2 * MT; ++q) {
    const int e = tid + 512 * q;
    const float gsum = part[q];
    const int mt = e >> 10, i = (e >> 6) & 15, ln = e & 63;
    const int b = mt * 32 + acc_row_b(i, ln >> 5), feat = n0 + (ln & 31);
    if (b >= B) continue;
    const uint8_t a = acode[q];
    const int oc = feat / 49, pp = feat % 49, py = pp / 7, px = pp % 7;
    gb[size_t(b) * kFeat + feat] = a < 4 ? gsum : 0.f;
    const uint16_t gv = f32_to_bf16(gsum);
    uint16_t* row = dc2m + (size_t(b) * kC2 + oc) * 224 + (2 * py) * 16 + 2 * px;
    const uint32_t top = (a == 0 ? gv : 0u) | (uint32_t(a == 1 ? gv : 0u) << 16);
    const uint32_t bot = (a == 2 ? gv : 0u) | (uint32_t(a == 3 ? gv : 0u) << 16);
    *reinterpret_cast<uint32_t*>(row) = top;
    *reinterpret_cast<uint32_t*>(row + 16) = bot;
  }
}

void route_fc2_rm(const uint16_t* dH, const uint16_t* w1, const uint8_t* am2, int mrows, int B, uint16_t* dc2m,
                  float* gb, const float* dlogits, const uint16_t* H, float* params, float* m, float* v,
                  float* gdump, Offsets off, const int* adam_t, int t_off, AdamCfg cfg, bool with_fc2,
                  float* ws, int* ctr, hipStream_t s) {
  const int ks = (ws && ctr) ? 2 : 1;
  const int xa = (ks == 1 && xcd_align()) ? kRouteBlocks / kXcdSplits : 0;
  static_assert(kRouteBlocks % kXcdSplits == 0 && kXcdSplits <= 8, "routing tiles split evenly over the aligned XCDs");
  const dim3 grid((xa ? 8 * xa : kRouteBlocks * ks) + (with_fc2 ? kFc2Blocks : 0));
  const int lds = kRouteRmLds / ks;
#define P2_ROUTE(MT, KS)                                                                                            \
  hipLaunchKernelGGL((route_rm_kernel<MT, KS>), grid, dim3(512), lds, s, dH, w1, am2, B, dc2m, gb, dlogits, H, params, \
                     m, v, gdump, off, adam_t, t_off, cfg, ws, ctr, xa)
  if (mrows == 32) {
    if (ks == 2) P2_ROUTE(1, 2); else P2_ROUTE(1, 1);
  } else {
    if (ks == 2) P2_ROUTE(2, 2); else P2_ROUTE(2, 1);
  }
#undef P2_ROUTE
}

void route_fc2(const uint16_t* dH, const uint16_t* w1t, const uint8_t* am2, int mrows, int B, uint16_t* dc2m,
               float* gb, const float* dlogits, const uint16_t* H, float* params, float* m, float* v, float* gdump,
               Offsets off, const int* adam_t, int t_off, AdamCfg cfg, bool with_fc2, hipStream_t s) {
  const dim3 grid(kRouteBlocks + (with_fc2 ? kFc2Blocks : 0));
  if (mrows == 32)
    hipLaunchKernelGGL(route_fc2_kernel<1>, grid, dim3(512), 0, s, dH, w1t, am2, B, dc2m, gb, dlogits, H, params, m,
                       v, gdump, off, adam_t, t_off, cfg);
  else
    hipLaunchKernelGGL(route_fc2_kernel<2>, grid, dim3(512), 0, s, dH, w1t, am2, B, dc2m, gb, dlogits, H, params, m,
                       v, gdump, off, adam_t, t_off, cfg);
}

// ---------------------------------------------------------------------------
// 7. FC1 weight gradient on MFMA with Adam fused into the epilogue.
//    dW1[n][k] = sum_b dH[b][n] * A1[b][k]  (K = batch).  Grid (25, 64):
//    block = 32 rows of n x 128 columns of k, one 32x32 tile per wave.  The
//    batch-major dH / A1 tiles are transposed through LDS (so no transposed
//    copies live in HBM).  The gradient tile never leaves the chip: it goes
//    from the MFMA accumulators through LDS into a row-major layout where
//    every lane owns 4 consecutive k of one row, so W1 / m / v move as 16-B
//    accesses (issued before the staging, so their latency overlaps it) and
//    the bf16 shadow as 8-B stores; W1^T is written as 16-B row segments from
//    a transposed bf16 tile.  (The accumulator-layout epilogue it replaces did
//    4-B / 2-B accesses: 37.0 -> 35.1 us per call, bitwise-identical results,
//    tools/lab/fc1_lab.hip.)
// ---------------------------------------------------------------------------
template <int MR>
struct Fc1Lds {
  static constexpr int AP = 144;  // bf16 pitch of the staged A1 rows (288 B: conflict-free transpose reads)
  static constexpr int GP = 132;  // fp32 pitch of the gradient tile
  static constexpr int kStage = MR * (32 + AP) * 2;  // dH rows [MR][32] | A1 rows [MR][AP]
  static constexpr int kGrad = 32 * GP * 4;
  static constexpr int kMain = kStage > kGrad ? kStage : kGrad;
  static constexpr int kBytes = kMain + 128 * 40 * 2;  // + the transposed bf16 tile
};

template <int MR>
P2_DEVICE void fc1_wgrad_adam_body(int bx, int by, const uint16_t* __restrict__ dH, const uint16_t* __restrict__ a1,
                                   float* __restrict__ p, float* __restrict__ m, float* __restrict__ v,
                                   float* __restrict__ gdump, uint16_t* __restrict__ w1bf,
                                   uint16_t* __restrict__ w1tbf, const Offsets& off,
                                   const int* __restrict__ adam_t, int t_off, const AdamCfg& cfg, char* smem) {
  constexpr int AP = Fc1Lds<MR>::AP;
  constexpr int GP = Fc1Lds<MR>::GP;
  uint16_t(*tr)[40] = reinterpret_cast<uint16_t(*)[40]>(smem + Fc1Lds<MR>::kMain);
  // dH and A1 are staged as they lie in memory (sample rows, 16-B LDS writes) and the
  // MFMA fragments are read with the gfx950 transpose read (ds_read_b64_tr_b16): the
  // transposed staging it replaces was 24 two-byte LDS writes per thread, 84 % of the
  // kernel's LDS-active cycles in bank conflicts (profiles/r4_cnn_pmc.md)
  uint16_t* sdh = reinterpret_cast<uint16_t*>(smem);  // [MR][32]  dH[b][n0 + n]
  uint16_t* sa1 = sdh + MR * 32;                      // [MR][AP]  A1[b][kb + k]
  float(*gt)[GP] = reinterpret_cast<float(*)[GP]>(smem);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const int n0 = by * 32;
  const int kb = bx * 128;
  // this thread's Adam elements: row nl, k = kb + kq + 32 j + [0, 4)
  const int nl = tid >> 3, kq = (tid & 7) * 4;
  float* pw = p + off.l1w;
  float* mw = m + off.l1w;
  float* vw = v + off.l1w;
  float4 pr[4], mr[4], vr[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int k = kb + kq + 32 * j;
    if (k < kFeat) {
      const int64_t e = int64_t(n0 + nl) * kFeat + k;
      pr[j] = *reinterpret_cast<const float4*>(pw + e);
      mr[j] = *reinterpret_cast<const float4*>(mw + e);
      vr[j] = *reinterpret_cast<const float4*>(vw + e);
    }
  }
  for (int i = tid; i < MR * 4; i += 256) {
    const int b = i >> 2, q = i & 3;
    *reinterpret_cast<uint4*>(sdh + b * 32 + q * 8) = reinterpret_cast<const uint4*>(dH + size_t(b) * kHid + n0)[q];
  }
  for (int i = tid; i < MR * 16; i += 256) {
    const int b = i >> 4, q = i & 15;
    const int k = kb + q * 8;
    uint4 u = make_uint4(0, 0, 0, 0);
    if (k < kFeat) u = reinterpret_cast<const uint4*>(a1 + size_t(b) * kFeat + k)[0];
    *reinterpret_cast<uint4*>(sa1 + b * AP + q * 8) = u;
  }
  __syncthreads();
  const AdamScal s = adam_scal(cfg, adam_t, t_off);
  if (bx == 0 && wave == 0 && lane < 32) {  // FC1 bias (reads the staged dH before the tile reuses it)
    const int n = n0 + lane;
    float g = 0.f;
    for (int b = 0; b < MR; ++b) g += bf16_to_f32(sdh[b * 32 + lane]);
    if (gdump) gdump[off.l1b + n] = g;
    adam_apply(p, m, v, off.l1b + n, g, cfg, s);
  }
  // C[n][k] = sum_b dH[b][n] A1[b][k]: both fragments by transpose reads of the sample
  // rows; one k permutation for both operands (lane half hh, substep st, j ->
  // b = MR/2 hh + 8 st + j), so the product is the plain sum over the batch
  const int g4 = lane >> 4, qq = (lane >> 2) & 3, c16 = 16 * (g4 & 1) + 4 * (lane & 3), hh = g4 >> 1;
  f32x16 acc = {};
#pragma unroll
  for (int st = 0; st < MR / 16; ++st) {
    uint4 a, bq;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int row = (MR / 2) * hh + 8 * st + 4 * t + qq;
      const uint2 ua = __builtin_bit_cast(uint2, __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) s16x4*)(sdh + row * 32 + c16)));
      const uint2 ub = __builtin_bit_cast(uint2, __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) s16x4*)(sa1 + row * AP + wave * 32 + c16)));
      if (t == 0) {
        a.x = ua.x, a.y = ua.y, bq.x = ub.x, bq.y = ub.y;
      } else {
        a.z = ua.x, a.w = ua.y, bq.z = ub.x, bq.w = ub.y;
      }
    }
    acc = mfma32b(a, bq, acc);
  }
  __syncthreads();  // staging dead -> gradient tile
#pragma unroll
  for (int i = 0; i < 16; ++i) gt[acc_row_b(i, h)][wave * 32 + r] = acc[i];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int kl = kq + 32 * j, k = kb + kl;
    if (k >= kFeat) continue;
    const float4 g = *reinterpret_cast<const float4*>(&gt[nl][kl]);
    const int64_t e = int64_t(n0 + nl) * kFeat + k;
    if (gdump) *reinterpret_cast<float4*>(gdump + off.l1w + e) = g;
    adam_regs(pr[j].x, mr[j].x, vr[j].x, g.x, cfg, s);
    adam_regs(pr[j].y, mr[j].y, vr[j].y, g.y, cfg, s);
    adam_regs(pr[j].z, mr[j].z, vr[j].z, g.z, cfg, s);
    adam_regs(pr[j].w, mr[j].w, vr[j].w, g.w, cfg, s);
    *reinterpret_cast<float4*>(pw + e) = pr[j];
    *reinterpret_cast<float4*>(mw + e) = mr[j];
    *reinterpret_cast<float4*>(vw + e) = vr[j];
    const uint16_t b0 = f32_to_bf16(pr[j].x), b1 = f32_to_bf16(pr[j].y), b2 = f32_to_bf16(pr[j].z),
                   b3 = f32_to_bf16(pr[j].w);
    uint2 o;
    o.x = uint32_t(b0) | (uint32_t(b1) << 16);
    o.y = uint32_t(b2) | (uint32_t(b3) << 16);
    *reinterpret_cast<uint2*>(w1bf + e) = o;
    if (!w1tbf) continue;
    tr[kl][nl] = b0;
    tr[kl + 1][nl] = b1;
    tr[kl + 2][nl] = b2;
    tr[kl + 3][nl] = b3;
  }
  if (!w1tbf) return;  // row-major dA1 routing: no W1^T shadow
  __syncthreads();
  for (int j = tid; j < 128 * 4; j += 256) {
    const int kl = j >> 2, q = j & 3;
    const int k = kb + kl;
    if (k < kFeat)
      *reinterpret_cast<uint4*>(w1tbf + size_t(k) * kHid + n0 + q * 8) = *reinterpret_cast<const uint4*>(&tr[kl][q * 8]);
  }
}

template <int MR>
__global__ __launch_bounds__(256) void fc1_wgrad_adam_kernel(const uint16_t* __restrict__ dH, const uint16_t* __restrict__ a1,
                                                             float* __restrict__ p, float* __restrict__ m,
                                                             float* __restrict__ v, float* __restrict__ gdump,
                                                             uint16_t* __restrict__ w1bf, uint16_t* __restrict__ w1tbf,
                                                             Offsets off, const int* __restrict__ adam_t, int t_off,
                                                             AdamCfg cfg) {
  __shared__ __attribute__((aligned(16))) char smem[Fc1Lds<MR>::kBytes];
  fc1_wgrad_adam_body<MR>(blockIdx.x, blockIdx.y, dH, a1, p, m, v, gdump, w1bf, w1tbf, off, adam_t, t_off, cfg, smem);
}

void fc1_wgrad_adam(const uint16_t* dH, const uint16_t* a1, int mrows, float* params, float* m, float* v,
                    float* gdump, uint16_t* w1bf, uint16_t* w1tbf, Offsets off, const int* adam_t, int t_off,
                    AdamCfg cfg, hipStream_t s) {
  const dim3 grid((kFeat + 127) / 128, kHid / 32);
  if (mrows == 32)
    hipLaunchKernelGGL(fc1_wgrad_adam_kernel<32>, grid, dim3(256), 0, s, dH, a1, params, m, v, gdump, w1bf, w1tbf,
                       off, adam_t, t_off, cfg);
  else
    hipLaunchKernelGGL(fc1_wgrad_adam_kernel<64>, grid, dim3(256), 0, s, dH, a1, params, m, v, gdump, w1bf, w1tbf,
                       off, adam_t, t_off, cfg);
}

// ---------------------------------------------------------------------------
// 8+9. conv2 backward: one launch of single-wave blocks with two roles, both
//    consuming the dC2 map.  The longer dgrad waves come first in the grid.
//
//  dgrad role, block j < 7B: (tile = j % 7, image b = j / 7).
//    Phase 1 (MFMA): C[pos][ic] = sum_{tap,oc} dC2pad[pos - tap][oc] W2[oc][ic][tap],
//      K = 25 taps x 64 oc = 100 k-steps.  A: the tile's window of the padded dC2
//      image (<= 8 rows x 18 cols x 64 oc) is transposed from the planar map
//      into HWC in LDS (pairs of channels per 4-B write), so every A fragment is
//      one 16-B LDS read; B: 16-B rows of the (ic, tap, oc) weight copy
//      streamed from L2 one 10-step chunk ahead.
//    Phase 2 (sparse, fp32): pooling routes dP1[pos][ic] to ONE conv1 pixel (its
//      argmax) or nowhere (ReLU-dead), so dW1[ic][tap] += dP1 * Xpad[pixel + tap]
//      is a 25-term gather from the input image in LDS -- no dense dC1 map.
//      Each lane owns one channel and 16 positions; half-waves are combined
//      with one shuffle; the tile's partial goes to its slab row.
//  wgrad role, block j - 7B = (tap t, image pair g): dW2[oc][ic][t] over
//    K = 2 images x 14 rows x 16 cols, 64 oc x 32 ic (two accumulators).  A
//    fragments are 16-B rows of the dC2 map (cols 14/15 are zero), B fragments
//    16-B rows of the kx-shifted P1 copy -- both aligned, streamed from L2
//    with loads one half-image ahead.  Written as one coalesced
//    [tap][oc][ic] slab row per image pair.
// ---------------------------------------------------------------------------
constexpr int kOCP = 72;                      // LDS pixel pitch of the dC2 window (144 B)

P2_DEVICE void conv2_wgrad_role(int t, int g, const uint16_t* __restrict__ dc2m, const uint16_t* __restrict__ p1s,
                                float* __restrict__ wslab, int B) {
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int ky = t / 5, kx = t % 5;
  const int b0 = g * kWgG, nb = min(kWgG, B - b0);
  // half-image chunks: 7 k-steps (rows) each
  auto load = [&](int c, uint4 (&A0)[7], uint4 (&A1)[7], uint4 (&Bv)[7]) {
    const int b = b0 + (c >> 1), row0 = (c & 1) * 7;
    const uint16_t* a = dc2m + (size_t(b) * kC2 + r) * 224 + 8 * h;
    const uint16_t* bb = p1s + ((size_t(b) * 5 + kx) * kC1 + r) * kP1sPlane + ky * 16 + 8 * h;
#pragma unroll
    for (int j = 0; j < 7; ++j) {
      const int ks = row0 + j;
      A0[j] = *reinterpret_cast<const uint4*>(a + ks * 16);
      A1[j] = *reinterpret_cast<const uint4*>(a + 32 * 224 + ks * 16);
      Bv[j] = *reinterpret_cast<const uint4*>(bb + ks * 16);
    }
  };
  f32x16 acc0 = {}, acc1 = {};
  uint4 xa0[7], xa1[7], xb[7], ya0[7], ya1[7], yb[7];
  const int nch = 2 * nb;
  load(0, xa0, xa1, xb);
#pragma unroll
  for (int c = 0; c < 2 * kWgG; c += 2) {
    if (c < nch) {
      if (c + 1 < nch) load(c + 1, ya0, ya1, yb);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < 7; ++j) {
        acc0 = mfma32b(xa0[j], xb[j], acc0);
        acc1 = mfma32b(xa1[j], xb[j], acc1);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if (c + 1 < nch) {
      if (c + 2 < nch) load(c + 2, xa0, xa1, xb);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < 7; ++j) {
        acc0 = mfma32b(ya0[j], yb[j], acc0);
        acc1 = mfma32b(ya1[j], yb[j], acc1);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  float* out = wslab + (size_t(g) * kTaps + t) * kC2 * kC1 + r;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int oc = acc_row_b(i, h);
    out[oc * kC1] = acc0[i];
    out[(oc + 32) * kC1] = acc1[i];
  }
}

// wgrad block (image pair g, column tap kx): the per-wave role above re-reads the
// pair's dC2 rows from L2 once per tap (25 x) -- 336 KB per 4-wave block, so the
// role is bound by what one CU can fetch (~11 B/cycle/CU, MI355X_MICROARCH.md),
// not by its 56 MFMAs per wave.  Here the block stages the pair's dC2 map
// (2 x 28 KB) and its kx-shifted P1 planes (2 x 18 KB) into LDS once, by
// global_load_lds, and wave w computes the row taps ky = w (and wave 0 also
// ky = 4) from LDS: 94 KB fetched per block, 5 x groups blocks.  Same slab
// layout and summation order per tap as the per-wave role.
constexpr int kWgA = kWgG * kC2 * 224 * 2;      // dC2 of the pair: [img][oc][224] bf16
constexpr int kWgB = kWgG * kC1 * kP1sPlane * 2;  // P1 planes at kx: [img][ic][18 x 16] bf16
static_assert(kWgA + kWgB <= 143424, "wgrad staging must fit the launch's LDS");

P2_DEVICE void glds_copy(const uint16_t* src, char* dst, int bytes, int wave, int lane) {
  // 1 KB per wave instruction (64 lanes x 16 B), lane-linear LDS image
  for (int c = wave; c * 1024 < bytes; c += 4)
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + c * 512 + lane * 8),
                                     (__attribute__((address_space(3))) void*)(dst + c * 1024), 16, 0, 0);
}

// Row-swizzled variant for images of CPR 16-byte chunks per row: LDS chunk j of
// row rho holds source chunk j ^ wg_swz(rho).  The wgrad blocks read 16 B per lane
// from 32 consecutive rows at one column; with rows of 448 B (dC2, 28 chunks) or
// 576 B (P1 planes, 36 chunks) rows r and r + 4 hit the same 16-byte bank slot, a
// 4-way conflict on every ds_read_b128 (profiles/r4_cnn_pmc.md: 58 % of the
// kernel's LDS cycles).  XOR-ing the low two chunk bits with (row >> 2) & 3 spreads
// every 16-lane read group over all 16 slots.  The destination stays lane-linear
// (LDS-DMA), the permutation is applied to the source address (CPR % 4 == 0 keeps
// it inside the row).
P2_DEVICE int wg_swz(int row) { return (row >> 2) & 3; }

template <int CPR>
P2_DEVICE void glds_copy_swz(const uint16_t* src, char* dst, int bytes, int wave, int lane) {
  static_assert(CPR % 4 == 0, "the swizzle permutes chunk groups of 4 inside a row");
  for (int c = wave; c * 1024 < bytes; c += 4) {
    const int q = c * 64 + lane, rho = q / CPR, j = q - rho * CPR;
    const int sq = rho * CPR + (j ^ wg_swz(rho));
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + sq * 8),
                                     (__attribute__((address_space(3))) void*)(dst + c * 1024), 16, 0, 0);
  }
}

P2_DEVICE void conv2_wgrad_block(int g, int kx, const uint16_t* __restrict__ dc2m, const uint16_t* __restrict__ p1s,
                                 float* __restrict__ wslab, int B, char* smem) {
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const int b0 = g * kWgG, nb = min(kWgG, B - b0);
  const uint16_t* sa = reinterpret_cast<const uint16_t*>(smem);
  const uint16_t* sb = reinterpret_cast<const uint16_t*>(smem + kWgA);
  // the pair's images are consecutive in the dC2 map; the P1 planes of one kx
  // are one contiguous [ic][plane] block per image
  static_assert(224 % 32 == 0 && kP1sPlane % 32 == 0, "whole 16-B chunk groups per row");
  glds_copy_swz<224 / 8>(dc2m + size_t(b0) * kC2 * 224, smem, nb * kC2 * 224 * 2, wave, lane);
  for (int i = 0; i < nb; ++i)
    glds_copy_swz<kP1sPlane / 8>(p1s + (size_t(b0 + i) * 5 + kx) * kC1 * kP1sPlane,
                                 smem + kWgA + i * (kC1 * kP1sPlane * 2), kC1 * kP1sPlane * 2, wave, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // rows i * kC2 + r (+ 32) and i * kC1 + r all have wg_swz == wg_swz(r)
  const int t = h ^ wg_swz(r);
  for (int ky = wave; ky < 5; ky += 4) {
    f32x16 acc0 = {}, acc1 = {};
    for (int i = 0; i < nb; ++i) {
      const uint16_t* a = sa + (i * kC2 + r) * 224;
      const uint16_t* bb = sb + (i * kC1 + r) * kP1sPlane;
#pragma unroll
      for (int ks = 0; ks < 14; ++ks) {
        // chunk 2 ks + h of the row, and chunk 2 (ky + ks) + h of the P1 plane, swizzled
        const int ca = (2 * ks) ^ t, cb = (2 * (ky + ks)) ^ t;
        const uint4 a0 = *reinterpret_cast<const uint4*>(a + 8 * ca);
        const uint4 a1 = *reinterpret_cast<const uint4*>(a + 32 * 224 + 8 * ca);
        const uint4 bq = *reinterpret_cast<const uint4*>(bb + 8 * cb);
        acc0 = mfma32b(a0, bq, acc0);
        acc1 = mfma32b(a1, bq, acc1);
      }
    }
    float* out = wslab + (size_t(g) * kTaps + ky * 5 + kx) * kC2 * kC1 + r;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int oc = acc_row_b(i, h);
      out[oc * kC1] = acc0[i];
      out[(oc + 32) * kC1] = acc1[i];
    }
  }
}

// dgrad block: 4 waves = 4 consecutive 32-position tiles of one image
// (group 0: tiles 0-3 = conv rows 0..9, group 1: tiles 4-6 = rows 9..13; the
// 4th wave of group 1 only helps staging).  The block stages, in one memory
// round trip, the whole W2q weight copy (32 ic rows x 25 taps x 64 oc, padded
// rows) and the group's zero-padded HWC window of the dC2 map into LDS, so
// every MFMA operand of the 100 k-steps is a 16-B LDS read.
constexpr int kW2qRow = kTaps * kC2 + 8;                 // 1608 elements per ic row (pad breaks bank aliasing)
constexpr int kDgW = kC1 * kW2qRow * 2;                  // 102912 B
constexpr int kDgWinRows = 14;                           // padded rows of a group's window
constexpr int kDgWin = kDgWinRows * 18 * kOCP * 2;       // 36288 B
constexpr int kDgXs = 32 * 33 * 4;                       // 4224 B
constexpr int kDgLds = kDgW + kDgWin + kDgXs;            // 143424 B (one dgrad block per CU)

// STREAM_W: the weight fragments come straight from L2 (16-B loads one 10-step chunk
// ahead of the MFMAs) instead of the 102 KB LDS copy every block stages before its
// first MFMA.  Measured slower (18.8 vs 12.6 us): off by default.
template <bool STREAM_W>
P2_DEVICE void conv2_dgrad_block(int grp, int b, const uint16_t* __restrict__ dc2m, const uint8_t* __restrict__ am1,
                                 const uint16_t* __restrict__ w2q, const uint8_t* __restrict__ xds,
                                 const int64_t* __restrict__ idx, float* __restrict__ wslab1, char* smem) {
  uint16_t* sw = reinterpret_cast<uint16_t*>(smem);
  uint16_t* win = reinterpret_cast<uint16_t*>(smem + kDgW);
  float(*xs)[33] = reinterpret_cast<float(*)[33]>(smem + kDgW + kDgWin);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const int tile = grp * 4 + wave;
  const bool active = tile < kDgTiles;
  const int ylo = grp ? (4 * 32) / 14 : 0;  // first padded window row of the group
  const int m = tile * 32 + r, mc = m < 196 ? m : 195;
  const int y = mc / 14, x = mc % 14;
  // ---- issue every load.  W2q goes global -> LDS directly (no VGPRs): each
  // ic row (1600 elements = 3200 B) is 4 wave instructions of 50 lanes x 16 B,
  // so no instruction crosses the 16-B row padding; 32 instructions per wave.
  if (!STREAM_W) {
#pragma unroll 4
    for (int k = 0; k < 32; ++k) {
      const int id = wave * 32 + k, ic = id >> 2, q = id & 3;
      if (lane < 50)
        __builtin_amdgcn_global_load_lds(
            (const __attribute__((address_space(1))) void*)(w2q + ic * (kTaps * kC2) + q * 400 + lane * 8),
            (__attribute__((address_space(3))) void*)(sw + ic * kW2qRow + q * 400), 16, 0, 0);
    }
  }
  // the window (4 items of two channels x 8 columns), this lane's pool1
  // argmax codes and the image go through registers
  uint4 wu0[4], wu1[4];
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int i = tid + 256 * it;  // 14 rows x 32 channel pairs x 2 chunks = 896 items
    const int wr = i >> 6, pr = (i >> 1) & 31, c = i & 1, yd = ylo + wr - 2;
    const int ydc = yd < 0 ? 0 : (yd > 13 ? 13 : yd);
    const uint16_t* src = dc2m + (size_t(b) * kC2 + 2 * pr) * 224 + ydc * 16 + c * 8;
    wu0[it] = *reinterpret_cast<const uint4*>(src);
    wu1[it] = *reinterpret_cast<const uint4*>(src + 224);
  }
  uint8_t acode[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int pos = tile * 32 + acc_row_b(i, h);
    acode[i] = (active && pos < 196) ? am1[(size_t(b) * 196 + pos) * kC1 + r] : uint8_t(4);
  }
  const int64_t row = idx ? idx[b] : b;
  const uint8_t* xsrc = xds + row * (kImg * kImg);
  const uint4 z4 = make_uint4(0, 0, 0, 0);
  for (int i = tid; i < kDgWin / 16; i += 256) reinterpret_cast<uint4*>(win)[i] = z4;
  for (int i = tid; i < 32 * 32; i += 256) {
    const int yy = i >> 5, xx = i & 31, sy = yy - 2, sx = xx - 2;
    float v = 0.f;
    if (sy >= 0 && sy < kImg && sx >= 0 && sx < kImg) v = float(xsrc[sy * kImg + sx]) * (1.f / 255.f);
    xs[yy][xx] = v;
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int i = tid + 256 * it;
    const int wr = i >> 6, pr = (i >> 1) & 31, c = i & 1, yd = ylo + wr - 2;
    if (i >= kDgWinRows * 64 || yd < 0 || yd > 13) continue;
    const uint16_t* e0 = reinterpret_cast<const uint16_t*>(&wu0[it]);
    const uint16_t* e1 = reinterpret_cast<const uint16_t*>(&wu1[it]);
    uint16_t* dst = win + (wr * 18 + c * 8 + 2) * kOCP + 2 * pr;
#pragma unroll
    for (int j = 0; j < 8; ++j) *reinterpret_cast<uint32_t*>(dst + j * kOCP) = uint32_t(e0[j]) | (uint32_t(e1[j]) << 16);
  }
  __syncthreads();
  if (!active) return;
  // ---- phase 1: C[pos][ic], 100 k-steps, both operands from LDS
  const uint16_t* abase = win + ((y - ylo) * 18 + x) * kOCP + 8 * h;
  f32x16 acc = {};
  if (STREAM_W) {
    // B fragment of k-step s: 16 B of ic row r at element 16 s + 8 h (row-major
    // [ic][tap][oc] = element t * 64 + oc0); 10 steps per chunk, one chunk ahead
    const uint16_t* brow = w2q + r * (kTaps * kC2) + 8 * h;
    uint4 bx[10], by[10];
#pragma unroll
    for (int j = 0; j < 10; ++j) bx[j] = *reinterpret_cast<const uint4*>(brow + 16 * j);
#pragma unroll
    for (int c = 0; c < 10; c += 2) {
      if (c + 1 < 10) {
#pragma unroll
        for (int j = 0; j < 10; ++j) by[j] = *reinterpret_cast<const uint4*>(brow + 16 * ((c + 1) * 10 + j));
      }
#pragma unroll
      for (int j = 0; j < 10; ++j) {
        const int s2 = c * 10 + j, t = s2 >> 2, ky = t / 5, kx = t % 5, oc0 = (s2 & 3) * 16;
        const uint4 a = *reinterpret_cast<const uint4*>(abase + ((4 - ky) * 18 + (4 - kx)) * kOCP + oc0);
        acc = mfma32b(a, bx[j], acc);
      }
      if (c + 2 < 10) {
#pragma unroll
        for (int j = 0; j < 10; ++j) bx[j] = *reinterpret_cast<const uint4*>(brow + 16 * ((c + 2) * 10 + j));
      }
#pragma unroll
      for (int j = 0; j < 10; ++j) {
        const int s2 = (c + 1) * 10 + j, t = s2 >> 2, ky = t / 5, kx = t % 5, oc0 = (s2 & 3) * 16;
        const uint4 a = *reinterpret_cast<const uint4*>(abase + ((4 - ky) * 18 + (4 - kx)) * kOCP + oc0);
        acc = mfma32b(a, by[j], acc);
      }
    }
  } else {
    const uint16_t* bbase = sw + r * kW2qRow + 8 * h;
#pragma unroll 4
    for (int s = 0; s < 100; ++s) {
      const int t = s >> 2, ky = t / 5, kx = t % 5, oc0 = (s & 3) * 16;
      const uint4 a = *reinterpret_cast<const uint4*>(abase + ((4 - ky) * 18 + (4 - kx)) * kOCP + oc0);
      const uint4 bq = *reinterpret_cast<const uint4*>(bbase + t * kC2 + oc0);
      acc = mfma32b(a, bq, acc);
    }
  }
  // ---- phase 2: sparse conv1 weight gradient at each pool1 argmax pixel
  float wg[kTaps];
#pragma unroll
  for (int t = 0; t < kTaps; ++t) wg[t] = 0.f;
  float bs = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int pos = tile * 32 + acc_row_b(i, h);
    const uint8_t a = acode[i];
    if (pos < 196 && a < 4) {
      const int yy = 2 * (pos / 14) + (a >> 1), xx = 2 * (pos % 14) + (a & 1);
      const float gv = acc[i];
      bs += gv;
#pragma unroll
      for (int ky = 0; ky < 5; ++ky)
#pragma unroll
        for (int kx = 0; kx < 5; ++kx) wg[ky * 5 + kx] = fmaf(gv, xs[yy + ky][xx + kx], wg[ky * 5 + kx]);
    }
  }
#pragma unroll
  for (int t = 0; t < kTaps; ++t) wg[t] += __shfl_xor(wg[t], 32, 64);
  bs += __shfl_xor(bs, 32, 64);
  if (h == 0) {
    float* o = wslab1 + (size_t(b) * kDgTiles + tile) * kSlab1;
#pragma unroll
    for (int t = 0; t < kTaps; ++t) o[r * kTaps + t] = wg[t];
    o[kC1 * kTaps + r] = bs;
  }
}

// 256-thread blocks: [0, 2B) dgrad blocks (image b = j / 2, group j % 2),
// then wgrad blocks of 4 independent (tap, image pair) waves.
__global__ __launch_bounds__(256) void conv2_bwd_kernel(const uint16_t* __restrict__ dc2m,
                                                        const uint16_t* __restrict__ p1s,
                                                        const uint8_t* __restrict__ am1,
                                                        const uint16_t* __restrict__ w2q,
                                                        const uint8_t* __restrict__ xds,
                                                        const int64_t* __restrict__ idx, float* __restrict__ wslab1,
                                                        float* __restrict__ wslab2, int B, int first_block,
                                                        int wg_blocks, int stream_w, int wg_first) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nd = 2 * B;
  // wg_first: the wgrad blocks take the low block ids (dispatched first)
  int j = blockIdx.x + first_block;
  if (wg_first) j = j < int(gridDim.x) - nd ? j + nd : j - (int(gridDim.x) - nd);
  if (j < nd) {
    if (stream_w)
      conv2_dgrad_block<true>(j & 1, j >> 1, dc2m, am1, w2q, xds, idx, wslab1, smem);
    else
      conv2_dgrad_block<false>(j & 1, j >> 1, dc2m, am1, w2q, xds, idx, wslab1, smem);
  } else if (wg_blocks) {
    const int k = j - nd;  // (image pair, kx)
    conv2_wgrad_block(k / 5, k % 5, dc2m, p1s, wslab2, B, smem);
  } else {
    const int k = (j - nd) * 4 + (threadIdx.x >> 6);
    if (k < kTaps * wgrad_groups(B)) conv2_wgrad_role(k % kTaps, k / kTaps, dc2m, p1s, wslab2, B);
  }
}

void conv2_bwd(const uint16_t* dc2m, const uint16_t* p1s, const uint8_t* am1, const uint16_t* w2q, const uint8_t* x,
               const int64_t* idx, float* wslab1, float* wslab2, int B, hipStream_t s) {
  // P2CNN_CONV2BWD_ROLES (measurement knob, read once): 1 = dgrad blocks
  // only, 2 = wgrad blocks only; unset = both (the product).  Measured
  // (scripts/kbench.py, B = 32): dgrad 7.3 us, wgrad 13.1 us, both 12.5 us.
  // One-image wgrad waves (kWgG = 1) cut the wgrad role to 5.7 us, but its 200
  // blocks plus the 64 dgrad blocks no longer fit one block per CU (the
  // launch's 143 KB LDS), and neither spare dgrad waves nor 8-wave blocks
  // (1 image per dgrad block) beat 13.9 us inside the step's HIP graph.
  static const int roles = [] {
    const char* e = getenv("P2CNN_CONV2BWD_ROLES");
    return e ? atoi(e) : 3;
  }();
  // wgrad as LDS-staged (image pair, kx) blocks (default) or as the per-wave
  // (tap, image pair) role streaming from L2 (P2CNN_CONV2_WG_BLOCKS=0)
  static const int wg_blocks = [] {
    const char* e = getenv("P2CNN_CONV2_WG_BLOCKS");
    return e ? atoi(e) : 1;
  }();
  // dgrad weight fragments staged in LDS (default) or streamed from L2
  // (P2CNN_DGRAD_STREAM_W=1: measured slower, 18.8 vs 12.6 us for the dgrad role,
  // scripts/kbench.py round 4 -- the four waves re-fetch every fragment)
  static const int stream_w = [] {
    const char* e = getenv("P2CNN_DGRAD_STREAM_W");
    return e ? atoi(e) : 0;
  }();
  // P2CNN_CONV2BWD_WG_FIRST=1 (measurement knob): wgrad blocks before the dgrad blocks
  static const int wg_first = [] {
    const char* e = getenv("P2CNN_CONV2BWD_WG_FIRST");
    return e ? atoi(e) : 0;
  }();
  const int nd = 2 * B, nw = wg_blocks ? 5 * wgrad_groups(B) : (kTaps * wgrad_groups(B) + 3) / 4;
  const int first = roles == 2 ? nd : 0;
  const int blocks = roles == 1 ? nd : roles == 2 ? nw : nd + nw;
  hipLaunchKernelGGL(conv2_bwd_kernel, dim3(blocks), dim3(256), kDgLds, s, dc2m, p1s, am1, w2q, x, idx, wslab1, wslab2,
                     B, first, wg_blocks, stream_w, roles == 3 ? wg_first : 0);
}

// ---------------------------------------------------------------------------
// 10. Conv parameters: fixed-order reduction of the gradient partials, Adam,
//     and the conv2 bf16 shadows (W2r for the forward, W2q for the dgrad).
//     Blocks 0..63: one conv2 output channel each -- its 800 weights are
//     summed over the image-pair slabs ([tap][oc][ic] rows, coalesced),
//     transposed through LDS into parameter order, and its bias gradient is
//     the block sum of the alive-masked dA1 terms (gB).  Blocks 64..115: 16
//     conv1 parameters each, the 7B tile partials split 16 ways.  Every load
//     loop is batched so a thread keeps 8-16 independent loads in flight.
// ---------------------------------------------------------------------------
constexpr int kC1Blocks = kSlab1 / 16;  // 52

constexpr int kConvAdamLds = (kTaps * (kC1 + 1) + 256) * 4;

// Stores of the values the next step's forward reads inside the same launch
// (fc1_conv_adam_fwd_kernel: conv weights / biases and the W2r shadow) go
// write-through with WT (device-coherent sc1 stores, as cnn_fwd_dev.h reads them).
template <bool WT>
P2_DEVICE void st_p(float* p, float v) {
  if constexpr (WT)
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else
    *p = v;
}
template <bool WT>
P2_DEVICE void st_h(uint16_t* p, uint16_t v) {
  if constexpr (WT)
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else
    *p = v;
}

template <bool WT = false>
P2_DEVICE void conv_adam_body(int blk, const float* __restrict__ ws1, const float* __restrict__ ws2,
                              const float* __restrict__ gb, int B, float* __restrict__ p, float* __restrict__ m,
                              float* __restrict__ v, float* __restrict__ gdump, uint16_t* __restrict__ w2r,
                              uint16_t* __restrict__ w2q, const Offsets& off, const int* __restrict__ adam_t, int t_off,
                              const AdamCfg& cfg, char* smem) {
  float(*g2)[kC1 + 1] = reinterpret_cast<float(*)[kC1 + 1]>(smem);
  float* red = reinterpret_cast<float*>(smem + kTaps * (kC1 + 1) * 4);
  const int tid = threadIdx.x;
  const AdamScal sc = adam_scal(cfg, adam_t, t_off);
  if (blk < kC2) {
    const int oc = blk, ng = wgrad_groups(B);
    // Adam state of this thread's (up to 4) weights and the bias: loaded first,
    // independent of the reductions below
    float pr[4], mr[4], vr[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int j = tid + 256 * u;
      const int64_t e = off.c2w + int64_t(oc) * kC1 * kTaps + (j < kC1 * kTaps ? j : 0);
      pr[u] = p[e];
      mr[u] = m[e];
      vr[u] = v[e];
    }
    float pb = 0.f, mb = 0.f, vb = 0.f;
    if (tid == 0) {
      pb = p[off.c2b + oc];
      mb = m[off.c2b + oc];
      vb = v[off.c2b + oc];
    }
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int g0 = 0; g0 < ng; g0 += 8) {
      float t[4][8];
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int j = tid + 256 * u, t_ = j >> 5, ic = j & 31, gg = g0 + k;
          t[u][k] = (j < kTaps * kC1 && gg < ng) ? ws2[((size_t(gg) * kTaps + t_) * kC2 + oc) * kC1 + ic] : 0.f;
        }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[u] += t[u][k];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int j = tid + 256 * u;
      if (j < kTaps * kC1) g2[j >> 5][j & 31] = acc[u];
    }
    float bs = 0.f;
    for (int e0 = 0; e0 < B * 49; e0 += 256 * 8) {
      float t[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int e = e0 + tid + 256 * u;
        t[u] = e < B * 49 ? gb[size_t(e / 49) * kFeat + oc * 49 + e % 49] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) bs += t[u];
    }
    red[tid] = bs;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
      if (tid < w) red[tid] += red[tid + w];
      __syncthreads();
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int j = tid + 256 * u;
      if (j >= kC1 * kTaps) break;
      const int ic = j / kTaps, t = j % kTaps;
      const float g = g2[t][ic];
      const int64_t e = off.c2w + int64_t(oc) * kC1 * kTaps + j;
      if (gdump) gdump[e] = g;
      adam_regs(pr[u], mr[u], vr[u], g, cfg, sc);
      st_p<WT>(p + e, pr[u]);
      m[e] = mr[u];
      v[e] = vr[u];
      const uint16_t hb = f32_to_bf16(pr[u]);
      st_h<WT>(w2r + (oc * kTaps + t) * kC1 + ic, hb);
      w2q[(ic * kTaps + t) * kC2 + oc] = hb;
    }
    if (tid == 0) {
      if (gdump) gdump[off.c2b + oc] = red[0];
      adam_regs(pb, mb, vb, red[0], cfg, sc);
      st_p<WT>(p + off.c2b + oc, pb);
      m[off.c2b + oc] = mb;
      v[off.c2b + oc] = vb;
    }
  } else {
    const int j = (blk - kC2) * 16 + (tid & 15), q = tid >> 4;  // 16 row splits
    const int rows = B * kDgTiles;
    const int64_t e = j < kC1 * kTaps ? off.c1w + j : off.c1b + (j - kC1 * kTaps);
    float pe = 0.f, me = 0.f, ve = 0.f;
    if (q == 0) {
      pe = p[e];
      me = m[e];
      ve = v[e];
    }
    float s = 0.f;
    for (int r0 = q; r0 < rows; r0 += 16 * 8) {
      float t[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int rw = r0 + 16 * u;
        t[u] = rw < rows ? ws1[size_t(rw) * kSlab1 + j] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) s += t[u];
    }
    red[tid] = s;
    __syncthreads();
    if (q == 0) {
      float g = 0.f;
#pragma unroll
      for (int k = 0; k < 16; ++k) g += red[k * 16 + tid];
      if (gdump) gdump[e] = g;
      adam_regs(pe, me, ve, g, cfg, sc);
      st_p<WT>(p + e, pe);
      m[e] = me;
      v[e] = ve;
    }
  }
}

__global__ __launch_bounds__(256) void conv_adam_kernel(const float* __restrict__ ws1, const float* __restrict__ ws2,
                                                        const float* __restrict__ gb, int B, float* __restrict__ p,
                                                        float* __restrict__ m, float* __restrict__ v,
                                                        float* __restrict__ gdump, uint16_t* __restrict__ w2r,
                                                        uint16_t* __restrict__ w2q, Offsets off,
                                                        const int* __restrict__ adam_t, int t_off, AdamCfg cfg) {
  __shared__ __attribute__((aligned(16))) char smem[kConvAdamLds];
  conv_adam_body(blockIdx.x, ws1, ws2, gb, B, p, m, v, gdump, w2r, w2q, off, adam_t, t_off, cfg, smem);
}

// ---------------------------------------------------------------------------
// 7+10 in one launch (after conv2_bwd): optionally the 81 FC2 Adam blocks,
// then the 116 conv-parameter blocks, then the 1600 FC1 weight-gradient + Adam
// blocks.  The FC1 part streams the 6.4M-parameter Adam state (HBM-bound, ~28
// B per parameter); the FC2 and conv parts are latency-bound reductions --
// sharing the launch hides them behind the stream instead of paying a kernel
// boundary and their tails.  (The FC2 role used to share route_fc2's launch:
// there the two roles did not overlap -- 11.8 us together vs 6.7 us for the
// dA1 blocks alone and 7.4 us for the FC2 blocks alone, scripts/kbench.py.)
// ---------------------------------------------------------------------------
constexpr int kFc2Blocks256 = (kCls * kHid + kCls + 255) / 256;  // 81

template <int MR>
__global__ __launch_bounds__(256) void fc1_conv_adam_kernel(
    const uint16_t* __restrict__ dH, const uint16_t* __restrict__ a1, const float* __restrict__ ws1,
    const float* __restrict__ ws2, const float* __restrict__ gb, int B, float* __restrict__ p, float* __restrict__ m,
    float* __restrict__ v, float* __restrict__ gdump, uint16_t* __restrict__ w1bf, uint16_t* __restrict__ w1tbf,
    uint16_t* __restrict__ w2r, uint16_t* __restrict__ w2q, Offsets off, const int* __restrict__ adam_t, int t_off,
    AdamCfg cfg, const float* __restrict__ dlogits, const uint16_t* __restrict__ H, int nf2,
    uint16_t* __restrict__ w2bf) {
  constexpr int kLds = Fc1Lds<MR>::kBytes > kConvAdamLds ? Fc1Lds<MR>::kBytes : kConvAdamLds;
  __shared__ __attribute__((aligned(16))) char smem[kLds];
  constexpr int kCA = kC2 + kC1Blocks, kBx = (kFeat + 127) / 128;
  int j = blockIdx.x;
  if (j < nf2) {
    fc2_role<256>(j, dlogits, H, B, p, m, v, gdump, off, adam_t, t_off, cfg, w2bf);
    return;
  }
  j -= nf2;
  if (j < kCA) {
    conv_adam_body(j, ws1, ws2, gb, B, p, m, v, gdump, w2r, w2q, off, adam_t, t_off, cfg, smem);
    return;
  }
  const int f = j - kCA;
  fc1_wgrad_adam_body<MR>(f % kBx, f / kBx, dH, a1, p, m, v, gdump, w1bf, w1tbf, off, adam_t, t_off, cfg, smem);
}

void fc1_conv_adam(const uint16_t* dH, const uint16_t* a1, int mrows, const float* wslab1, const float* wslab2,
                   const float* gb, int B, float* params, float* m, float* v, float* gdump, uint16_t* w1bf,
                   uint16_t* w1tbf, uint16_t* w2r, uint16_t* w2q, Offsets off, const int* adam_t, int t_off,
                   AdamCfg cfg, const float* dlogits, const uint16_t* H, uint16_t* w2bf, hipStream_t s) {
  const int nf2 = dlogits ? kFc2Blocks256 : 0;
  const dim3 grid(nf2 + kC2 + kC1Blocks + ((kFeat + 127) / 128) * (kHid / 32));
  if (mrows == 32)
    hipLaunchKernelGGL(fc1_conv_adam_kernel<32>, grid, dim3(256), 0, s, dH, a1, wslab1, wslab2, gb, B, params, m, v,
                       gdump, w1bf, w1tbf, w2r, w2q, off, adam_t, t_off, cfg, dlogits, H, nf2, w2bf);
  else
    hipLaunchKernelGGL(fc1_conv_adam_kernel<64>, grid, dim3(256), 0, s, dH, a1, wslab1, wslab2, gb, B, params, m, v,
                       gdump, w1bf, w1tbf, w2r, w2q, off, adam_t, t_off, cfg, dlogits, H, nf2, w2bf);
}

// ---------------------------------------------------------------------------
// fc1_conv_adam + the NEXT step's conv1 and conv2 in one launch.  The FC1 Adam
// stream is HBM-bound (~28 us); conv1 + conv2 of the next step are latency-bound
// (~4.6 + 6.0 us as their own launches) and only need the conv parameters this
// launch's conv-Adam workgroups produce -- so they run beside the stream instead
// of after it.  Workgroup roles in id order: FC2 Adam, conv-parameter Adam (WT
// stores, then a ticket on sync[0]), the FC1 wgrad + Adam stream, conv1 of (row
// pair, image) (waits for every conv-Adam ticket; WT P1 stores, ticket on
// sync[1]), conv2 (4 (row, oc half, image) items per workgroup; waits for every
// conv1 ticket; the last one to finish resets sync[0..2]).  The convolution
// workgroups come last so they take CU slots as the stream's first workgroups
// retire: placed ahead of the stream, their waits held the slots it needed
// (72 us for the launch vs 28.8 + 4.6 + 6.0 us for the three kernels).  A waiting role
// only waits for roles with lower workgroup ids, which the dispatcher starts
// first and which wait for nothing later, so the launch always drains; the wait
// is bounded anyway (sync[3] records a timeout).  Same arithmetic as the
// separate launches: the parameters and activations are bitwise equal.
// ---------------------------------------------------------------------------
P2_DEVICE void wait_tickets(int* ctr, int target, int* stall) {
  if (threadIdx.x == 0) {
    int it = 0;
    while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      if (++it > (1 << 22)) {
        __hip_atomic_store(stall, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
}
// after this workgroup's write-through stores: drain them, then one ticket
P2_DEVICE void put_ticket(int* ctr) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int MR>
__global__ __launch_bounds__(256) void fc1_conv_adam_fwd_kernel(
    const uint16_t* __restrict__ dH, const uint16_t* __restrict__ a1, const float* __restrict__ ws1,
    const float* __restrict__ ws2, const float* __restrict__ gb, int B, float* __restrict__ p, float* __restrict__ m,
    float* __restrict__ v, float* __restrict__ gdump, uint16_t* __restrict__ w1bf, uint16_t* __restrict__ w1tbf,
    uint16_t* __restrict__ w2r, uint16_t* __restrict__ w2q, Offsets off, const int* __restrict__ adam_t, int t_off,
    AdamCfg cfg, const float* __restrict__ dlogits, const uint16_t* __restrict__ H, int nf2,
    uint16_t* __restrict__ w2bf, FwdNext f) {
  constexpr int kA = Fc1Lds<MR>::kBytes > kConvAdamLds ? Fc1Lds<MR>::kBytes : kConvAdamLds;
  constexpr int kB = int(sizeof(Conv1Smem)) > 4 * 32 * 33 * 4 ? int(sizeof(Conv1Smem)) : 4 * 32 * 33 * 4;
  __shared__ __attribute__((aligned(16))) char smem[kA > kB ? kA : kB];
  constexpr int kCA = kC2 + kC1Blocks, kBx = (kFeat + 127) / 128;
  const int n1 = 7 * f.B, n2 = (14 * f.B + 3) / 4;
  int j = blockIdx.x;
  if (j < nf2) {
    fc2_role<256>(j, dlogits, H, B, p, m, v, gdump, off, adam_t, t_off, cfg, w2bf);
    return;
  }
  j -= nf2;
  if (j < kCA) {
    conv_adam_body<true>(j, ws1, ws2, gb, B, p, m, v, gdump, w2r, w2q, off, adam_t, t_off, cfg, smem);
    put_ticket(f.sync);
    return;
  }
  j -= kCA;
  constexpr int nfc1 = kBx * (kHid / 32);
  if (j < nfc1) {
    fc1_wgrad_adam_body<MR>(j % kBx, j / kBx, dH, a1, p, m, v, gdump, w1bf, w1tbf, off, adam_t, t_off, cfg, smem);
    return;
  }
  j -= nfc1;
  if (j < n1) {
    wait_tickets(f.sync, kCA, f.sync + 3);
    conv1_body<true>(j % 7, j / 7, f.x, f.idx, p + off.c1w, p + off.c1b, f.p1, f.am1, f.p1s,
                     *reinterpret_cast<Conv1Smem*>(smem));
    put_ticket(f.sync + 1);
    return;
  }
  j -= n1;
  if (j < n2) {
    wait_tickets(f.sync + 1, n1, f.sync + 3);
    const int wave = threadIdx.x >> 6, item = j * 4 + wave;  // item = (image, oc half, pooled row)
    float(*sout)[33] = reinterpret_cast<float(*)[33]>(smem + wave * (32 * 33 * 4));
    conv2_body<true>(item < 14 * f.B, item % 7, (item / 7) & 1, item / 14, threadIdx.x & 63, f.p1, w2r, p + off.c2b,
                     f.a1, f.am2, sout);
    __syncthreads();
    if (threadIdx.x == 0 &&
        __hip_atomic_fetch_add(f.sync + 2, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == n2 - 1) {
      // every conv1 / conv2 workgroup is past its wait: the counters are free for the next launch
      __hip_atomic_store(f.sync, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(f.sync + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(f.sync + 2, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

void fc1_conv_adam_fwd(const uint16_t* dH, const uint16_t* a1, int mrows, const float* wslab1, const float* wslab2,
                       const float* gb, int B, float* params, float* m, float* v, float* gdump, uint16_t* w1bf,
                       uint16_t* w1tbf, uint16_t* w2r, uint16_t* w2q, Offsets off, const int* adam_t, int t_off,
                       AdamCfg cfg, const float* dlogits, const uint16_t* H, uint16_t* w2bf, const FwdNext& f,
                       hipStream_t s) {
  const int nf2 = dlogits ? kFc2Blocks256 : 0;
  const int n1 = 7 * f.B, n2 = (14 * f.B + 3) / 4;
  const dim3 grid(nf2 + kC2 + kC1Blocks + n1 + n2 + ((kFeat + 127) / 128) * (kHid / 32));
  if (mrows == 32)
    hipLaunchKernelGGL(fc1_conv_adam_fwd_kernel<32>, grid, dim3(256), 0, s, dH, a1, wslab1, wslab2, gb, B, params, m,
                       v, gdump, w1bf, w1tbf, w2r, w2q, off, adam_t, t_off, cfg, dlogits, H, nf2, w2bf, f);
  else
    hipLaunchKernelGGL(fc1_conv_adam_fwd_kernel<64>, grid, dim3(256), 0, s, dH, a1, wslab1, wslab2, gb, B, params, m,
                       v, gdump, w1bf, w1tbf, w2r, w2q, off, adam_t, t_off, cfg, dlogits, H, nf2, w2bf, f);
}

void conv_adam(const float* wslab1, const float* wslab2, const float* gb, int B, float* params, float* m, float* v,
               float* gdump, uint16_t* w2r, uint16_t* w2q, Offsets off, const int* adam_t, int t_off, AdamCfg cfg,
               hipStream_t s) {
  hipLaunchKernelGGL(conv_adam_kernel, dim3(kC2 + kC1Blocks), dim3(256), 0, s, wslab1, wslab2, gb, B, params, m, v,
                     gdump, w2r, w2q, off, adam_t, t_off, cfg);
}

void init_fwd_attributes();

// Raise the dynamic-LDS limit of the kernels that stage > 64 KB.  Called once
// (from the bindings) before any HIP-graph capture.
void init_attributes() {
  init_fwd_attributes();
  P2_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(conv2_bwd_kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, kDgLds));
  P2_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(route_rm_kernel<1, 1>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, kRouteRmLds));
  P2_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(route_rm_kernel<2, 1>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, kRouteRmLds));
  P2_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(route_rm_kernel<1, 2>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, kRouteRmLds / 2));
  P2_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(route_rm_kernel<2, 2>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, kRouteRmLds / 2));
}

}  // namespace p2cnn
