// Host-side launch API of the fused attention kernels (attention.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace p2attn {

constexpr int kMaxT = 256;     // tokens (keys staged whole in LDS)
constexpr int kHeadDim = 64;

struct AttnShape {
  int B, H, T, C;               // C = H * 64
  int64_t qkv_row, qkv_batch;   // element strides of the [B, T, 3, H, 64] QKV tensor (and its gradient)
  int64_t o_row, o_batch;       // element strides of O / dO [B, T, H, 64]
  float scale;                  // softmax scale (1 / sqrt(64))
};

// o = softmax(scale * q k^T) v per (batch, head); lse2 [B, H, T] (log2 domain) saved for the backward.
void attention_fwd(const uint16_t* qkv, uint16_t* o, float* lse2, const AttnShape& sh, hipStream_t s);
// dqkv [B, T, 3, H, 64] (fully written) from dout = dL/do.
void attention_bwd(const uint16_t* qkv, const uint16_t* o, const uint16_t* dout, const float* lse2, uint16_t* dqkv,
                   const AttnShape& sh, hipStream_t s);

}  // namespace p2attn
