// Fused transformer / classifier ops (fused_ops.hip).  bf16 selects uint16
// bf16 activations, else fp32; parameters, statistics and partials are fp32.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace p2fused {

constexpr int kMaxLnCols = 2048;  // row kept in registers (C % 8 == 0)

// residual (optional, nullptr = none): y = LN(x + residual), sum = x + residual (rounded to the activation dtype)
void layer_norm_fwd(bool bf16, const void* x, const void* residual, const float* w, const float* b, void* y,
                    void* sum, float* mean, float* rstd, int N, int C, float eps, hipStream_t s);
// partial buffers: [layer_norm_bwd_blocks(N)][C] each
int layer_norm_bwd_blocks(int N);
// gsum (optional): gradient reaching the residual sum directly, added into dx
void layer_norm_bwd(bool bf16, const void* dy, const void* x, const float* w, const float* mean, const float* rstd,
                    const void* gsum, void* dx, float* pdw, float* pdb, float* dw, float* db, int N, int C,
                    hipStream_t s);

void bias_gelu_fwd(bool bf16, const void* x, const float* b, void* y, int64_t n, int H, hipStream_t s);
// partial buffer: [bias_gelu_bwd_splits(N)][H]
int bias_gelu_bwd_splits(int N);
void bias_gelu_bwd(bool bf16, const void* dy, const void* x, const float* b, void* dx, float* pdb, float* db, int N,
                   int H, hipStream_t s);

// out[c] = sum_r x[r][c] over an [N, H] activation (H % 8 == 0); partials [bias_gelu_bwd_splits(N)][H]
// (out_bf != nullptr: the result is written as bf16 to out_bf instead of out)
void column_sum(bool bf16, const void* x, float* part, float* out, uint16_t* out_bf, int N, int H, hipStream_t s);

// dw / db (layer_norm_bwd), db (bias_gelu_bwd), out and out_bf (column_sum) all nullptr: only
// the partials are written; their column reduction is left to col_reduce_multi.

// Column reductions out[c] = sum_r part[r][c] (fixed order, as the single launches) of many
// [R, C] fp32 partial arrays in one launch; a job reduces a (and b if set); oa_bf set: a's
// result as bf16 into oa_bf instead of oa.  blk0 is filled by col_reduce_multi.
struct CrJob {
  const float* a;
  float* oa;
  const float* b;
  float* ob;
  uint16_t* oa_bf;
  int R, C, blk0, pad;
};
constexpr int kCrMaxJobs = 40;  // 2.2 KB of kernel arguments
struct CrJobs {
  CrJob j[kCrMaxJobs];
  int n;
};
void col_reduce_multi(CrJobs& jobs, hipStream_t s);

// column_sum's [S = bias_gelu_bwd_splits(N), H] partials of many bf16 [N, H] activations
// in one launch (blk0 filled by colsum_multi); reduce them with col_reduce_multi
struct CsJob {
  const uint16_t* x;
  float* part;
  int N, H, S, blk0;
};
constexpr int kCsMaxJobs = 64;  // 1.5 KB of kernel arguments
struct CsJobs {
  CsJob j[kCsMaxJobs];
  int n;
};
void colsum_multi(CsJobs& jobs, hipStream_t s);

// out[i] = bf16(sum_s parts[s][i]) over S bf16 partial arrays of n elements (n % 8 == 0)
void split_sum_bf16(const uint16_t* parts, uint16_t* out, int64_t n, int S, hipStream_t s);

// (dst, src, bytes) regions copied by one launch; pointers 16-byte aligned,
// byte counts multiples of 4
constexpr int kMaxCopies = 12;
struct CopyList {
  void* dst[kMaxCopies];
  const void* src[kMaxCopies];
  int64_t bytes[kMaxCopies];
  int n;
};
void multi_copy(const CopyList& cl, hipStream_t s);

// ViT patch embedding input: uint8 images [B][C][H][W] -> bf16 patch rows [B * (H/P) * (W/P)][C * P * P]
// in Conv2d(C, D, P, stride P) weight order, values / 255 (P % 8 == 0)
void patchify_u8(const uint8_t* x, uint16_t* out, int B, int C, int H, int W, int P, hipStream_t s);
// h[b][0] = cls + pos[0], h[b][1 + i] = y[b][i] + pos[1 + i]  (bf16, D % 8 == 0): the token concat + position
// embedding of a ViT in one pass; backward: dy = dh[:, 1:] (contiguous), dpos = sum_b dh[b], dcls = dpos[0]
void embed_tokens_fwd(const uint16_t* y, const uint16_t* cls, const uint16_t* pos, uint16_t* h, int B, int N, int D,
                      hipStream_t s);
void embed_tokens_bwd(const uint16_t* dh, uint16_t* dy, uint16_t* dpos, uint16_t* dcls, int B, int N, int D,
                      hipStream_t s);

void xent_fwd(bool bf16, const void* z, const int64_t* y, float* loss, float* lse, int N, int K, hipStream_t s);
void xent_bwd(bool bf16, const void* z, const int64_t* y, const float* lse, const float* gscale, void* dz, int N, int K,
              hipStream_t s);

}  // namespace p2fused
