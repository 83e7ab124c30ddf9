// Fused BatchNorm (+ residual add) (+ ReLU) for channels-last activations
// (batchnorm.hip).  An NHWC activation is an [M, C] row-major matrix with
// M = N*H*W; bf16 selects uint16 bf16 activations, else fp32.  Parameters,
// statistics, partials and coefficients are fp32.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace p2bn {

// Work split of the column-statistics passes: tpr threads per row (8 channels
// each), rp row phases per 256-thread block, gx column blocks, S row splits.
struct BnPlan {
  int tpr, rp, gx, S;
};
BnPlan bn_plan(int M, int C);
// Plan of the statistics + finalize kernels (one launch instead of two; bf16,
// C <= 2048, S * C <= 16384): S == 0 when the shape is not eligible.
BnPlan bn_fused_plan(int M, int C);

// Training forward: batch statistics (biased variance, shifted sums), running
// stats update (unbiased variance, PyTorch momentum convention), then
//   y = act((x - mean) * scale + b [+ res])      scale = w * rstd
// part: [2, S, C] fp32; coef: [3, C] fp32 scratch; mean / rstd: [C] (saved for backward).
// run_mean / run_var / nbt may be null (no running statistics).  ctr: a zeroed
// int (left zero) enabling the statistics + finalize kernel when bn_fused_plan
// allows it (part then needs [2, fused S, C]); null keeps the separate launches.
void bn_fwd_train(bool bf16, const void* x, const void* res, const float* w, const float* b, float* run_mean,
                  float* run_var, int64_t* nbt, float momentum, float eps, void* y, float* mean, float* rstd,
                  float* coef, float* part, int* ctr, int M, int C, bool relu, hipStream_t s);

// Apply pass only, with coefficients [mean | w * rstd | b] computed elsewhere
// (the statistics epilogue of a convolution, gemm_core.h BnEpi).
void bn_apply_train(bool bf16, const void* x, const void* res, const float* coef, void* y, int M, int C, bool relu,
                    hipStream_t s);

// Backward apply pass only (bf16), coef = [A | B | D] computed elsewhere (the
// backward statistics epilogue of a convolution's input gradient):
//   dx = A dz' + B (x - mean) + D,  dz' = relu ? dy * (y > 0) : dy
void bn_apply_bwd_only(const void* dy, const void* y, const void* x, const float* mean, const float* coef, void* dx,
                       int M, int C, bool relu, hipStream_t s);

// Inference forward with running statistics (one launch; coef unused, kept for
// the call signature).  w, b, run_mean, run_var must be 16-byte aligned.
void bn_fwd_eval(bool bf16, const void* x, const void* res, const float* w, const float* b, const float* run_mean,
                 const float* run_var, float eps, void* y, float* coef, int M, int C, bool relu, hipStream_t s);

// Backward of y = act(bn(x) [+ res]) given dy and the saved output y (ReLU mask):
//   dz = relu ? dy * (y > 0) : dy
//   db = sum dz, dw = rstd * sum dz (x - mean)
//   dx = w rstd (dz - db / M - xhat dw / M);   dres = dz (if dres != null)
// part: [2, S, C]; coef: [3, C] scratch; ctr as bn_fwd_train.
void bn_bwd(bool bf16, const void* dy, const void* dy2, const void* y, const void* x, const float* w, const float* mean,
            const float* rstd, void* dx, void* dres, float* dw, float* db, float* coef, float* part, int* ctr, int M,
            int C, bool relu, hipStream_t s);

}  // namespace p2bn
