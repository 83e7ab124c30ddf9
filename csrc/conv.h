// Host launch API of the implicit-GEMM convolutions (csrc/conv.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gemm.h"

namespace p2 {

// NHWC activations, (O, kh, kw, C) weights, bf16.  Output spatial size
// OH = (H + 2 pad - dil (kh - 1) - 1) / stride + 1 (same for W).
struct ConvShape {
  int N, H, W, C;  // input
  int O, OH, OW;   // output
  int kh, kw, stride, pad, dil;
};

// y[N*OH*OW][O] = conv(x, w)                                    (C % 64 == 0, O % 8 == 0)
// dx[N*H*W][C] = conv_transpose(dy, w)                           (O % 64 == 0, C % 8 == 0, stride 1 or 2)
// splits == 1: bf16 output; splits > 1 without counters: fp32 slabs [splits][rows][cols]
// at the output pointer (reduce with slab_sum); with counters (one zeroed int per 128x128
// output tile) the slabs go to `ws` and the launch reduces them into the bf16 output itself.
struct SplitK {
  int splits = 1;
  float* ws = nullptr;
  int* counters = nullptr;
};
// bn (optional): BatchNorm training statistics of the bf16 output computed in the
// launch (gemm.h BnEpi); needs splits == 1 or in-launch split-K (counters).
void conv_fwd(const ConvShape& s, const uint16_t* x, const uint16_t* w, void* y, const SplitK& k, int variant,
              hipStream_t st, const BnEpi* bn = nullptr);
// bn (optional, backward mode: BnEpi::bx set): BatchNorm backward statistics of the
// BN whose output this dgrad differentiates, computed in the launch.
// stride-2 input gradient by output phase (conv.hip ConvDgradS2A): dx_phases is
// [4 N (H/2) (W/2)][C] phase-major (or its split-K slabs); phase_interleave
// writes it into dX [N, H, W, C].  conv_dgrad_s2_ok: the shapes it takes.
bool conv_dgrad_s2_ok(const ConvShape& s);
// phases conv_dgrad_s2 computes (rows = s2_phases * N (H/2) (W/2)): 4, or 1 for a 1x1 kernel
int s2_phases(const ConvShape& s);
void conv_dgrad_s2(const ConvShape& s, const uint16_t* dy, const uint16_t* w, void* dx_phases, const SplitK& k,
                   int variant, hipStream_t st);
void phase_interleave(const ConvShape& s, const uint16_t* src, uint16_t* dx, hipStream_t st);
void conv_dgrad(const ConvShape& s, const uint16_t* dy, const uint16_t* w, void* dx, const SplitK& k, int variant,
                hipStream_t st, const BnEpi* bn = nullptr);
// dw[O][kh*kw*C] = sum over output pixels of dy (x) im2col(x)    (O % 8 == 0, C % 8 == 0)
// splits == 1: written as bf16 (out_bf16) or fp32; splits > 1: fp32 slabs
// [splits][O][kh*kw*C] at `out` (reduce with slab_sum).
void conv_wgrad(const ConvShape& s, const uint16_t* dy, const uint16_t* x, void* out, int out_bf16, const SplitK& k,
                int variant, hipStream_t st);

// Small-C direct convolution (the 3-channel stem, csrc/stem.hip).  x is fp32
// (xtype 0), bf16 (1) or uint8 (2) with arbitrary element strides, scaled by
// xscale and rounded to bf16; w is (O, kh, kw, C) bf16, y (N, OH, OW, O) bf16.
// O % 16 == 0 (forward) and O in {32, 64} (wgrad); kh * kw * C <= 160.
struct StemShape {
  int N, H, W, C, O, OH, OW, kh, kw, stride, pad;
  int64_t sn, sc, sh, sw;
  float xscale;
};
void stem_fwd(const StemShape& s, const void* x, int xtype, const uint16_t* w, uint16_t* y, hipStream_t st);
// part: fp32 workspace of stem_wgrad_parts(N, OH, OW) * O * kh * kw * C elements;
// dw (O, kh, kw, C) bf16 (out_bf16) or fp32.
int stem_wgrad_parts(int N, int OH, int OW);
void stem_wgrad(const StemShape& s, const void* x, int xtype, const uint16_t* dy, float* part, void* dw, int out_bf16,
                hipStream_t st);

// out[i] = sum_s slabs[s][i] (fp32 in; bf16 or fp32 out), n % 4 == 0.
void slab_sum(const float* slabs, int splits, int64_t n, void* out, int out_bf16, hipStream_t st);

}  // namespace p2
