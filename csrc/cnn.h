// Fused MNIST-CNN training step for MI355X (gfx950).
//
// Model (reference p2pfl/learning/pytorch/mnist_examples/models/cnn.py:55-98):
//   conv5x5(1->32,"same") -> ReLU -> maxpool2 -> conv5x5(32->64,"same") -> ReLU
//   -> maxpool2 -> flatten(3136) -> FC 3136->2048 -> ReLU -> FC 2048->10 -> CE
// trained with Adam.  One training step is 8 kernel launches (cnn_*.hip):
//
//  1 conv1_fwd         direct 5x5 conv + bias + ReLU + maxpool, input gathered
//                      by index from the uint8 dataset (/255 folded in) -> P1 (HWC bf16) + argmax
//                      (+ kx-shifted planar copies of P1 for conv2_wgrad when training)
//  2 conv2_fwd         implicit-GEMM on MFMA 32x32x16 bf16, one wave per pooled row,
//                      operands streamed from L2, bias + ReLU + maxpool epilogue -> A1 + argmax
//  3 gemm_skinny       FC1: [B x 3136] x [3136 x 2048], split-K fp32 slabs
//  4 head              slab reduce + bias + ReLU -> H; FC2; softmax-xent; dlogits;
//                      dH = relu'(H) * dlogits W2; loss/accuracy stats
//  5 route_fc2         dA1 = dH x W1 (W1^T bf16 shadow) + pool2/ReLU backward in
//                      the epilogue -> dC2 map + fp32 bias terms;  extra blocks:
//                      dW2 = dlogits^T H and db2 with Adam applied in place
//  6 fc1_wgrad_adam    dW1 = dH^T A1 on MFMA with Adam fused into the epilogue:
//                      the 6.4 M-element gradient never touches memory; writes
//                      W1 (fp32), m, v and both bf16 shadows (W1, W1^T)
//  7 conv2_bwd         single-wave blocks, two roles:
//                      dgrad (image, 32-position tile): dP1 = transposed conv on
//                      MFMA from an LDS HWC window of dC2, then the conv1 weight
//                      gradient as a sparse fp32 gather at each pool1 argmax pixel;
//                      wgrad (tap, image pair): dW2[:, :, tap] = dC2 x shifted P1
//                      on MFMA, operands streamed from L2 -> slab per pair
//  8 conv_adam         fixed-order slab reduction (+ conv2 bias from gB) + Adam
//                      for the conv params + packed bf16 conv2 shadows (two layouts)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace p2cnn {

constexpr int kImg = 28;
constexpr int kC1 = 32;
constexpr int kC2 = 64;
constexpr int kFeat = 3136;  // 64 * 7 * 7
constexpr int kHid = 2048;
constexpr int kCls = 10;
constexpr int kTaps = 25;
// FC1 K-splits whose layout the XCDs share (gemm_skinny / route_rm, xcd_align):
// 49 K-groups of 64 features -> 7 splits of 448 features = 14 routing tiles each
constexpr int kXcdSplits = 7;
bool xcd_align();

// Adam hyper-parameters.  The step count t is read from device memory as
// (*adam_t + t_off): the host sets the base once per epoch and each captured
// step bakes in its own offset, so a whole epoch replays as one HIP graph
// with no per-step counter kernel.
struct AdamCfg {
  float lr, beta1, beta2, eps, weight_decay;
};

// Arena offsets (elements) of every parameter, from ParamLayout.
struct Offsets {
  int64_t c1w, c1b, c2w, c2b, l1w, l1b, l2w, l2b;
};

// p1s (may be null = inference): [B][5][32][18][16] shifted copies, zero padding.
void conv1_fwd(const uint8_t* x, const int64_t* idx, const float* params, Offsets off, uint16_t* p1, uint8_t* am1,
               uint16_t* p1s, int B, hipStream_t s);

void conv2_fwd(const uint16_t* p1, const uint16_t* w2r, const float* params, Offsets off, uint16_t* a1, uint8_t* am2,
               int B, hipStream_t s);

// conv1_fwd + conv2_fwd in one launch (P1 window in LDS per pooled row): writes AM1,
// P1s (may be null = inference), A1, AM2 -- and P1 only when p1 is non-null
void conv12_fwd(const uint8_t* x, const int64_t* idx, const float* params, Offsets off, const uint16_t* w2r,
                uint16_t* p1, uint8_t* am1, uint16_t* p1s, uint16_t* a1, uint8_t* am2, int B, hipStream_t s);

void gemm_skinny(const uint16_t* A, const uint16_t* Bt, float* slabs, int mrows, int N, int K, int S, hipStream_t s);

// w2bf non-null: the FC2 weight is read from its bf16 copy [10][2048] (half the
// bytes of the fp32 master) -- kept current by fc1_conv_adam / pack_shadows
void head(const float* slabs, int S, int mrows, const float* params, Offsets off, const int64_t* labels,
          const int64_t* idx, int B, int train, uint16_t* H, uint16_t* dH, float* dlogits, float* stats,
          const uint16_t* w2bf, hipStream_t s);

void fc1_wgrad_adam(const uint16_t* dH, const uint16_t* a1, int mrows, float* params, float* m, float* v,
                    float* gdump, uint16_t* w1bf, uint16_t* w1tbf, Offsets off, const int* adam_t, int t_off,
                    AdamCfg cfg, hipStream_t s);

// One launch: dA1 = dH x W1 (reads the W1^T shadow) with the pool2/ReLU
// backward fused into the epilogue -> dC2 map [B][64][14x16] (all 4 window
// positions written, so no clearing; cols 14/15 stay zero from allocation) and
// the fp32 alive-masked dA1 [B][3136] (conv2 bias terms); plus, in extra
// blocks (with_fc2), the FC2 weight/bias gradient with Adam.
void route_fc2(const uint16_t* dH, const uint16_t* w1t, const uint8_t* am2, int mrows, int B, uint16_t* dc2m,
               float* gb, const float* dlogits, const uint16_t* H, float* params, float* m, float* v, float* gdump,
               Offsets off, const int* adam_t, int t_off, AdamCfg cfg, bool with_fc2, hipStream_t s);

// route_fc2 reading the row-major W1 (the forward shadow w1bf) through LDS
// transpose reads, so no W1^T shadow is needed (fc1 Adam with w1tbf = null).
void route_fc2_rm(const uint16_t* dH, const uint16_t* w1, const uint8_t* am2, int mrows, int B, uint16_t* dc2m,
                  float* gb, const float* dlogits, const uint16_t* H, float* params, float* m, float* v,
                  float* gdump, Offsets off, const int* adam_t, int t_off, AdamCfg cfg, bool with_fc2,
                  float* ws, int* ctr, hipStream_t s);  // ws/ctr non-null: split-K over 2 slices

// One launch: conv2 input gradient + pool1/ReLU backward + conv1 weight
// gradient (-> wslab1 [B][7][832]) and conv2 weight gradient
// (-> wslab2 [ceil(B/2)][25][64][32]).
void conv2_bwd(const uint16_t* dc2m, const uint16_t* p1s, const uint8_t* am1, const uint16_t* w2q, const uint8_t* x,
               const int64_t* idx, float* wslab1, float* wslab2, int B, hipStream_t s);

void conv_adam(const float* wslab1, const float* wslab2, const float* gb, int B, float* params, float* m, float* v,
               float* gdump, uint16_t* w2r, uint16_t* w2q, Offsets off, const int* adam_t, int t_off, AdamCfg cfg,
               hipStream_t s);

// conv_adam and fc1_wgrad_adam in one launch (run after conv2_bwd): the conv
// reduction + Adam blocks hide behind the HBM-bound FC1 Adam stream.  With
// dlogits / H non-null the FC2 gradient + Adam blocks join the launch too
// (then route_fc2 runs with with_fc2 = false).
// The next step's forward inputs / outputs for fc1_conv_adam_fwd: the uint8 dataset,
// its row indices, P1 / AM1 / P1s / A1 / AM2 buffers (A1: the other of two
// step-parity buffers -- this launch's FC1 wgrad still reads the current one), the
// next batch size, and 4 zero int32 (3 tickets, reset by the launch itself, and a
// timeout flag).
struct FwdNext {
  const uint8_t* x;
  const int64_t* idx;
  uint16_t* p1;
  uint8_t* am1;
  uint16_t* p1s;
  uint16_t* a1;
  uint8_t* am2;
  int B;
  int* sync;
};
void fc1_conv_adam_fwd(const uint16_t* dH, const uint16_t* a1, int mrows, const float* wslab1, const float* wslab2,
                       const float* gb, int B, float* params, float* m, float* v, float* gdump, uint16_t* w1bf,
                       uint16_t* w1tbf, uint16_t* w2r, uint16_t* w2q, Offsets off, const int* adam_t, int t_off,
                       AdamCfg cfg, const float* dlogits, const uint16_t* H, uint16_t* w2bf, const FwdNext& f,
                       hipStream_t s);

void fc1_conv_adam(const uint16_t* dH, const uint16_t* a1, int mrows, const float* wslab1, const float* wslab2,
                   const float* gb, int B, float* params, float* m, float* v, float* gdump, uint16_t* w1bf,
                   uint16_t* w1tbf, uint16_t* w2r, uint16_t* w2q, Offsets off, const int* adam_t, int t_off,
                   AdamCfg cfg, const float* dlogits, const uint16_t* H, uint16_t* w2bf, hipStream_t s);

// Standalone packing of the bf16 shadows from fp32 params (after set_parameters).
void pack_shadows(const float* params, Offsets off, uint16_t* w2r, uint16_t* w2q, uint16_t* w1bf, uint16_t* w1tbf,
                  uint16_t* w2bf, hipStream_t s);

constexpr int kP1sPlane = 18 * 16;                 // one shifted padded P1 channel plane
constexpr int kP1s = 5 * kC1 * kP1sPlane;          // P1s elements per image (46080)
constexpr int kDgTiles = 7;                        // 32-position tiles per image in conv2_dgrad
constexpr int kSlab1 = kC1 * kTaps + kC1;          // conv1 weight + bias partial per (image, tile) (832)
constexpr int kWgG = 2;                            // images per conv2_wgrad wave
constexpr int kSlab2 = kTaps * kC2 * kC1;          // conv2 weight partial per image pair, [tap][oc][ic]
__host__ __device__ inline int wgrad_groups(int B) { return (B + kWgG - 1) / kWgG; }

}  // namespace p2cnn
