#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pdt {

// fp32 implicit-GEMM convolution (same geometry contract as ConvFwdArgs, conv_fwd.hip): forward, multi-phase
// backward-data, 1x1 / linear layers.  Optional residual add and BN statistics rows.
struct Conv32Args {
  const float* x;
  const float* w;
  float* y;
  const float* res;
  double* stats;  // optional [kStatSlots][Kout][2] (sum, sumsq); filled through per-block rows (srows)
  // bnb != 0 (backward-data only): the consumer BatchNorm's backward reduce fused into the epilogue -- the output is
  // dz = dx * (bn_mref > 0) (bn_mref: the post-ReLU activation) and stats receives (sum dz, sum dz * xhat) with
  // xhat = (bn_y1 - mean) * invstd, coef = [scale | shift | mean | invstd] x Kout
  int bnb = 0;
  const float* bn_mref = nullptr;
  const float* bn_y1 = nullptr;
  const float* bn_coef = nullptr;
  // a second BN branch sharing dz (a downsample block's output: the main-branch and the downsample BN); stats then
  // receive 4 quantities per channel: (sum dz, sum dz * xhat1, sum dz, sum dz * xhat2)
  const float* bn_y2 = nullptr;
  const float* bn_coef2 = nullptr;
  float* srows;
  int srows_pp;
  int N, H, W, C, Kout, T, U;
  int cs;  // elements per input pixel (0: == C).  4: the stem's "window" mode over a zero-padded NHWC4 image, one
           // 32-element K-step = 8 consecutive pixels x 4 channels of a kernel row (conv_fwd.hip's window mode)
  int Pm, Qm;
  int ist_h, ist_w, ioff_h, ioff_w, tstep_h, tstep_w;
  int OH, OW, ost_h, ost_w, ooff_h, ooff_w;
  int64_t M;
  int m_tiles, n_tiles;
  uint32_t pq_mul, pq_shift, q_mul, q_shift;
  int nphase;
  int pT[4], pU[4], pioff_h[4], pioff_w[4], pPm[4], pQm[4], pooff_h[4], pooff_w[4], pmt[4];
  int64_t pwoff[4];
  uint32_t ppq_mul[4], ppq_shift[4], pq1_mul[4], pq1_shift[4];
};
void conv32_launch(Conv32Args a, int bm, int bn, hipStream_t s);
// 3x3 / stride-1 same-grid convolutions on 64-channel output tiles: the halo kernel (default) or conv32_kernel (0); returns the
// previous setting
int conv32_set_halo(int on);

// fp32 weight gradient: ws[split][Kout][ldw], column tap*C + c, split-K over pixels (sum with wgrad_reduce).
struct Wgrad32Args {
  const float* x;   // [N][H][W][C]
  const float* dy;  // [N][Pm][Qm][Kout]
  float* ws;
  int N, H, W, C, Kout, T, U, Pm, Qm, stride, pad, ldw, splits, pix_per_split;
  int64_t P;
  int tile = 64;  // 64: 64x64 output tile, 4 waves | 128: 128x128, 8 waves (C, Kout % 128 == 0)
  // window-pair mode (the fp32 stem's weight gradient over the zero-padded NHWC4 image; 64x64 tile only): cs = 4
  // elements per pixel, a "tap" t is the kernel-row pair (2t, 2t+1) = input row offset t * tstep, and its 64 columns
  // are 8 pixels x 4 channels of row 2t (chunks 0..7) then of row 2t+1 (chunks 8..15 read element sc * 4 + pair_skip:
  // pair_skip = one padded row - 32)
  int cs = 0, pair_skip = 0, tstep = 1;
  // 4-pair stem kernel only (f_y != nullptr): dY is not read but computed per staged chunk from the max-pool backward,
  // the ReLU mask and the BN-backward apply (the math of stem_pool_bwd_apply32): f_dp / f_idx pooled gradient and
  // argmax [N][f_OH][f_OW][64], f_y the conv output [P][64], f_coef the forward BN coefficients (scale | shift),
  // f_bcoef the backward apply's A | B | C (64 each)
  const float* f_dp = nullptr;
  const uint8_t* f_idx = nullptr;
  const float* f_y = nullptr;
  const float* f_coef = nullptr;
  const float* f_bcoef = nullptr;
  int f_OH = 0, f_OW = 0;
};
void wgrad32_launch(const Wgrad32Args& a, hipStream_t s);

// elementwise / reduction kernels over NHWC fp32 activations (C % 4 == 0)
void bn_apply32_launch(const float* y, const float* coef, const float* res, const float* rcoef, float* out, int64_t n,
                       int C, int resmode, bool relu, hipStream_t s);
int bn_bwd_reduce32_blocks(int64_t rows, int C);
void bn_bwd_reduce32_launch(const float* g, const float* mref, const float* y1, const float* coef1, const float* y2,
                            const float* coef2, double* slots, int blocks, int64_t rows, int C, hipStream_t s);
void bn_bwd_apply32_launch(const float* g, const float* mref, const float* y1, const float* b1, float* dy1,
                           const float* y2, const float* b2, float* dy2, float* dz, int64_t n, int C, hipStream_t s);
void bn_relu_maxpool32_launch(const float* y, const float* coef, float* out, uint8_t* idx, int N, int H, int W, int C,
                              hipStream_t s);
// the stem's backward tail with dz recomputed instead of stored (max-pool backward x ReLU mask): BN-backward reduce
// into fp64 slots, and the apply dy = A*dz + B*y + C
void stem_pool_bwd_reduce32_launch(const float* dp, const uint8_t* idx, const float* y, const float* coef, double* slots,
                                   int blocks, int N, int H, int W, int C, hipStream_t s);
// the same sums over the pooled output (mask out > 0, BN input (out - shift) / scale): no window gather, no y0 read
void stem_pool_bwd_reduce_out32_launch(const float* dp, const float* out, const float* coef, double* slots, int blocks,
                                       int64_t rows, int C, hipStream_t s);
void stem_pool_bwd_apply32_launch(const float* dp, const uint8_t* idx, const float* y, const float* coef, const float* b,
                                  float* dy, int N, int H, int W, int C, hipStream_t s);
void maxpool_bwd_relu32_launch(const float* dp, const uint8_t* idx, const float* y, const float* coef, float* dz, int N,
                               int H, int W, int C, hipStream_t s);
void avgpool32_fwd_launch(const float* x, float* feat, int N, int HW, int C, int ldf, hipStream_t s);
void avgpool32_bwd_launch(const float* dfeat, float* g, int N, int HW, int C, int ldf, hipStream_t s);
void xent32_launch(const float* logits, int ldl, const float* bias, const int64_t* target, int B, int ncls,
                   float* out_logits, float* dlogits, const float* loss_scale, float grad_div, float* row_loss,
                   float* row_correct, hipStream_t s);
void colsum32_launch(const float* d, int B, int ld, int ncols, float* out, float scale, hipStream_t s);
// fp32 NCHW images -> zero-padded NHWC4 [N][Hp][Wp][4] (channel 3 and the border zero): the window-mode stem operand
void stem_pack32_launch(const float* x, float* out, int N, int C, int H, int W, int pad, int Hp, int Wp, hipStream_t s);
void im2col32_launch(const float* x, float* out, int N, int C, int H, int W, int R, int S, int stride, int pad, int ldk,
                     hipStream_t s);

}  // namespace pdt
