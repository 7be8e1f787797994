#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pdt {

struct ConvWgradArgs {
  const uint16_t* x;   // [N][H][W][C] forward input
  const uint16_t* dy;  // [P][Kout] gradient of the forward output (P = N*Pm*Qm pixels, NHWC)
  float* ws;           // [splits][Kout][ldw] fp32 partials
  int N, H, W, C, Kout, T, U;
  int Pm, Qm;
  int stride_h, stride_w, pad_h, pad_w, dil_h, dil_w;
  int P;               // N*Pm*Qm
  int ldw;             // >= T*U*C
  int cs;              // elements per pixel of x (== C except in window mode)
  int win;             // stem window mode (see conv_wgrad.hip)
  int ldy = 0;         // dY pixel stride (0 = Kout): a channel slice of a wider gradient (grouped conv; 64x64 tile only)
  // nslice > 1: ONE launch over every channel slice of a grouped conv (blockIdx.z = slice s; 64x64 tile only): x and dy
  // advance by s * C / s * Kout elements and the partials are [splits][nslice][Kout][ldw] (one wgrad_reduce over
  // nslice * Kout rows sums every slice)
  int nslice = 0;
  int splits, pix_per_split;  // filled by conv_wgrad_plan
  int tile;                   // 64, 128, 256 or kWgradWide (filled by conv_wgrad_plan)
  uint32_t div_pq_mul, div_pq_shift, div_q_mul, div_q_shift;  // FastDiv of Pm*Qm and Qm (launcher)
  // stem only (f_y != nullptr): dY computed in-kernel from the 3x3/2 max-pool backward + ReLU + BN backward
  // (dy unused).  f_y: conv output [P][64]; f_dp / f_idx: pooled gradient and argmax [N][f_OH][f_OW][64];
  // f_coef: BN forward scale, shift (not read: the argmax carries the ReLU mask, see bn_relu_maxpool); f_bcoef:
  // backward apply A, B, C (64 each)
  const uint16_t* f_y = nullptr;
  const uint16_t* f_dp = nullptr;
  const uint8_t* f_idx = nullptr;
  const float* f_coef = nullptr;
  const float* f_bcoef = nullptr;
  int f_OH = 0, f_OW = 0;
  // layer1 3x3 kernel only: x is the RAW output of the producer conv; its BatchNorm + ReLU (scale[64] | shift[64])
  // is applied to each staged input halo in LDS (see conv_l1.hip, PRE)
  const float* pre_coef = nullptr;
};

constexpr int kWgradWide = 2;  // ConvWgradArgs::tile code of the 256 (c: two 128-wide column blocks) x 128 (k) kernel
int wgrad_tile(int C, int Kout, int win);  // 256 (ping-pong), 128 (C == 64: two-tap pairs) or 64
int wgrad_ctiles(const ConvWgradArgs& a);  // (tap, c) tiles of the dW column axis for a.tile
void conv_wgrad_plan(ConvWgradArgs& a, int target_blocks);
void conv_wgrad_launch(const ConvWgradArgs& a, int dtype, hipStream_t s);
// 3x3/s1/p1 C = Kout = 64, W = 56 specialisation: all 9 taps per block, persistent over 4-row tiles;
// writes `blocks` fp32 partials [blocks][64][ldw] (ldw >= 576) for wgrad_reduce.
bool wgrad3x3_c64_supported(int C, int Kout, int T, int U, int W, int stride, int pad, int win);
int wgrad3x3_c64_blocks();
int wgrad3x3_c64_launch(const ConvWgradArgs& a, int partials, int dtype, hipStream_t s);  // partials written
void wgrad_reduce_launch(const float* ws, int splits, int rows, int cols, int ldw, int64_t split_stride,
                         float* out, int ldo, float scale, bool accumulate, hipStream_t s);

}  // namespace pdt
