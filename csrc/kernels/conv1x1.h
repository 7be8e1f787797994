#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pdt {

// 1x1 / stride-1 convolution with 64 input and 256 output channels (ResNet-50 layer1's expanding conv3 and its
// downsample): y[m][k] = sum_c x[m][c] * w[k][c] over M pixels, optional BN statistics of the rounded outputs into
// fp64 slots (conv_fwd.h).  See conv1x1.hip.
bool conv1x1_c64_supported(int C, int Kout);
int conv1x1_c64_mode(int set);  // returns the previous on/off mode; set >= 0 changes it (PDT_CONV1X1 seeds it)
// The same GEMM as the backward-data pass of a 1x1 256 -> 64 conv, with the fused block-output BN-backward epilogue
// (conv_fwd.h EPI 3: + residual, ReLU bit of the block output, sum dz and sum dz * xhat1 into fp64 slots).
// y2 / coef2 != nullptr: a second BN branch (EPI 4), slots [C][4] = (sum dz, sum dz*xhat1, sum dz, sum dz*xhat2).
// cin = reduction channels of x (64, or 128 with one branch: ResNet-50 layer2.0's 256 -> 128 conv1).
void conv1x1_c64_bnb_launch(const uint16_t* x, const uint16_t* w, uint16_t* y, const uint16_t* res,
                            const uint16_t* y1, const float* coef1, const uint16_t* y2, const float* coef2,
                            const uint8_t* mask, double* slots, int64_t M, int cin, int dtype, hipStream_t s);
// pre_coef != nullptr (training, with stats): x is the producer conv's raw output, the kernel applies that BN + ReLU
// (scale[64] | shift[64]) to its input fragments
void conv1x1_c64_launch(const uint16_t* x, const uint16_t* w, uint16_t* y, double* stats, int64_t M, int dtype,
                        hipStream_t s, const float* pre_coef = nullptr);

// The same two GEMMs for C = 128 / 256 / 512 reduction channels and N output channels (ResNet-50 layers 2-4: conv3
// forward, conv1 backward-data), N split into slices of 256 (C = 128) or 128 channels (conv1x1x.hip).  w is [N][C].
bool conv1x1x_supported(int C, int N);
bool conv1x1x_bnb_supported(int C, int N);  // the backward-data kernel: also C = 64
bool conv1x1x_prefer_l1();  // conv1x1x_l1_mode(1): layer1's 64 / 128 -> 256 backward-data on conv1x1x_bnb (A/B)
int conv1x1x_l1_mode(int set);  // ... switched at run time (tests); returns the previous mode
int conv1x1x_mode(int set);  // PDT_CONV1X1X seeds it; set >= 0 changes it, returns the previous mode
// st > 1: a 1x1 / stride-st conv over nimg H x W images (M = nimg * P * Q output pixels; the downsample convs)
void conv1x1x_launch(const uint16_t* x, const uint16_t* w, uint16_t* y, double* stats, int64_t M, int C, int N,
                     int dtype, hipStream_t s, int st = 1, int nimg = 0, int H = 0, int W = 0);
void conv1x1x_bnb_launch(const uint16_t* x, const uint16_t* w, uint16_t* y, const uint16_t* res, const uint16_t* y1,
                         const float* coef1, const uint16_t* y2, const float* coef2, const uint8_t* mask,
                         double* slots, int64_t M, int C, int N, int dtype, hipStream_t s);

}  // namespace pdt
