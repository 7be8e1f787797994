#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
// VGG-family kernels (vgg.hip): fused BN/bias + ReLU + MaxPool(2, 2) and its backward, classifier bias + ReLU +
// Dropout forward / backward, NHWC <-> NCHW feature reorder, bias-as-BN coefficients
namespace pdt {
void bn_relu_maxpool2_launch(int dtype, const uint16_t* y, const float* coef, uint16_t* out, uint8_t* idx, int64_t N,
                             int H, int W, int C, hipStream_t s);
void maxpool2_bwd_launch(int dtype, const uint16_t* dp, const uint8_t* idx, const uint16_t* out, const uint16_t* y,
                         const float* bcoef, uint16_t* dy, int64_t N, int H, int W, int C, hipStream_t s);
void fc_act_fwd_launch(int dtype, const uint16_t* z, const float* bias, uint16_t* out, int64_t rows, int F, double p,
                       uint64_t seed, hipStream_t s);
void fc_act_bwd_launch(int dtype, const uint16_t* dh, const uint16_t* out, uint16_t* dz, int64_t n, double p,
                       hipStream_t s);
void nhwc_nchw16_launch(const uint16_t* src, uint16_t* dst, int64_t N, int HW, int C, bool to_nchw, hipStream_t s);
void bias_coef_launch(const float* bias, float* coef, int C, hipStream_t s);
}  // namespace pdt
