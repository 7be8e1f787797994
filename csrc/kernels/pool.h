#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
namespace pdt {
void bn_relu_maxpool_launch(int dtype, const uint16_t* y, const float* coef, uint16_t* out, uint8_t* idx, int N, int H,
                            int W, int C, hipStream_t s, int pad = 1);
void maxpool_bwd_relu_launch(int dtype, const uint16_t* dp, const uint8_t* idx, const uint16_t* y, const float* coef,
                             uint16_t* dz, int N, int H, int W, int C, hipStream_t s, int pad = 1);
void stem_pool_bwd_reduce_launch(int dtype, const uint16_t* dp, const uint8_t* idx, const uint16_t* y,
                                 const float* coef, double* slots, int N, int H, int W, int C, hipStream_t s);
void stem_pool_bwd_reduce_out_launch(int dtype, const uint16_t* dp, const uint16_t* out, const float* coef,
                                     double* slots, int N, int H, int W, int C, hipStream_t s);
void pooled_bwd_reduce_launch(int dtype, const uint16_t* dp, const uint16_t* out, const float* coef, double* slots,
                              int64_t rows, int C, hipStream_t s);
void stem_pool_bwd_apply_launch(int dtype, const uint16_t* dp, const uint8_t* idx, const uint16_t* y,
                                const float* coef, const float* bcoef, uint16_t* dy, int N, int H, int W, int C,
                                hipStream_t s);
void avgpool_fwd_launch(int dtype, const uint16_t* x, uint16_t* feat, int N, int HW, int C, int ldf, hipStream_t s);
void avgpool_bwd_launch(int dtype, const uint16_t* dfeat, uint16_t* g, int N, int HW, int C, int ldf, hipStream_t s);
}  // namespace pdt
