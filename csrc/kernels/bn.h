#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pdt {
void bn_slot_sum_launch(const double* slots, int C, int K, double* sums, hipStream_t s);
void bn_finalize_slots_launch(const double* slots, double count, const float* gamma, const float* beta, float eps,
                              float momentum, float* rm, float* rv, float* coef, double* sums, int C,
                              bool update_running, hipStream_t s);
void bn_bwd_finalize_slots_launch(const double* slots, int K, double count, const float* coef1, const float* gamma1,
                                  float* dgamma1, float* dbeta1, float* bcoef1, const float* coef2,
                                  const float* gamma2, float* dgamma2, float* dbeta2, float* bcoef2, float gscale,
                                  int C, hipStream_t s);
void bn_finalize_launch(const double* sums, double count, const float* gamma, const float* beta, float eps,
                        float momentum, float* rm, float* rv, float* coef, int C, bool update_running,
                        hipStream_t s);
void bn_eval_coef_launch(const float* gamma, const float* beta, const float* rm, const float* rv, float eps,
                         float* coef, int C, hipStream_t s);
void bn_apply_launch(int dtype, const uint16_t* y, const float* coef, const uint16_t* res, const float* rcoef,
                     uint16_t* out, uint8_t* mask, int64_t n, int C, int resmode, bool relu, hipStream_t s);
int bn_bwd_reduce_blocks(int64_t rows, int C);
void bn_bwd_reduce_launch(int dtype, const uint16_t* g, const uint8_t* mask, const uint16_t* y1, const float* coef1,
                          const uint16_t* y2, const float* coef2, double* slots, int blocks, int64_t rows, int C,
                          hipStream_t s);
void bn_bwd_finalize_launch(const double* sums, double count, const float* coef, const float* gamma, float* dgamma,
                            float* dbeta, float gscale, float* bcoef, int C, hipStream_t s);
void bn_bwd_apply_launch(int dtype, const uint16_t* g, const uint8_t* mask, const uint16_t* y1, const float* b1,
                         uint16_t* dy1, const uint16_t* y2, const float* b2, uint16_t* dy2, uint16_t* dz_out, int64_t n,
                         int C, hipStream_t s);
}  // namespace pdt
