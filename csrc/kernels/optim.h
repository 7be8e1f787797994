#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
namespace pdt {
void nonfinite_check_launch(const float* g, int64_t n, float* found, hipStream_t s);
void sgd_launch(int dtype, float* p, const float* g, float* buf, uint16_t* shadow, const float* wd_mask, int64_t n,
                float lr, float momentum, float wd, float gscale, const float* loss_scale, const float* found_inf,
                bool first, hipStream_t s);
void cast16_launch(int dtype, const float* p, uint16_t* out, int64_t n, hipStream_t s);
void widen16_launch(int dtype, const uint16_t* in, float* out, int64_t n, hipStream_t s);
void amp_update_launch(float* scale, int* tracker, float* found_inf, float growth, float backoff, int interval,
                       hipStream_t s);
void gather16_launch(const uint16_t* src, const int* idx, uint16_t* dst, int64_t n, hipStream_t s);
void im2col_launch(int dtype, const float* x, uint16_t* out, int N, int C, int H, int W, int R, int S, int stride, int pad,
                   int ldk, hipStream_t s);
void stem_pack_launch(int dtype, const float* x, uint16_t* out, int N, int C, int H, int W, int pad, int Hp, int Wp,
                      hipStream_t s);
void stem_pack_u8_launch(int dtype, const uint8_t* x, uint16_t* out, int N, int C, int H, int W, int pad, int Hp,
                         int Wp, const float* scale, const float* shift, hipStream_t s);
void gather32_launch(const float* src, const int* idx, float* dst, int64_t n, hipStream_t s);
void scatter32_launch(const float* src, const int* idx, float* dst, int64_t n, hipStream_t s);
void bw_probe_launch(int mode, const uint16_t* x, const uint16_t* y, uint16_t* out, int64_t n, int blocks,
                     hipStream_t s);

}  // namespace pdt
