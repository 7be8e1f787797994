#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
namespace pdt {
void xent_launch(int dtype, const uint16_t* logits, int ldl, const float* bias, const int64_t* target, int B, int ncls,
                 float* out_logits, uint16_t* dlogits, const float* loss_scale, float grad_div, float* row_loss,
                 float* row_correct, hipStream_t s);
void metrics_launch(const float* row_loss, const float* row_correct, int B, float* out, hipStream_t s);
void colsum_launch(int dtype, const uint16_t* d, int B, int ld, int ncols, float* out, float scale, hipStream_t s);
}  // namespace pdt
