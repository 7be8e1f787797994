// Fused softmax cross-entropy forward + backward + top-1 accuracy.
//
// One wave per row.  Reads 16-bit logits (+ fp32 bias), writes
//   * fp32 logits with bias (the model output returned to the caller),
//   * dlogits = (softmax - onehot) * (loss_scale / batch) in 16-bit (the backward seed, with the
//     AMP loss scale folded in: no separate scale kernel),
//   * per-row loss and correctness flags; metrics_reduce sums them into [loss_mean, acc_fraction].
// Accuracy follows the reference: top-1 index (first maximum) == target, as a fraction of the batch.
#include "../common.h"
#include "loss.h"

namespace pdt {

template <int DT>
__global__ __launch_bounds__(256) void xent_kernel(const uint16_t* __restrict__ logits, int ldl, const float* __restrict__ bias,
                                                   const int64_t* __restrict__ target, int B, int ncls,
                                                   float* __restrict__ out_logits, uint16_t* __restrict__ dlogits,
                                                   const float* __restrict__ loss_scale, float grad_div,
                                                   float* __restrict__ row_loss, float* __restrict__ row_correct) {
  using E = E16<DT>;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= B) return;
  const uint16_t* lr = logits + (int64_t)row * ldl;
  const int tgt = (int)target[row];
  float mx = -INFINITY;
  int amax = 0x7fffffff;
  for (int c = lane; c < ncls; c += 64) {
    const float v = E::to_f(lr[c]) + (bias ? bias[c] : 0.f);
    if (out_logits) out_logits[(int64_t)row * ncls + c] = v;
    if (v > mx) { mx = v; amax = c; }
  }
  // wave argmax (first index among equal maxima)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(mx, o, 64);
    const int oa = __shfl_xor(amax, o, 64);
    if (om > mx || (om == mx && oa < amax)) { mx = om; amax = oa; }
  }
  float se = 0.f;
  for (int c = lane; c < ncls; c += 64) se += __expf(E::to_f(lr[c]) + (bias ? bias[c] : 0.f) - mx);
  se = wave_sum(se);
  const float lse = mx + __logf(se);
  const float xt = E::to_f(lr[tgt]) + (bias ? bias[tgt] : 0.f);
  if (dlogits) {
    const float gs = (loss_scale ? *loss_scale : 1.f) / grad_div;
    uint16_t* dr = dlogits + (int64_t)row * ldl;
    const float inv = 1.f / se;
    for (int c = lane; c < ldl; c += 64) {
      float d = 0.f;
      if (c < ncls) {
        const float p = __expf(E::to_f(lr[c]) + (bias ? bias[c] : 0.f) - mx) * inv;
        d = (p - (c == tgt ? 1.f : 0.f)) * gs;
      }
      dr[c] = E::from_f(d);
    }
  }
  if (lane == 0) {
    row_loss[row] = lse - xt;
    row_correct[row] = (amax == tgt) ? 1.f : 0.f;
  }
}

void xent_launch(int dtype, const uint16_t* logits, int ldl, const float* bias, const int64_t* target, int B, int ncls,
                 float* out_logits, uint16_t* dlogits, const float* loss_scale, float grad_div, float* row_loss,
                 float* row_correct, hipStream_t s) {
  dim3 g((B + 3) / 4), b(256);
  if (dtype == kBF16)
    hipLaunchKernelGGL(xent_kernel<kBF16>, g, b, 0, s, logits, ldl, bias, target, B, ncls, out_logits, dlogits, loss_scale,
                       grad_div, row_loss, row_correct);
  else
    hipLaunchKernelGGL(xent_kernel<kF16>, g, b, 0, s, logits, ldl, bias, target, B, ncls, out_logits, dlogits, loss_scale,
                       grad_div, row_loss, row_correct);
}

// out[0] = mean(row_loss), out[1] = mean(row_correct)   (single block, deterministic)
__global__ __launch_bounds__(256) void metrics_kernel(const float* __restrict__ row_loss, const float* __restrict__ row_correct,
                                                      int B, float* __restrict__ out) {
  float l = 0.f, c = 0.f;
  for (int i = threadIdx.x; i < B; i += 256) { l += row_loss[i]; c += row_correct[i]; }
  l = wave_sum(l);
  c = wave_sum(c);
  __shared__ float sl[4], sc[4];
  if ((threadIdx.x & 63) == 0) { sl[threadIdx.x >> 6] = l; sc[threadIdx.x >> 6] = c; }
  __syncthreads();
  if (threadIdx.x == 0) {
    out[0] = (sl[0] + sl[1] + sl[2] + sl[3]) / (float)B;
    out[1] = (sc[0] + sc[1] + sc[2] + sc[3]) / (float)B;
  }
}

void metrics_launch(const float* row_loss, const float* row_correct, int B, float* out, hipStream_t s) {
  hipLaunchKernelGGL(metrics_kernel, dim3(1), dim3(256), 0, s, row_loss, row_correct, B, out);
}

// db[o] = scale * sum_b d[b][o]  (column sums of a 16-bit [B][ld] matrix; 64 columns per block)
template <int DT>
__global__ __launch_bounds__(256) void colsum_kernel(const uint16_t* __restrict__ d, int B, int ld, int ncols,
                                                     float* __restrict__ out, float scale) {
  using E = E16<DT>;
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rl = threadIdx.x >> 6;
  float s = 0.f;
  if (c < ncols)
    for (int b = rl; b < B; b += 4) s += E::to_f(d[(int64_t)b * ld + c]);
  __shared__ float red[4][64];
  red[rl][threadIdx.x & 63] = s;
  __syncthreads();
  if (rl == 0 && c < ncols) out[c] = scale * (red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x]);
}

// 16-byte loads: thread = 8 columns x one of 32 row lanes, LDS reduction over the lanes (deterministic).  The
// scalar kernel above (4 row lanes, 2-byte loads, 16 blocks for 1000 classes) took ~70 us for a 2.4 MB read.
template <int DT>
__global__ __launch_bounds__(256) void colsum8_kernel(const uint16_t* __restrict__ d, int B, int ld, int ncols,
                                                      float* __restrict__ out, float scale) {
  using E = E16<DT>;
  const int cg = threadIdx.x & 7, rl = threadIdx.x >> 3;
  const int c0 = blockIdx.x * 64 + cg * 8;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c0 < ncols) {
    for (int b = rl; b < B; b += 32) {
      const uint4 q = *(const uint4*)(d + (int64_t)b * ld + c0);
      const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) s[e] += E::to_f((uint16_t)(w[e >> 1] >> (16 * (e & 1))));
    }
  }
  __shared__ float red[32][65];
#pragma unroll
  for (int e = 0; e < 8; ++e) red[rl][cg * 8 + e] = s[e];
  __syncthreads();
  if (threadIdx.x < 64) {
    const int c = blockIdx.x * 64 + threadIdx.x;
    float t = 0.f;
#pragma unroll 8
    for (int r = 0; r < 32; ++r) t += red[r][threadIdx.x];
    if (c < ncols) out[c] = scale * t;
  }
}

void colsum_launch(int dtype, const uint16_t* d, int B, int ld, int ncols, float* out, float scale, hipStream_t s) {
  dim3 g((ncols + 63) / 64), b(256);
  if (ncols % 8 == 0 && ld % 8 == 0 && (reinterpret_cast<uintptr_t>(d) & 15) == 0) {
    if (dtype == kBF16)
      hipLaunchKernelGGL(colsum8_kernel<kBF16>, g, b, 0, s, d, B, ld, ncols, out, scale);
    else
      hipLaunchKernelGGL(colsum8_kernel<kF16>, g, b, 0, s, d, B, ld, ncols, out, scale);
    return;
  }
  if (dtype == kBF16)
    hipLaunchKernelGGL(colsum_kernel<kBF16>, g, b, 0, s, d, B, ld, ncols, out, scale);
  else
    hipLaunchKernelGGL(colsum_kernel<kF16>, g, b, 0, s, d, B, ld, ncols, out, scale);
}

}  // namespace pdt
