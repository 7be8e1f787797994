// Pooling kernels, NHWC 16-bit.
//   * bn_relu_maxpool3x3s2: the ResNet stem's BN-apply + ReLU fused with MaxPool(3, 2, 1) (also AlexNet's bias +
//     ReLU + MaxPool(3, 2), pad 0); the full-resolution post-ReLU tensor is never written.  The window argmax (0..8)
//     is kept as uint8.
//   * maxpool_bwd_relu: gather form of the max-pool backward (each input pixel collects from the
//     <= 4 windows that selected it) fused with the ReLU mask recomputed from the BN input.
//   * stem_pool_bwd_reduce / stem_pool_bwd_apply: the whole stem backward (max-pool backward, ReLU
//     mask, BatchNorm backward) in two passes with no 112x112 intermediate: the reduce pass visits
//     only the selected (argmax) elements through the pooled tensor; the apply pass gathers dz for
//     each input pixel and writes dy = A*dz + B*y + C directly (SURVEY K9 + K7/K8 fused).
//   * avgpool (global, HxW -> 1) forward and backward.
#include "../common.h"
#include "conv_fwd.h"
#include "pool.h"

namespace pdt {

static int ew_blocks(int64_t n) {
  int64_t b = (n + 255) / 256;
  if (b > 16384) b = 16384;
  return (int)(b < 1 ? 1 : b);
}

template <int DT>
__global__ __launch_bounds__(256) void bn_relu_maxpool_kernel(const uint16_t* __restrict__ y, const float* __restrict__ coef,
                                                              uint16_t* __restrict__ out, uint8_t* __restrict__ idx,
                                                              int N, int H, int W, int C, int OH, int OW, int pad) {
  using E = E16<DT>;
  const int cv = C / 8;
  const uint32_t total = (uint32_t)N * OH * OW * cv;  // 32-bit index math (host checks sizes < 2^32)
  for (uint32_t v = blockIdx.x * 256u + threadIdx.x; v < total; v += gridDim.x * 256u) {
    const uint32_t pixv = v / cv;
    const int c0 = (int)(v - pixv * cv) * 8;
    const int ow = (int)(pixv % OW);
    const uint32_t t = pixv / OW;
    const int oh = (int)(t % OH);
    const int n = (int)(t / OH);
    float best[8];
    int bi[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { best[e] = -1.f; bi[e] = 0; }
    float sc[8], sh[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { sc[e] = coef[c0 + e]; sh[e] = coef[C + c0 + e]; }
    // all 9 window loads issued up front (branch-free: an out-of-image tap reads the clamped in-image pixel
    // and is then ignored), so a thread pays one memory latency instead of one per in-bounds tap
    uint4 q[9];
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int h = min(max(oh * 2 - pad + kh, 0), H - 1), w = min(max(ow * 2 - pad + kw, 0), W - 1);
        q[kh * 3 + kw] = *(const uint4*)(y + ((uint32_t)(n * H + h) * W + w) * C + c0);
      }
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const bool hok = (unsigned)(oh * 2 - pad + kh) < (unsigned)H;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const bool ok = hok && (unsigned)(ow * 2 - pad + kw) < (unsigned)W;
        const uint32_t qw[4] = {q[kh * 3 + kw].x, q[kh * 3 + kw].y, q[kh * 3 + kw].z, q[kh * 3 + kw].w};
        // branch-free running max (the conditional update had compiled to 72 divergent branches per thread)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float val = fmaxf(E::to_f((uint16_t)(qw[e >> 1] >> (16 * (e & 1)))) * sc[e] + sh[e], 0.f);
          const bool take = ok & (val > best[e]);
          best[e] = take ? val : best[e];
          bi[e] = take ? kh * 3 + kw : bi[e];
        }
      }
    }
    uint32_t ow_[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) ow_[e] = (uint32_t)E::from_f(best[2 * e]) | ((uint32_t)E::from_f(best[2 * e + 1]) << 16);
    const uint32_t o = pixv * C + c0;
    *(uint4*)(out + o) = make_uint4(ow_[0], ow_[1], ow_[2], ow_[3]);
    // a window whose maximum is the ReLU's zero passes no gradient (the ReLU mask at its argmax is 0): its index
    // is the dead marker 255, which no window position matches -- the backward kernels route nothing from it, and
    // the fused stem weight gradients need no per-pixel ReLU mask
#pragma unroll
    for (int e = 0; e < 8; ++e) bi[e] = best[e] > 0.f ? bi[e] : 0xff;
    uint2 ib;
    ib.x = (uint32_t)bi[0] | ((uint32_t)bi[1] << 8) | ((uint32_t)bi[2] << 16) | ((uint32_t)bi[3] << 24);
    ib.y = (uint32_t)bi[4] | ((uint32_t)bi[5] << 8) | ((uint32_t)bi[6] << 16) | ((uint32_t)bi[7] << 24);
    *(uint2*)(idx + o) = ib;
  }
}

// (Round 5: a row-pair variant -- one block per pooled row, a thread per two adjacent outputs sharing their middle
// window column, 15 loads for 2 outputs, no index divisions -- measured SLOWER on the same box: ResNet-18
// 20.16 -> 20.24 ms, ResNet-50 71.7 -> 72.0 ms; not kept.)
// eval / generic variant without index output is the same kernel with idx == nullptr handled by caller
// pad: 1 = the ResNet stem's MaxPool(3, 2, 1); 0 = AlexNet's MaxPool(3, 2)
void bn_relu_maxpool_launch(int dtype, const uint16_t* y, const float* coef, uint16_t* out, uint8_t* idx, int N, int H,
                            int W, int C, hipStream_t s, int pad) {
  const int OH = (H + 2 * pad - 3) / 2 + 1, OW = (W + 2 * pad - 3) / 2 + 1;
  const int64_t total = (int64_t)N * OH * OW * (C / 8);
  if (dtype == kBF16)
    hipLaunchKernelGGL(bn_relu_maxpool_kernel<kBF16>, dim3(ew_blocks(total)), dim3(256), 0, s, y, coef, out, idx, N, H, W,
                       C, OH, OW, pad);
  else
    hipLaunchKernelGGL(bn_relu_maxpool_kernel<kF16>, dim3(ew_blocks(total)), dim3(256), 0, s, y, coef, out, idx, N, H, W,
                       C, OH, OW, pad);
}

template <int DT>
__global__ __launch_bounds__(256) void maxpool_bwd_relu_kernel(const uint16_t* __restrict__ dp, const uint8_t* __restrict__ idx,
                                                               const uint16_t* __restrict__ y, const float* __restrict__ coef,
                                                               uint16_t* __restrict__ dz, int N, int H, int W, int C,
                                                               int OH, int OW, int pad) {
  using E = E16<DT>;
  const int cv = C / 8;
  const int64_t total = (int64_t)N * H * W * cv;
  for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < total; v += (int64_t)gridDim.x * 256) {
    const int c0 = (int)(v % cv) * 8;
    int64_t pix = v / cv;
    const int w = (int)(pix % W);
    pix /= W;
    const int h = (int)(pix % H);
    const int n = (int)(pix / H);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    // candidate windows: oh with 2*oh-pad <= h <= 2*oh-pad+2, i.e. (h+pad)/2 and the one before it
    const int oh_hi = (h + pad) >> 1, ow_hi = (w + pad) >> 1;
    for (int oh = oh_hi - 1; oh <= oh_hi; ++oh) {
      if (oh < 0 || oh >= OH) continue;
      const int kh = h - (oh * 2 - pad);
      if (kh < 0 || kh > 2) continue;
      for (int ow = ow_hi - 1; ow <= ow_hi; ++ow) {
        if (ow < 0 || ow >= OW) continue;
        const int kw = w - (ow * 2 - pad);
        if (kw < 0 || kw > 2) continue;
        const uint8_t pos = (uint8_t)(kh * 3 + kw);
        const int64_t o = (((int64_t)n * OH + oh) * OW + ow) * C + c0;
        const uint2 ib = *(const uint2*)(idx + o);
        const uint4 g = *(const uint4*)(dp + o);
        const uint32_t gw[4] = {g.x, g.y, g.z, g.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const uint8_t b = (uint8_t)(((e < 4) ? ib.x : ib.y) >> (8 * (e & 3)));
          acc[e] += b == pos ? E::to_f((uint16_t)(gw[e >> 1] >> (16 * (e & 1)))) : 0.f;
        }
      }
    }
    const int64_t i = (((int64_t)n * H + h) * W + w) * C + c0;
    const uint4 yy = *(const uint4*)(y + i);
    const uint32_t yw[4] = {yy.x, yy.y, yy.z, yy.w};
    uint32_t o_[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      uint16_t r[2];
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int c = c0 + 2 * e + hh;
        const float pre = E::to_f((uint16_t)(yw[e] >> (16 * hh))) * coef[c] + coef[C + c];
        r[hh] = E::from_f(pre > 0.f ? acc[2 * e + hh] : 0.f);
      }
      o_[e] = (uint32_t)r[0] | ((uint32_t)r[1] << 16);
    }
    *(uint4*)(dz + i) = make_uint4(o_[0], o_[1], o_[2], o_[3]);
  }
}

void maxpool_bwd_relu_launch(int dtype, const uint16_t* dp, const uint8_t* idx, const uint16_t* y, const float* coef,
                             uint16_t* dz, int N, int H, int W, int C, hipStream_t s, int pad) {
  const int OH = (H + 2 * pad - 3) / 2 + 1, OW = (W + 2 * pad - 3) / 2 + 1;
  const int64_t total = (int64_t)N * H * W * (C / 8);
  if (dtype == kBF16)
    hipLaunchKernelGGL(maxpool_bwd_relu_kernel<kBF16>, dim3(ew_blocks(total)), dim3(256), 0, s, dp, idx, y, coef, dz, N, H,
                       W, C, OH, OW, pad);
  else
    hipLaunchKernelGGL(maxpool_bwd_relu_kernel<kF16>, dim3(ew_blocks(total)), dim3(256), 0, s, dp, idx, y, coef, dz, N, H,
                       W, C, OH, OW, pad);
}

// Stem backward, pass 1: per-channel sum(dz) and sum(dz * xhat) over the stem's conv output, visiting
// only the elements each pooling window selected.  dz at an input element is the sum of the pooled
// gradients of the windows that chose it, masked by ReLU; the sums are linear in dz, so they are
// accumulated per window (no 112x112 dz tensor).  One thread per (pooled pixel, 8 channels).
template <int DT>
__global__ __launch_bounds__(256) void stem_pool_bwd_reduce_kernel(const uint16_t* __restrict__ dp,
                                                                   const uint8_t* __restrict__ idx,
                                                                   const uint16_t* __restrict__ y,
                                                                   const float* __restrict__ coef,
                                                                   float* __restrict__ srows, int N, int H, int W,
                                                                   int C, int OH, int OW) {
  using E = E16<DT>;
  const int vpr = C / 8;
  const int rpi = 256 / vpr;
  const int cv = threadIdx.x % vpr, rl = threadIdx.x / vpr;
  const int c0 = cv * 8;
  float sc[8], sh[8], mu[8], is[8], s0[8], s1[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    sc[e] = coef[c0 + e];
    sh[e] = coef[C + c0 + e];
    mu[e] = coef[2 * C + c0 + e];
    is[e] = coef[3 * C + c0 + e];
    s0[e] = 0.f;
    s1[e] = 0.f;
  }
  const int64_t rows = (int64_t)N * OH * OW;
  if (rl < rpi) {
    for (int64_t r = (int64_t)blockIdx.x * rpi + rl; r < rows; r += (int64_t)gridDim.x * rpi) {
      const int ow = (int)(r % OW);
      const int64_t t = r / OW;
      const int oh = (int)(t % OH);
      const int n = (int)(t / OH);
      const int64_t o = r * C + c0;
      const uint2 ib = *(const uint2*)(idx + o);
      const uint4 g = *(const uint4*)(dp + o);
      const uint32_t gw[4] = {g.x, g.y, g.z, g.w};
      const uint16_t* ybase = y + ((int64_t)n * H * W) * C + c0;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int pos0 = (int)((((e < 4) ? ib.x : ib.y) >> (8 * (e & 3))) & 0xff);
        // a dead window (255: its maximum is the ReLU's zero) passes nothing; it reads the always-inside centre tap
        const bool live = pos0 < 9;
        const int pos = live ? pos0 : 4;
        const int kh = pos / 3, kw = pos - 3 * (pos / 3);
        const int h = oh * 2 - 1 + kh, w = ow * 2 - 1 + kw;  // always inside (argmax is a valid tap)
        const float yv = E::to_f(ybase[((int64_t)h * W + w) * C + e]);
        const float dz =
            (live && yv * sc[e] + sh[e] > 0.f) ? E::to_f((uint16_t)(gw[e >> 1] >> (16 * (e & 1)))) : 0.f;
        s0[e] += dz;
        s1[e] += dz * (yv - mu[e]) * is[e];
      }
    }
  }
  extern __shared__ float red[];  // [rpi][C][2]
  if (rl < rpi) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[((int64_t)rl * C + c0 + e) * 2 + 0] = s0[e];
      red[((int64_t)rl * C + c0 + e) * 2 + 1] = s1[e];
    }
  }
  __syncthreads();
  float* dst = srows + (int64_t)blockIdx.x * C * 2;  // this block's own partial row (conv_fwd.h)
  for (int i = threadIdx.x; i < C * 2; i += 256) {
    float t = 0.f;
    for (int q = 0; q < rpi; ++q) t += red[(int64_t)q * C * 2 + i];
    dst[i] = t;
  }
}

void stem_pool_bwd_reduce_launch(int dtype, const uint16_t* dp, const uint8_t* idx, const uint16_t* y,
                                 const float* coef, double* slots, int N, int H, int W, int C, hipStream_t s) {
  const int OH = (H + 2 - 3) / 2 + 1, OW = (W + 2 - 3) / 2 + 1;
  const int rpi = 256 / (C / 8);
  int64_t blocks = ((int64_t)N * OH * OW + rpi * 8 - 1) / (rpi * 8);
  if (blocks > 4096) blocks = 4096;
  const size_t smem = (size_t)rpi * C * 2 * sizeof(float);
  Scratch part((size_t)blocks * C * 2 * sizeof(float), s);
  float* srows = part.as<float>();
  if (dtype == kBF16)
    hipLaunchKernelGGL(stem_pool_bwd_reduce_kernel<kBF16>, dim3((int)blocks), dim3(256), smem, s, dp, idx, y, coef, srows,
                       N, H, W, C, OH, OW);
  else
    hipLaunchKernelGGL(stem_pool_bwd_reduce_kernel<kF16>, dim3((int)blocks), dim3(256), smem, s, dp, idx, y, coef, srows,
                       N, H, W, C, OH, OW);
  stat_rows_reduce_launch(srows, (int)blocks, C * 2, slots, s);
}

// Stem backward, pass 1 without touching the 112x112 tensor: the pooled output IS relu(scale*y + shift)
// at the window's argmax, so the ReLU mask is (out > 0) and the BatchNorm input there is recovered as
// y = (out - shift) / scale, xhat = (y - mean) * invstd -- the sums need only the two pooled-resolution
// tensors (dp, out: 2 x 0.48 GB at ResNet-18 B=1200) instead of a gather from the 1.9 GB conv output.
// (scale == 0, i.e. gamma == 0, contributes xhat = 0.)  One thread per (pooled pixel, 8 channels).
template <int DT>
__global__ __launch_bounds__(256) void stem_pool_bwd_reduce_out_kernel(const uint16_t* __restrict__ dp,
                                                                       const uint16_t* __restrict__ out,
                                                                       const float* __restrict__ coef,
                                                                       float* __restrict__ srows, int64_t rows,
                                                                       int C) {
  using E = E16<DT>;
  const int vpr = C / 8;
  const int rpi = 256 / vpr;
  const int cv = threadIdx.x % vpr, rl = threadIdx.x / vpr;
  const int c0 = cv * 8;
  float rsc[8], sh[8], mu[8], is[8], s0[8], s1[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float sc = coef[c0 + e];
    rsc[e] = sc != 0.f ? 1.f / sc : 0.f;
    sh[e] = coef[C + c0 + e];
    mu[e] = coef[2 * C + c0 + e];
    is[e] = coef[3 * C + c0 + e];
    s0[e] = 0.f;
    s1[e] = 0.f;
  }
  if (rl < rpi) {
    for (int64_t r = (int64_t)blockIdx.x * rpi + rl; r < rows; r += (int64_t)gridDim.x * rpi) {
      const int64_t o = r * C + c0;
      const uint4 g = *(const uint4*)(dp + o);
      const uint4 q = *(const uint4*)(out + o);
      const uint32_t gw[4] = {g.x, g.y, g.z, g.w}, qw[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float ov = E::to_f((uint16_t)(qw[e >> 1] >> (16 * (e & 1))));
        const float dz = ov > 0.f ? E::to_f((uint16_t)(gw[e >> 1] >> (16 * (e & 1)))) : 0.f;
        const float xhat = rsc[e] != 0.f ? ((ov - sh[e]) * rsc[e] - mu[e]) * is[e] : 0.f;
        s0[e] += dz;
        s1[e] += dz * xhat;
      }
    }
  }
  extern __shared__ float red[];  // [rpi][C][2]
  if (rl < rpi) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[((int64_t)rl * C + c0 + e) * 2 + 0] = s0[e];
      red[((int64_t)rl * C + c0 + e) * 2 + 1] = s1[e];
    }
  }
  __syncthreads();
  float* dst = srows + (int64_t)blockIdx.x * C * 2;  // this block's own partial row (conv_fwd.h)
  for (int i = threadIdx.x; i < C * 2; i += 256) {
    float t = 0.f;
    for (int q = 0; q < rpi; ++q) t += red[(int64_t)q * C * 2 + i];
    dst[i] = t;
  }
}

void stem_pool_bwd_reduce_out_launch(int dtype, const uint16_t* dp, const uint16_t* out, const float* coef,
                                     double* slots, int N, int H, int W, int C, hipStream_t s) {
  const int OH = (H + 2 - 3) / 2 + 1, OW = (W + 2 - 3) / 2 + 1;
  pooled_bwd_reduce_launch(dtype, dp, out, coef, slots, (int64_t)N * OH * OW, C, s);
}

// the same sums for any max-pool whose output is relu(BN(y)) at the argmax (the VGG 2x2 pools too): only the pooled
// gradient and the pooled output are read, ``rows`` pooled pixels
void pooled_bwd_reduce_launch(int dtype, const uint16_t* dp, const uint16_t* out, const float* coef, double* slots,
                              int64_t rows, int C, hipStream_t s) {
  const int rpi = 256 / (C / 8);
  int64_t blocks = (rows + rpi * 8 - 1) / (rpi * 8);
  if (blocks > 2048) blocks = 2048;
  const size_t smem = (size_t)rpi * C * 2 * sizeof(float);
  Scratch part((size_t)blocks * C * 2 * sizeof(float), s);
  float* srows = part.as<float>();
  if (dtype == kBF16)
    hipLaunchKernelGGL(stem_pool_bwd_reduce_out_kernel<kBF16>, dim3((int)blocks), dim3(256), smem, s, dp, out, coef,
                       srows, rows, C);
  else
    hipLaunchKernelGGL(stem_pool_bwd_reduce_out_kernel<kF16>, dim3((int)blocks), dim3(256), smem, s, dp, out, coef,
                       srows, rows, C);
  stat_rows_reduce_launch(srows, (int)blocks, C * 2, slots, s);
}

// Stem backward, pass 2: dy = A*dz + B*y + Cc at every conv-output element, with dz gathered from the
// pooling windows that selected it and masked by ReLU (recomputed from y and the BN coefficients).
// One thread per (pooled pixel (oh, ow), 8 channels) owns the 2x2 input block (2oh..2oh+1, 2ow..2ow+1):
// exactly the windows (oh|oh+1, ow|ow+1) can select into it, so each window's argmax/gradient is read by
// 4 threads (not 9) and all index math is 32-bit.
template <int DT>
__global__ __launch_bounds__(256) void stem_pool_bwd_apply_kernel(const uint16_t* __restrict__ dp,
                                                                  const uint8_t* __restrict__ idx,
                                                                  const uint16_t* __restrict__ y,
                                                                  const float* __restrict__ coef,
                                                                  const float* __restrict__ bcoef,
                                                                  uint16_t* __restrict__ dy, int N, int H, int W,
                                                                  int C, int OH, int OW) {
  using E = E16<DT>;
  const int cv = C / 8;
  const uint32_t total = (uint32_t)N * OH * OW * cv;
  for (uint32_t v = blockIdx.x * 256u + threadIdx.x; v < total; v += gridDim.x * 256u) {
    const uint32_t pix = v / cv;
    const int c0 = (int)(v - pix * cv) * 8;
    const uint32_t ow = pix % OW, t = pix / OW;
    const uint32_t oh = t % OH, n = t / OH;
    float acc[2][2][8];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[a][b][e] = 0.f;
#pragma unroll
    for (int dh = 0; dh < 2; ++dh)
#pragma unroll
      for (int dw = 0; dw < 2; ++dw) {
        const uint32_t wh = oh + dh, ww = ow + dw;
        if (wh >= (uint32_t)OH || ww >= (uint32_t)OW) continue;
        const uint32_t o = ((n * OH + wh) * OW + ww) * C + c0;
        const uint2 ib = *(const uint2*)(idx + o);
        const uint4 g = *(const uint4*)(dp + o);
        const uint32_t gw[4] = {g.x, g.y, g.z, g.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int pos = (int)((((e < 4) ? ib.x : ib.y) >> (8 * (e & 3))) & 0xffu);
          const int kh = pos / 3, kw = pos - 3 * (pos / 3);
          // selected input (2wh-1+kh, 2ww-1+kw) relative to this block's corner (2oh, 2ow)
          const int rh = 2 * dh - 1 + kh, rw = 2 * dw - 1 + kw;
          const float gv = E::to_f((uint16_t)(gw[e >> 1] >> (16 * (e & 1))));
#pragma unroll
          for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b)
              if (rh == a && rw == b) acc[a][b][e] += gv;
        }
      }
    float A[8], B[8], Cc[8], sc[8], sh[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      A[e] = bcoef[c0 + e]; B[e] = bcoef[C + c0 + e]; Cc[e] = bcoef[2 * C + c0 + e];
      sc[e] = coef[c0 + e]; sh[e] = coef[C + c0 + e];
    }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const uint32_t h = 2 * oh + a, w = 2 * ow + b;
        if (h >= (uint32_t)H || w >= (uint32_t)W) continue;
        const uint32_t i = ((n * H + h) * W + w) * C + c0;
        const uint4 yy = *(const uint4*)(y + i);
        const uint32_t yw[4] = {yy.x, yy.y, yy.z, yy.w};
        uint32_t o_[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          uint16_t r[2];
#pragma unroll
          for (int hh = 0; hh < 2; ++hh) {
            const int c = 2 * e + hh;
            const float yv = E::to_f((uint16_t)(yw[e] >> (16 * hh)));
            const float dz = yv * sc[c] + sh[c] > 0.f ? acc[a][b][c] : 0.f;
            r[hh] = E::from_f(A[c] * dz + B[c] * yv + Cc[c]);
          }
          o_[e] = (uint32_t)r[0] | ((uint32_t)r[1] << 16);
        }
        *(uint4*)(dy + i) = make_uint4(o_[0], o_[1], o_[2], o_[3]);
      }
  }
}

void stem_pool_bwd_apply_launch(int dtype, const uint16_t* dp, const uint8_t* idx, const uint16_t* y,
                                const float* coef, const float* bcoef, uint16_t* dy, int N, int H, int W, int C,
                                hipStream_t s) {
  const int OH = (H + 2 - 3) / 2 + 1, OW = (W + 2 - 3) / 2 + 1;
  const int64_t total = (int64_t)N * OH * OW * (C / 8);
  if (dtype == kBF16)
    hipLaunchKernelGGL(stem_pool_bwd_apply_kernel<kBF16>, dim3(ew_blocks(total)), dim3(256), 0, s, dp, idx, y, coef,
                       bcoef, dy, N, H, W, C, OH, OW);
  else
    hipLaunchKernelGGL(stem_pool_bwd_apply_kernel<kF16>, dim3(ew_blocks(total)), dim3(256), 0, s, dp, idx, y, coef,
                       bcoef, dy, N, H, W, C, OH, OW);
}

// feat[n][c] = mean_{hw} x[n][hw][c]    (one thread per (n, 8 channels))
template <int DT>
__global__ __launch_bounds__(256) void avgpool_fwd_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ feat, int N,
                                                          int HW, int C, int ldf) {
  using E = E16<DT>;
  const int cv = C / 8;
  const int64_t total = (int64_t)N * cv;
  for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < total; v += (int64_t)gridDim.x * 256) {
    const int c0 = (int)(v % cv) * 8;
    const int n = (int)(v / cv);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const uint16_t* p = x + (int64_t)n * HW * C + c0;
    for (int i = 0; i < HW; ++i) {
      const uint4 q = *(const uint4*)(p + (int64_t)i * C);
      const uint32_t qw[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += E::to_f((uint16_t)(qw[e >> 1] >> (16 * (e & 1))));
    }
    const float inv = 1.f / (float)HW;
    uint32_t o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = (uint32_t)E::from_f(acc[2 * e] * inv) | ((uint32_t)E::from_f(acc[2 * e + 1] * inv) << 16);
    *(uint4*)(feat + (int64_t)n * ldf + c0) = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

// g[n][hw][c] = dfeat[n][c] / HW
template <int DT>
__global__ __launch_bounds__(256) void avgpool_bwd_kernel(const uint16_t* __restrict__ dfeat, uint16_t* __restrict__ g, int N,
                                                          int HW, int C, int ldf) {
  using E = E16<DT>;
  const int cv = C / 8;
  const int64_t total = (int64_t)N * HW * cv;
  const float inv = 1.f / (float)HW;
  for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < total; v += (int64_t)gridDim.x * 256) {
    const int c0 = (int)(v % cv) * 8;
    const int n = (int)(v / ((int64_t)cv * HW));
    const uint4 q = *(const uint4*)(dfeat + (int64_t)n * ldf + c0);
    const uint32_t qw[4] = {q.x, q.y, q.z, q.w};
    uint32_t o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float a = E::to_f((uint16_t)(qw[e] & 0xffff)) * inv, b = E::to_f((uint16_t)(qw[e] >> 16)) * inv;
      o[e] = (uint32_t)E::from_f(a) | ((uint32_t)E::from_f(b) << 16);
    }
    *(uint4*)(g + v * 8) = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

void avgpool_fwd_launch(int dtype, const uint16_t* x, uint16_t* feat, int N, int HW, int C, int ldf, hipStream_t s) {
  const int64_t total = (int64_t)N * (C / 8);
  if (dtype == kBF16)
    hipLaunchKernelGGL(avgpool_fwd_kernel<kBF16>, dim3(ew_blocks(total)), dim3(256), 0, s, x, feat, N, HW, C, ldf);
  else
    hipLaunchKernelGGL(avgpool_fwd_kernel<kF16>, dim3(ew_blocks(total)), dim3(256), 0, s, x, feat, N, HW, C, ldf);
}

void avgpool_bwd_launch(int dtype, const uint16_t* dfeat, uint16_t* g, int N, int HW, int C, int ldf, hipStream_t s) {
  const int64_t total = (int64_t)N * HW * (C / 8);
  if (dtype == kBF16)
    hipLaunchKernelGGL(avgpool_bwd_kernel<kBF16>, dim3(ew_blocks(total)), dim3(256), 0, s, dfeat, g, N, HW, C, ldf);
  else
    hipLaunchKernelGGL(avgpool_bwd_kernel<kF16>, dim3(ew_blocks(total)), dim3(256), 0, s, dfeat, g, N, HW, C, ldf);
}

}  // namespace pdt
