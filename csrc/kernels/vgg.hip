// VGG-family kernels (SURVEY §2.2 model registry: `distributed.py:39-40` builds any torchvision constructor; the
// native engine's VGG path, models/executor_vgg.py).  NHWC 16-bit activations, fp32 math, 64-bit element indexing
// (VGG's 224 x 224 x 64 activations pass 2^32 elements at a few hundred images).
//   * bn_relu_maxpool2: the conv's BatchNorm (or bias) + ReLU fused with MaxPool(2, 2): the full-resolution
//     post-ReLU tensor is never written; the window argmax (0..3) is kept as uint8 per pooled element.
//   * maxpool2_bwd: the pooled gradient scattered to each window's argmax, masked by ReLU (out > 0 at the argmax:
//     the pooled value IS relu(pre-activation) there), then -- for a BatchNorm -- dy = A*dz + B*y + C at every
//     conv-output element; for a bias the conv-output gradient is dz itself and y is not read.  The BN-backward
//     sums come from the pooled tensors alone (pool.hip pooled_bwd_reduce_launch).
//   * fc_act: classifier bias + ReLU + Dropout in one pass after the GEMM; dropout keeps an element when a
//     counter-based hash of (seed, element) clears the threshold, and backward recovers the keep mask from the
//     stored output (out > 0 <=> pre-activation > 0 and kept), so no mask tensor exists.
#include "../common.h"
#include "vgg.h"

namespace pdt {

static int vgg_blocks(int64_t n) {
  int64_t b = (n + 255) / 256;
  if (b > 65536) b = 65536;
  return (int)(b < 1 ? 1 : b);
}

template <int DT>
__global__ __launch_bounds__(256) void bn_relu_maxpool2_kernel(const uint16_t* __restrict__ y,
                                                               const float* __restrict__ coef,
                                                               uint16_t* __restrict__ out, uint8_t* __restrict__ idx,
                                                               int64_t total, int W, int C, int OH, int OW) {
  using E = E16<DT>;
  const int cv = C / 8;
  for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < total; v += (int64_t)gridDim.x * 256) {
    const int64_t pix = v / cv;
    const int c0 = (int)(v - pix * cv) * 8;
    const int ow = (int)(pix % OW);
    const int64_t t = pix / OW;
    const int oh = (int)(t % OH);
    const int64_t n = t / OH;
    float sc[8], sh[8], best[8];
    uint32_t bi[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      sc[e] = coef[c0 + e];
      sh[e] = coef[C + c0 + e];
      best[e] = -1.f;
      bi[e] = 0;
    }
    const int64_t H = 2 * (int64_t)OH;
    uint4 q[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      q[k] = *(const uint4*)(y + (((n * H + 2 * oh + (k >> 1)) * W + 2 * ow + (k & 1)) * C + c0));
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t qw[4] = {q[k].x, q[k].y, q[k].z, q[k].w};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float val = fmaxf(E::to_f((uint16_t)(qw[e >> 1] >> (16 * (e & 1)))) * sc[e] + sh[e], 0.f);
        if (val > best[e]) { best[e] = val; bi[e] = (uint32_t)k; }
      }
    }
    uint32_t o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = (uint32_t)E::from_f(best[2 * e]) | ((uint32_t)E::from_f(best[2 * e + 1]) << 16);
    const int64_t oo = pix * C + c0;
    *(uint4*)(out + oo) = make_uint4(o[0], o[1], o[2], o[3]);
    if (idx != nullptr)
      *(uint2*)(idx + oo) = make_uint2(bi[0] | (bi[1] << 8) | (bi[2] << 16) | (bi[3] << 24),
                                       bi[4] | (bi[5] << 8) | (bi[6] << 16) | (bi[7] << 24));
  }
}

void bn_relu_maxpool2_launch(int dtype, const uint16_t* y, const float* coef, uint16_t* out, uint8_t* idx, int64_t N,
                             int H, int W, int C, hipStream_t s) {
  const int OH = H / 2, OW = W / 2;
  const int64_t total = N * OH * OW * (C / 8);
  if (total == 0) return;
  if (dtype == kBF16)
    hipLaunchKernelGGL(bn_relu_maxpool2_kernel<kBF16>, dim3(vgg_blocks(total)), dim3(256), 0, s, y, coef, out, idx,
                       total, W, C, OH, OW);
  else
    hipLaunchKernelGGL(bn_relu_maxpool2_kernel<kF16>, dim3(vgg_blocks(total)), dim3(256), 0, s, y, coef, out, idx,
                       total, W, C, OH, OW);
}

// One thread per (pooled pixel, 8 channels) owns that window's 2 x 2 conv-output block: every conv-output element is
// written exactly once (stride-2, size-2 windows do not overlap; H and W are even).
template <int DT, bool BN>
__global__ __launch_bounds__(256) void maxpool2_bwd_kernel(const uint16_t* __restrict__ dp,
                                                           const uint8_t* __restrict__ idx,
                                                           const uint16_t* __restrict__ out,
                                                           const uint16_t* __restrict__ y,
                                                           const float* __restrict__ bcoef,
                                                           uint16_t* __restrict__ dy, int64_t total, int W, int C,
                                                           int OH, int OW) {
  using E = E16<DT>;
  const int cv = C / 8;
  for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < total; v += (int64_t)gridDim.x * 256) {
    const int64_t pix = v / cv;
    const int c0 = (int)(v - pix * cv) * 8;
    const int ow = (int)(pix % OW);
    const int64_t t = pix / OW;
    const int oh = (int)(t % OH);
    const int64_t n = t / OH;
    const int64_t oo = pix * C + c0;
    const uint2 ib = *(const uint2*)(idx + oo);
    const uint4 g = *(const uint4*)(dp + oo);
    const uint4 q = *(const uint4*)(out + oo);
    const uint32_t gw[4] = {g.x, g.y, g.z, g.w}, qw[4] = {q.x, q.y, q.z, q.w};
    float gz[8];
    int pos[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float ov = E::to_f((uint16_t)(qw[e >> 1] >> (16 * (e & 1))));
      gz[e] = ov > 0.f ? E::to_f((uint16_t)(gw[e >> 1] >> (16 * (e & 1)))) : 0.f;
      pos[e] = (int)((((e < 4) ? ib.x : ib.y) >> (8 * (e & 3))) & 3u);
    }
    float A[8], B[8], Cc[8];
    if constexpr (BN) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        A[e] = bcoef[c0 + e];
        B[e] = bcoef[C + c0 + e];
        Cc[e] = bcoef[2 * C + c0 + e];
      }
    }
    const int64_t H = 2 * (int64_t)OH;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t i = ((n * H + 2 * oh + (k >> 1)) * W + 2 * ow + (k & 1)) * C + c0;
      uint32_t yw[4] = {0u, 0u, 0u, 0u};
      if constexpr (BN) {
        const uint4 yy = *(const uint4*)(y + i);
        yw[0] = yy.x; yw[1] = yy.y; yw[2] = yy.z; yw[3] = yy.w;
      }
      uint32_t o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        uint32_t r[2];
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          const int c = 2 * e + hh;
          const float dz = pos[c] == k ? gz[c] : 0.f;
          float val = dz;
          if constexpr (BN) val = A[c] * dz + B[c] * E::to_f((uint16_t)(yw[e] >> (16 * hh))) + Cc[c];
          r[hh] = (uint32_t)E::from_f(val);
        }
        o[e] = r[0] | (r[1] << 16);
      }
      *(uint4*)(dy + i) = make_uint4(o[0], o[1], o[2], o[3]);
    }
  }
}

void maxpool2_bwd_launch(int dtype, const uint16_t* dp, const uint8_t* idx, const uint16_t* out, const uint16_t* y,
                         const float* bcoef, uint16_t* dy, int64_t N, int H, int W, int C, hipStream_t s) {
  const int OH = H / 2, OW = W / 2;
  const int64_t total = N * OH * OW * (C / 8);
  if (total == 0) return;
  const dim3 g(vgg_blocks(total)), b(256);
  if (bcoef != nullptr) {
    if (dtype == kBF16)
      hipLaunchKernelGGL((maxpool2_bwd_kernel<kBF16, true>), g, b, 0, s, dp, idx, out, y, bcoef, dy, total, W, C, OH, OW);
    else
      hipLaunchKernelGGL((maxpool2_bwd_kernel<kF16, true>), g, b, 0, s, dp, idx, out, y, bcoef, dy, total, W, C, OH, OW);
  } else {
    if (dtype == kBF16)
      hipLaunchKernelGGL((maxpool2_bwd_kernel<kBF16, false>), g, b, 0, s, dp, idx, out, y, bcoef, dy, total, W, C, OH,
                         OW);
    else
      hipLaunchKernelGGL((maxpool2_bwd_kernel<kF16, false>), g, b, 0, s, dp, idx, out, y, bcoef, dy, total, W, C, OH,
                         OW);
  }
}

// counter-based keep decision: a 32-bit mix of (seed, element index); deterministic for a given seed / step
PDT_DEVICE uint32_t vgg_hash(uint64_t seed, uint64_t i) {
  uint64_t z = seed + 0x9E3779B97F4A7C15ull * (i + 1);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return (uint32_t)((z ^ (z >> 31)) >> 32);
}

// out[r][f] = dropout(relu(z[r][f] + bias[f])), 8 features per thread; keep_thr = 0: no dropout (eval, p = 0)
template <int DT>
__global__ __launch_bounds__(256) void fc_act_fwd_kernel(const uint16_t* __restrict__ z, const float* __restrict__ bias,
                                                         uint16_t* __restrict__ out, int64_t total, int F,
                                                         uint32_t keep_thr, float scale, uint64_t seed) {
  using E = E16<DT>;
  const int fv = F / 8;
  for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < total; v += (int64_t)gridDim.x * 256) {
    const int f0 = (int)(v % fv) * 8;
    const uint4 q = *(const uint4*)(z + v * 8);
    const uint32_t qw[4] = {q.x, q.y, q.z, q.w};
    uint32_t o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      uint32_t r[2];
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int k = 2 * e + hh;
        float val = fmaxf(E::to_f((uint16_t)(qw[e] >> (16 * hh))) + bias[f0 + k], 0.f);
        if (keep_thr != 0u) val = vgg_hash(seed, (uint64_t)(v * 8 + k)) >= keep_thr ? val * scale : 0.f;
        r[hh] = (uint32_t)E::from_f(val);
      }
      o[e] = r[0] | (r[1] << 16);
    }
    *(uint4*)(out + v * 8) = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

void fc_act_fwd_launch(int dtype, const uint16_t* z, const float* bias, uint16_t* out, int64_t rows, int F, double p,
                       uint64_t seed, hipStream_t s) {
  const int64_t total = rows * (F / 8);
  if (total == 0) return;
  uint32_t thr = 0u;
  float scale = 1.f;
  if (p > 0.0) {
    const double t = p * 4294967296.0;
    thr = t >= 4294967295.0 ? 0xffffffffu : (uint32_t)t;
    if (thr == 0u) thr = 1u;
    scale = (float)(1.0 / (1.0 - p));
  }
  if (dtype == kBF16)
    hipLaunchKernelGGL(fc_act_fwd_kernel<kBF16>, dim3(vgg_blocks(total)), dim3(256), 0, s, z, bias, out, total, F, thr,
                       scale, seed);
  else
    hipLaunchKernelGGL(fc_act_fwd_kernel<kF16>, dim3(vgg_blocks(total)), dim3(256), 0, s, z, bias, out, total, F, thr,
                       scale, seed);
}

// dz = (out > 0) ? dh * scale : 0  -- out > 0 exactly where the pre-activation was positive and the element kept
template <int DT>
__global__ __launch_bounds__(256) void fc_act_bwd_kernel(const uint16_t* __restrict__ dh, const uint16_t* __restrict__ out,
                                                         uint16_t* __restrict__ dz, int64_t total, float scale) {
  using E = E16<DT>;
  for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < total; v += (int64_t)gridDim.x * 256) {
    const uint4 g = *(const uint4*)(dh + v * 8);
    const uint4 q = *(const uint4*)(out + v * 8);
    const uint32_t gw[4] = {g.x, g.y, g.z, g.w}, qw[4] = {q.x, q.y, q.z, q.w};
    uint32_t o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      uint32_t r[2];
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const bool on = E::to_f((uint16_t)(qw[e] >> (16 * hh))) > 0.f;
        r[hh] = (uint32_t)E::from_f(on ? E::to_f((uint16_t)(gw[e] >> (16 * hh))) * scale : 0.f);
      }
      o[e] = r[0] | (r[1] << 16);
    }
    *(uint4*)(dz + v * 8) = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

void fc_act_bwd_launch(int dtype, const uint16_t* dh, const uint16_t* out, uint16_t* dz, int64_t n, double p,
                       hipStream_t s) {
  const int64_t total = n / 8;
  if (total == 0) return;
  const float scale = p > 0.0 ? (float)(1.0 / (1.0 - p)) : 1.f;
  if (dtype == kBF16)
    hipLaunchKernelGGL(fc_act_bwd_kernel<kBF16>, dim3(vgg_blocks(total)), dim3(256), 0, s, dh, out, dz, total, scale);
  else
    hipLaunchKernelGGL(fc_act_bwd_kernel<kF16>, dim3(vgg_blocks(total)), dim3(256), 0, s, dh, out, dz, total, scale);
}

// NHWC [N][HW][C] <-> torchvision's flatten order [N][C][HW] (the classifier's input features)
template <bool TO_NCHW>
__global__ __launch_bounds__(256) void nhwc_nchw16_kernel(const uint16_t* __restrict__ src, uint16_t* __restrict__ dst,
                                                          int64_t total, int HW, int C) {
  for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < total; v += (int64_t)gridDim.x * 256) {
    // v indexes the NHWC element (n, hw, c)
    const int c = (int)(v % C);
    const int64_t t = v / C;
    const int hw = (int)(t % HW);
    const int64_t n = t / HW;
    const int64_t w = (n * C + c) * HW + hw;
    if constexpr (TO_NCHW)
      dst[w] = src[v];
    else
      dst[v] = src[w];
  }
}

void nhwc_nchw16_launch(const uint16_t* src, uint16_t* dst, int64_t N, int HW, int C, bool to_nchw, hipStream_t s) {
  const int64_t total = N * HW * C;
  if (total == 0) return;
  if (to_nchw)
    hipLaunchKernelGGL(nhwc_nchw16_kernel<true>, dim3(vgg_blocks(total)), dim3(256), 0, s, src, dst, total, HW, C);
  else
    hipLaunchKernelGGL(nhwc_nchw16_kernel<false>, dim3(vgg_blocks(total)), dim3(256), 0, s, src, dst, total, HW, C);
}

// coef = [1 | bias | 0 | 1]: a conv bias + ReLU expressed as the BatchNorm coefficient block the fused kernels read
// (scale, shift, mean, invstd), so the bias layers run the BN layers' apply / pool / fused dgrad-epilogue kernels
__global__ void bias_coef_kernel(const float* __restrict__ bias, float* __restrict__ coef, int C) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  coef[c] = 1.f;
  coef[C + c] = bias[c];
  coef[2 * C + c] = 0.f;
  coef[3 * C + c] = 1.f;
}

void bias_coef_launch(const float* bias, float* coef, int C, hipStream_t s) {
  hipLaunchKernelGGL(bias_coef_kernel, dim3((C + 255) / 256), dim3(256), 0, s, bias, coef, C);
}

}  // namespace pdt
