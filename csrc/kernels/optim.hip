// Optimizer / AMP / weight-layout kernels.
//
//   * nonfinite_check: GradScaler's found_inf over the flat fp32 gradient buffer (device flag, no
//     host sync).
//   * sgd_fused: torch.optim.SGD semantics (d_p = g + wd*p; buf = d_p on the first step, else
//     momentum*buf + d_p; p -= lr*buf) over the flat fp32 parameter/gradient/momentum buffers, with
//     the gradient pre-scale (1/world for DDP averaging, 1/loss_scale for AMP unscale) folded in,
//     the whole step skipped when found_inf is set, and the 16-bit compute copy of every parameter
//     written in the same pass (no per-forward autocast weight casts).
//   * amp_update_scale: GradScaler's growth/backoff update on device.
//   * gather16: builds every derived weight layout (dgrad tap-transposes, padded stem / fc
//     matrices) from the 16-bit shadow in one launch, driven by a precomputed index map.
#include "../common.h"
#include "optim.h"

namespace pdt {

static int ew_blocks(int64_t n) {
  int64_t b = (n + 255) / 256;
  if (b > 8192) b = 8192;
  return (int)(b < 1 ? 1 : b);
}

__global__ __launch_bounds__(256) void nonfinite_kernel(const float* __restrict__ g, int64_t n, float* __restrict__ found) {
  bool bad = false;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float v = g[i];
    bad |= !isfinite(v);
  }
  if (__any(bad) && (threadIdx.x & 63) == 0) *found = 1.f;
}

void nonfinite_check_launch(const float* g, int64_t n, float* found, hipStream_t s) {
  hipLaunchKernelGGL(nonfinite_kernel, dim3(ew_blocks(n)), dim3(256), 0, s, g, n, found);
}

template <int DT>
__global__ __launch_bounds__(256) void sgd_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                  float* __restrict__ buf, uint16_t* __restrict__ shadow,
                                                  const float* __restrict__ wd_mask, int64_t n, float lr,
                                                  float momentum, float wd, float gscale,
                                                  const float* __restrict__ loss_scale_ptr,
                                                  const float* __restrict__ found_inf, int first) {
  using E = E16<DT>;
  if (found_inf && *found_inf != 0.f) return;
  const float gs = gscale * (loss_scale_ptr ? 1.f / *loss_scale_ptr : 1.f);
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    float pv = p[i];
    float d = g[i] * gs + wd * pv * (wd_mask ? wd_mask[i] : 1.f);
    float b;
    if (momentum != 0.f) {
      b = first ? d : momentum * buf[i] + d;
      buf[i] = b;
    } else {
      b = d;
    }
    pv -= lr * b;
    p[i] = pv;
    if (shadow) shadow[i] = E::from_f(pv);
  }
}

void sgd_launch(int dtype, float* p, const float* g, float* buf, uint16_t* shadow, const float* wd_mask, int64_t n,
                float lr, float momentum, float wd, float gscale, const float* loss_scale, const float* found_inf,
                bool first, hipStream_t s) {
  if (dtype == kBF16)
    hipLaunchKernelGGL(sgd_kernel<kBF16>, dim3(ew_blocks(n)), dim3(256), 0, s, p, g, buf, shadow, wd_mask, n, lr, momentum,
                       wd, gscale, loss_scale, found_inf, (int)first);
  else
    hipLaunchKernelGGL(sgd_kernel<kF16>, dim3(ew_blocks(n)), dim3(256), 0, s, p, g, buf, shadow, wd_mask, n, lr, momentum,
                       wd, gscale, loss_scale, found_inf, (int)first);
}

template <int DT>
__global__ __launch_bounds__(256) void cast16_kernel(const float* __restrict__ p, uint16_t* __restrict__ out, int64_t n) {
  using E = E16<DT>;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) out[i] = E::from_f(p[i]);
}

void cast16_launch(int dtype, const float* p, uint16_t* out, int64_t n, hipStream_t s) {
  if (dtype == kBF16)
    hipLaunchKernelGGL(cast16_kernel<kBF16>, dim3(ew_blocks(n)), dim3(256), 0, s, p, out, n);
  else
    hipLaunchKernelGGL(cast16_kernel<kF16>, dim3(ew_blocks(n)), dim3(256), 0, s, p, out, n);
}

// 16-bit -> fp32 widening (gradient-compression epilogue of the native bucketer: bf16 all-reduce, fp32 grads)
template <int DT>
__global__ __launch_bounds__(256) void widen16_kernel(const uint16_t* __restrict__ in, float* __restrict__ out, int64_t n) {
  using E = E16<DT>;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) out[i] = E::to_f(in[i]);
}

void widen16_launch(int dtype, const uint16_t* in, float* out, int64_t n, hipStream_t s) {
  if (dtype == kBF16)
    hipLaunchKernelGGL(widen16_kernel<kBF16>, dim3(ew_blocks(n)), dim3(256), 0, s, in, out, n);
  else
    hipLaunchKernelGGL(widen16_kernel<kF16>, dim3(ew_blocks(n)), dim3(256), 0, s, in, out, n);
}

// GradScaler._amp_update_scale_: scale *= backoff on inf (tracker = 0), else tracker += 1 and
// scale *= growth when tracker reaches the interval (tracker = 0).  Resets found_inf for the next step.
__global__ void amp_update_kernel(float* scale, int* tracker, float* found_inf, float growth, float backoff,
                                  int interval) {
  if (threadIdx.x != 0) return;
  if (*found_inf != 0.f) {
    *scale = *scale * backoff;
    *tracker = 0;
  } else {
    const int t = *tracker + 1;
    if (t == interval) {
      const float ns = *scale * growth;
      if (isfinite(ns)) *scale = ns;
      *tracker = 0;
    } else {
      *tracker = t;
    }
  }
}

void amp_update_launch(float* scale, int* tracker, float* found_inf, float growth, float backoff, int interval,
                       hipStream_t s) {
  hipLaunchKernelGGL(amp_update_kernel, dim3(1), dim3(64), 0, s, scale, tracker, found_inf, growth, backoff, interval);
}

__global__ __launch_bounds__(256) void gather16_kernel(const uint16_t* __restrict__ src, const int* __restrict__ idx,
                                                       uint16_t* __restrict__ dst, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int j = idx[i];
    dst[i] = j >= 0 ? src[j] : (uint16_t)0;
  }
}

void gather16_launch(const uint16_t* src, const int* idx, uint16_t* dst, int64_t n, hipStream_t s) {
  hipLaunchKernelGGL(gather16_kernel, dim3(ew_blocks(n)), dim3(256), 0, s, src, idx, dst, n);
}

// Stem input: fp32 NCHW image batch -> 16-bit im2col rows [N*OH*OW][ldk], column k = (r*S + s)*C + c
// for k < R*S*C, zero padding beyond (and outside the image).  One thread per 8 columns of a row.
template <int DT>
__global__ __launch_bounds__(256) void im2col_kernel(const float* __restrict__ x, uint16_t* __restrict__ out, int N, int C,
                                                     int H, int W, int R, int S, int stride, int pad, int OH, int OW,
                                                     int ldk) {
  using E = E16<DT>;
  const int kv = ldk / 8;
  const int KK = R * S * C;
  const int64_t total = (int64_t)N * OH * OW * kv;
  for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < total; v += (int64_t)gridDim.x * 256) {
    const int k0 = (int)(v % kv) * 8;
    int64_t pix = v / kv;
    const int ow = (int)(pix % OW);
    pix /= OW;
    const int oh = (int)(pix % OH);
    const int n = (int)(pix / OH);
    uint16_t o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int k = k0 + e;
      float val = 0.f;
      if (k < KK) {
        const int c = k % C;
        const int rs = k / C;
        const int r = rs / S, s = rs - (rs / S) * S;
        const int h = oh * stride - pad + r, w = ow * stride - pad + s;
        if ((unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W) val = x[(((int64_t)n * C + c) * H + h) * W + w];
      }
      o[e] = E::from_f(val);
    }
    uint4 q;
    q.x = (uint32_t)o[0] | ((uint32_t)o[1] << 16);
    q.y = (uint32_t)o[2] | ((uint32_t)o[3] << 16);
    q.z = (uint32_t)o[4] | ((uint32_t)o[5] << 16);
    q.w = (uint32_t)o[6] | ((uint32_t)o[7] << 16);
    *(uint4*)(out + v * 8) = q;
  }
}

void im2col_launch(int dtype, const float* x, uint16_t* out, int N, int C, int H, int W, int R, int S, int stride, int pad,
                   int ldk, hipStream_t s) {
  const int OH = (H + 2 * pad - R) / stride + 1, OW = (W + 2 * pad - S) / stride + 1;
  const int64_t total = (int64_t)N * OH * OW * (ldk / 8);
  if (dtype == kBF16)
    hipLaunchKernelGGL(im2col_kernel<kBF16>, dim3(ew_blocks(total)), dim3(256), 0, s, x, out, N, C, H, W, R, S, stride, pad,
                       OH, OW, ldk);
  else
    hipLaunchKernelGGL(im2col_kernel<kF16>, dim3(ew_blocks(total)), dim3(256), 0, s, x, out, N, C, H, W, R, S, stride, pad,
                       OH, OW, ldk);
}

// Stem input: fp32 NCHW image batch -> zero-padded 16-bit NHWC4 image [N][H+2p][W+2p+ex][4]
// (channel 3 and the border are zero).  The stem conv then reads 8-pixel x 4-channel windows of it
// directly (window mode of conv_fwd / conv_wgrad): no im2col matrix.
// TIN = float: x is already normalised; TIN = uint8_t: raw pixels, v = x * scale[c] + shift[c] (the
// ImageNet Normalize of the data pipeline fused here, so batches cross PCIe as uint8 -- SURVEY K28)
template <int DT, typename TIN>
__global__ __launch_bounds__(256) void stem_pack_kernel(const TIN* __restrict__ x, uint16_t* __restrict__ out, int N,
                                                        int C, int H, int W, int pad, int Hp, int Wp,
                                                        const float* __restrict__ scale,
                                                        const float* __restrict__ shift, FastDiv fwp, FastDiv fhp) {
  using E = E16<DT>;
  // 32-bit index math (the host checks N*Hp*Wp < 2^31): 64-bit div/mod by the padded sizes made this pass
  // ALU-bound at ~3 TB/s
  const uint32_t total = (uint32_t)N * Hp * Wp;
  for (uint32_t v = blockIdx.x * 256u + threadIdx.x; v < total; v += gridDim.x * 256u) {
    const uint32_t t = fdiv(v, fwp);
    const int wp = (int)(v - t * (uint32_t)Wp);
    const int n = (int)fdiv(t, fhp);
    const int hp = (int)(t - (uint32_t)n * (uint32_t)Hp);
    const int h = hp - pad, w = wp - pad;
    uint16_t o[4] = {0, 0, 0, 0};
    if ((unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W) {
      const TIN* px = x + ((size_t)n * C * H + h) * W + w;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        if (c < C) {
          const float v = (float)px[(size_t)c * H * W];
          o[c] = E::from_f(scale ? v * scale[c] + shift[c] : v);
        }
      }
    }
    uint2 q;
    q.x = (uint32_t)o[0] | ((uint32_t)o[1] << 16);
    q.y = (uint32_t)o[2] | ((uint32_t)o[3] << 16);
    *(uint2*)(out + (size_t)v * 4) = q;
  }
}

// Row-tiled fp32 variant (W % 4 == 0, Wp even, C <= 4, 16-B aligned input): a block packs kRows padded rows.
// Every channel row is read with coalesced float4 loads, transposed to pixel-major through LDS, and the padded
// NHWC4 row is written with 16-B stores (two pixels each).  The per-pixel kernel above issues three 4-B loads
// and one 8-B store per pixel and streams ~4.4 TB/s.
template <int DT>
__global__ __launch_bounds__(256) void stem_pack_rows_kernel(const float* __restrict__ x, uint16_t* __restrict__ out,
                                                             int N, int C, int H, int W, int pad, int Hp, int Wp) {
  using E = E16<DT>;
  constexpr int kRows = 4;
  constexpr int kMaxWp = 256;
  __shared__ uint2 tile[kRows][kMaxWp];  // [row][padded pixel] -> 4 channels
  const int rows = N * Hp;
  const int r0 = blockIdx.x * kRows;
  const int W4 = W >> 2;
  // zero-fill (padding pixels, channel 3 and channels >= C)
  for (int i = threadIdx.x; i < kRows * kMaxWp; i += 256) tile[i / kMaxWp][i % kMaxWp] = make_uint2(0u, 0u);
  __syncthreads();
  uint16_t* t16 = (uint16_t*)&tile[0][0];
  for (int i = threadIdx.x; i < kRows * C * W4; i += 256) {
    const int rr = i / (C * W4), rem = i - rr * (C * W4);
    const int c = rem / W4, w4 = rem - c * W4;
    const int r = r0 + rr;
    if (r >= rows) continue;
    const int n = r / Hp, h = r - n * Hp - pad;
    if ((unsigned)h >= (unsigned)H) continue;
    const float4 v = *(const float4*)(x + (((size_t)n * C + c) * H + h) * W + 4 * w4);
    uint16_t* d = t16 + ((size_t)rr * kMaxWp + pad + 4 * w4) * 4 + c;
    d[0] = E::from_f(v.x);
    d[4] = E::from_f(v.y);
    d[8] = E::from_f(v.z);
    d[12] = E::from_f(v.w);
  }
  __syncthreads();
  const int P2 = Wp >> 1;  // 16-B pixel pairs per row
  for (int i = threadIdx.x; i < kRows * P2; i += 256) {
    const int rr = i / P2, pp = i - rr * P2;
    const int r = r0 + rr;
    if (r >= rows) continue;
    const uint2 a = tile[rr][2 * pp], b = tile[rr][2 * pp + 1];
    *(uint4*)(out + ((size_t)r * Wp + 2 * pp) * 4) = make_uint4(a.x, a.y, b.x, b.y);
  }
}

void stem_pack_launch(int dtype, const float* x, uint16_t* out, int N, int C, int H, int W, int pad, int Hp, int Wp,
                      hipStream_t s) {
  if (W % 4 == 0 && Wp % 2 == 0 && Wp <= 256 && C <= 4 && (uintptr_t)x % 16 == 0 && (uintptr_t)out % 16 == 0) {
    const int rows = N * Hp, blocks = (rows + 3) / 4;
    if (dtype == kBF16)
      hipLaunchKernelGGL(stem_pack_rows_kernel<kBF16>, dim3(blocks), dim3(256), 0, s, x, out, N, C, H, W, pad, Hp, Wp);
    else
      hipLaunchKernelGGL(stem_pack_rows_kernel<kF16>, dim3(blocks), dim3(256), 0, s, x, out, N, C, H, W, pad, Hp, Wp);
    return;
  }
  const int64_t total = (int64_t)N * Hp * Wp;
  if (dtype == kBF16)
    hipLaunchKernelGGL((stem_pack_kernel<kBF16, float>), dim3(ew_blocks(total)), dim3(256), 0, s, x, out, N, C, H, W,
                       pad, Hp, Wp, nullptr, nullptr, make_fastdiv((uint32_t)Wp), make_fastdiv((uint32_t)Hp));
  else
    hipLaunchKernelGGL((stem_pack_kernel<kF16, float>), dim3(ew_blocks(total)), dim3(256), 0, s, x, out, N, C, H, W,
                       pad, Hp, Wp, nullptr, nullptr, make_fastdiv((uint32_t)Wp), make_fastdiv((uint32_t)Hp));
}

void stem_pack_u8_launch(int dtype, const uint8_t* x, uint16_t* out, int N, int C, int H, int W, int pad, int Hp,
                         int Wp, const float* scale, const float* shift, hipStream_t s) {
  const int64_t total = (int64_t)N * Hp * Wp;
  if (dtype == kBF16)
    hipLaunchKernelGGL((stem_pack_kernel<kBF16, uint8_t>), dim3(ew_blocks(total)), dim3(256), 0, s, x, out, N, C, H,
                       W, pad, Hp, Wp, scale, shift, make_fastdiv((uint32_t)Wp), make_fastdiv((uint32_t)Hp));
  else
    hipLaunchKernelGGL((stem_pack_kernel<kF16, uint8_t>), dim3(ew_blocks(total)), dim3(256), 0, s, x, out, N, C, H,
                       W, pad, Hp, Wp, scale, shift, make_fastdiv((uint32_t)Wp), make_fastdiv((uint32_t)Hp));
}

__global__ __launch_bounds__(256) void gather32_kernel(const float* __restrict__ src, const int* __restrict__ idx,
                                                       float* __restrict__ dst, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int j = idx[i];
    dst[i] = j >= 0 ? src[j] : 0.f;
  }
}

void gather32_launch(const float* src, const int* idx, float* dst, int64_t n, hipStream_t s) {
  hipLaunchKernelGGL(gather32_kernel, dim3(ew_blocks(n)), dim3(256), 0, s, src, idx, dst, n);
}

// dst[idx[i]] = src[i]: the inverse of gather32 over distinct indices (DataParallel replicas receive the fp32
// values of the parameters the kernels read from the master copy -- BN affine, fc bias -- through a packed buffer)
__global__ __launch_bounds__(256) void scatter32_kernel(const float* __restrict__ src, const int* __restrict__ idx,
                                                        float* __restrict__ dst, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) dst[idx[i]] = src[i];
}

void scatter32_launch(const float* src, const int* idx, float* dst, int64_t n, hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL(scatter32_kernel, dim3(ew_blocks(n)), dim3(256), 0, s, src, idx, dst, n);
}

}  // namespace pdt

namespace pdt {
// ---------------------------------------------------------------------------------------------------------
// Streaming-bandwidth probe (tools/bw_probe.py): out = 0.5 * x + y over n 16-bit elements (6 B per element,
// the shape of the BN apply / backward-apply passes), in variants of bytes in flight per thread, grid size
// and cache policy, to pick the structure of the elementwise kernels.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <int U, bool NT_LD, bool NT_ST>
__global__ __launch_bounds__(256) void bw_probe_kernel(const uint4* __restrict__ x, const uint4* __restrict__ y,
                                                       uint4* __restrict__ out, int64_t n8) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t v0 = (int64_t)blockIdx.x * 256 + threadIdx.x; v0 < n8; v0 += stride * U) {
    uint4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t v = v0 + u * stride;
      if (v < n8) {
        if constexpr (NT_LD) {
          const u32x4 ta = __builtin_nontemporal_load((const u32x4*)(x + v));
          const u32x4 tb = __builtin_nontemporal_load((const u32x4*)(y + v));
          a[u] = make_uint4(ta[0], ta[1], ta[2], ta[3]);
          b[u] = make_uint4(tb[0], tb[1], tb[2], tb[3]);
        } else {
          a[u] = x[v];
          b[u] = y[v];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t v = v0 + u * stride;
      if (v >= n8) continue;
      const uint32_t aw[4] = {a[u].x, a[u].y, a[u].z, a[u].w}, bw[4] = {b[u].x, b[u].y, b[u].z, b[u].w};
      uint32_t o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float l = 0.5f * __uint_as_float(aw[e] << 16) + __uint_as_float(bw[e] << 16);
        const float h = 0.5f * __uint_as_float(aw[e] & 0xffff0000u) + __uint_as_float(bw[e] & 0xffff0000u);
        o[e] = (uint32_t)E16<kBF16>::from_f(l) | ((uint32_t)E16<kBF16>::from_f(h) << 16);
      }
      if constexpr (NT_ST) {
        const u32x4 r = {o[0], o[1], o[2], o[3]};
        __builtin_nontemporal_store(r, (u32x4*)(out + v));
      } else {
        out[v] = make_uint4(o[0], o[1], o[2], o[3]);
      }
    }
  }
}

void bw_probe_launch(int mode, const uint16_t* x, const uint16_t* y, uint16_t* out, int64_t n, int blocks,
                     hipStream_t s) {
  const int64_t n8 = n / 8;
  const uint4 *a = (const uint4*)x, *b = (const uint4*)y;
  uint4* o = (uint4*)out;
  dim3 g(blocks), bl(256);
  switch (mode) {
    case 0: hipLaunchKernelGGL((bw_probe_kernel<1, false, false>), g, bl, 0, s, a, b, o, n8); break;
    case 1: hipLaunchKernelGGL((bw_probe_kernel<2, false, false>), g, bl, 0, s, a, b, o, n8); break;
    case 2: hipLaunchKernelGGL((bw_probe_kernel<4, false, false>), g, bl, 0, s, a, b, o, n8); break;
    case 3: hipLaunchKernelGGL((bw_probe_kernel<2, true, true>), g, bl, 0, s, a, b, o, n8); break;
    case 4: hipLaunchKernelGGL((bw_probe_kernel<2, false, true>), g, bl, 0, s, a, b, o, n8); break;
    case 5: hipLaunchKernelGGL((bw_probe_kernel<1, false, true>), g, bl, 0, s, a, b, o, n8); break;
    case 6: hipLaunchKernelGGL((bw_probe_kernel<4, false, true>), g, bl, 0, s, a, b, o, n8); break;
    default: hipLaunchKernelGGL((bw_probe_kernel<1, true, true>), g, bl, 0, s, a, b, o, n8); break;
  }
}
}  // namespace pdt
