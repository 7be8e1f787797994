// BatchNorm (+ReLU, +residual) kernels over NHWC 16-bit activations, fp32 math.
//
// Training forward:  conv epilogue accumulates per-channel (sum, sumsq) into fp64 slot copies
//                    -> bn_slot_sum (fp64 per-channel sums; SyncBN all-reduces these)
//                    -> bn_finalize (mean, invstd, folded scale/shift, running-stat update)
//                    -> bn_apply (y*scale+shift [+ residual | + BN(residual)] -> ReLU)
// Training backward: bn_bwd_reduce (dz = g * relu'(out); sum dz, sum dz*xhat for up to two BN
//                    branches that share dz, e.g. the main and downsample branch of a residual block)
//                    -> bn_slot_sum -> bn_bwd_finalize (dgamma/dbeta into the grad buffer,
//                    per-channel coefficients) -> bn_bwd_apply (dy = a*dz + b*y + c per branch).
#include <cstdlib>
#include "../common.h"
#include "bn.h"
#include "conv_fwd.h"

namespace pdt {

// -------------------------------------------------------------------------------------------------
// rows [R][CK] fp32 per-block partials -> slots [kStatSlots][CK] fp64 in a fixed summation order
// (deterministic: no atomics anywhere in the statistics path, see conv_fwd.h).
// Block (column chunk of 64, slot s) sums the CONTIGUOUS row range [s*R/64, (s+1)*R/64): 4 row lanes x 64
// columns, each lane visiting every 4th row with 4 independent loads in flight, the 4 lanes then combined in
// LDS in a fixed order.  (R grows with the conv's M tiles -- ~30k rows x 256 channels for a ResNet-50 layer1
// conv -- so the reduction must stream at HBM rate, not walk 64 long dependent chains.)
__global__ __launch_bounds__(256) void stat_rows_reduce_kernel(const float* __restrict__ rows, int R, int CK,
                                                               double* __restrict__ slots, int LD) {
  __shared__ double part[3][64];
  const int col = blockIdx.x * 64 + (threadIdx.x & 63), lane4 = threadIdx.x >> 6;
  const int s = blockIdx.y;
  const int lo = (int)((int64_t)s * R / kStatSlots), hi = (int)((int64_t)(s + 1) * R / kStatSlots);
  double a = 0.0;
  if (col < CK) {
    const float* p = rows + col;
    int r = lo + lane4;
    double b = 0.0, c = 0.0, d = 0.0;
    for (; r + 12 < hi; r += 16) {
      a += (double)p[(int64_t)r * CK];
      b += (double)p[(int64_t)(r + 4) * CK];
      c += (double)p[(int64_t)(r + 8) * CK];
      d += (double)p[(int64_t)(r + 12) * CK];
    }
    for (; r < hi; r += 4) a += (double)p[(int64_t)r * CK];
    a = (a + b) + (c + d);
  }
  if (lane4 > 0) part[lane4 - 1][threadIdx.x & 63] = a;
  __syncthreads();
  if (lane4 == 0 && col < CK)
    slots[(int64_t)s * LD + col] = ((a + part[0][threadIdx.x]) + part[1][threadIdx.x]) + part[2][threadIdx.x];
}

// slots_ld: row stride of the slots (0 = CK; a channel slice of a wider tensor's statistics: the wider row)
void stat_rows_reduce_launch(const float* rows, int R, int CK, double* slots, hipStream_t s, int slots_ld) {
  hipLaunchKernelGGL(stat_rows_reduce_kernel, dim3((CK + 63) / 64, kStatSlots), dim3(256), 0, s, rows, R, CK, slots,
                     slots_ld ? slots_ld : CK);
}

// slots [kStatSlots][C][K] double (the fixed-order row sums of stat_rows_reduce)
//   -> sums[k*C + c] double  (channel-major per quantity: the SyncBN all-reduce message)
__global__ void bn_slot_sum_kernel(const double* __restrict__ slots, int C, int K, double* __restrict__ sums) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= C * K) return;
  const int c = idx / K, k = idx - (idx / K) * K;
  double s0 = 0, s1 = 0;
  for (int g = 0; g < kStatSlots; g += 2) {
    s0 += slots[((int64_t)g * C + c) * K + k];
    s1 += slots[((int64_t)(g + 1) * C + c) * K + k];
  }
  sums[k * C + c] = s0 + s1;
}

void bn_slot_sum_launch(const double* slots, int C, int K, double* sums, hipStream_t s) {
  hipLaunchKernelGGL(bn_slot_sum_kernel, dim3((C * K + 255) / 256), dim3(256), 0, s, slots, C, K, sums);
}

// -------------------------------------------------------------------------------------------------
// sums[0:C] = sum x, sums[C:2C] = sum x^2, count = number of elements per channel (global)
// coef[0:C] = scale = gamma*invstd, coef[C:2C] = shift = beta - mean*scale,
// coef[2C:3C] = mean, coef[3C:4C] = invstd
__global__ void bn_finalize_kernel(const double* __restrict__ sums, double count, const float* __restrict__ gamma,
                                   const float* __restrict__ beta, float eps, float momentum,
                                   float* __restrict__ running_mean, float* __restrict__ running_var,
                                   float* __restrict__ coef, int C, int update_running) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const double mean = sums[c] / count;
  double var = sums[C + c] / count - mean * mean;
  if (var < 0) var = 0;
  const float invstd = (float)(1.0 / sqrt(var + (double)eps));
  const float sc = gamma[c] * invstd;
  coef[c] = sc;
  coef[C + c] = beta[c] - (float)mean * sc;
  coef[2 * C + c] = (float)mean;
  coef[3 * C + c] = invstd;
  if (update_running) {
    const double unbiased = count > 1 ? var * count / (count - 1) : var;
    running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * (float)mean;
    running_var[c] = (1.f - momentum) * running_var[c] + momentum * (float)unbiased;
  }
}

// Fused (no SyncBN) form of bn_slot_sum + bn_finalize: one thread per channel sums its kStatSlots fp64
// slot copies and finalizes in place (one launch per BN layer instead of two).
// Slot totals for 64 channels per 256-thread block: 4 thread quarters each sum 16 of the kStatSlots slot
// copies (16 independent loads in flight per thread instead of a 64-long serial chain), combined in LDS.
// Returns true in the threads (quarter 0) that hold the totals of a valid channel c.
template <int K>
__device__ inline bool slot_sum_block(const double* __restrict__ slots, int C, double (&s)[K], int& c) {
  static_assert(kStatSlots == 64, "slot_sum_block splits 64 slots in 4 quarters");
  __shared__ double part[3][64][K];
  const int cl = threadIdx.x & 63, q = threadIdx.x >> 6;
  c = blockIdx.x * 64 + cl;
#pragma unroll
  for (int k = 0; k < K; ++k) s[k] = 0.0;
  if (c < C) {
#pragma unroll
    for (int g = 0; g < 16; ++g)
#pragma unroll
      for (int k = 0; k < K; ++k) s[k] += slots[((int64_t)(q * 16 + g) * C + c) * K + k];
  }
  if (q > 0)
#pragma unroll
    for (int k = 0; k < K; ++k) part[q - 1][cl][k] = s[k];
  __syncthreads();
  if (q != 0) return false;
#pragma unroll
  for (int p = 0; p < 3; ++p)
#pragma unroll
    for (int k = 0; k < K; ++k) s[k] += part[p][cl][k];
  return c < C;
}

__global__ __launch_bounds__(256) void bn_finalize_slots_kernel(const double* __restrict__ slots, double count,
                                         const float* __restrict__ gamma, const float* __restrict__ beta, float eps,
                                         float momentum, float* __restrict__ running_mean,
                                         float* __restrict__ running_var, float* __restrict__ coef,
                                         double* __restrict__ sums, int C, int update_running) {
  double sv[2];
  int c;
  if (!slot_sum_block<2>(slots, C, sv, c)) return;
  const double s0 = sv[0], s1 = sv[1];
  sums[c] = s0;
  sums[C + c] = s1;
  const double mean = s0 / count;
  double var = s1 / count - mean * mean;
  if (var < 0) var = 0;
  const float invstd = (float)(1.0 / sqrt(var + (double)eps));
  const float sc = gamma[c] * invstd;
  coef[c] = sc;
  coef[C + c] = beta[c] - (float)mean * sc;
  coef[2 * C + c] = (float)mean;
  coef[3 * C + c] = invstd;
  if (update_running) {
    const double unbiased = count > 1 ? var * count / (count - 1) : var;
    running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * (float)mean;
    running_var[c] = (1.f - momentum) * running_var[c] + momentum * (float)unbiased;
  }
}

void bn_finalize_slots_launch(const double* slots, double count, const float* gamma, const float* beta, float eps,
                              float momentum, float* rm, float* rv, float* coef, double* sums, int C,
                              bool update_running, hipStream_t s) {
  hipLaunchKernelGGL(bn_finalize_slots_kernel, dim3((C + 63) / 64), dim3(256), 0, s, slots, count, gamma, beta, eps,
                     momentum, rm, rv, coef, sums, C, update_running ? 1 : 0);
}

// eval-mode coefficients from running statistics
__global__ void bn_eval_coef_kernel(const float* __restrict__ gamma, const float* __restrict__ beta,
                                    const float* __restrict__ running_mean, const float* __restrict__ running_var,
                                    float eps, float* __restrict__ coef, int C) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float invstd = rsqrtf(running_var[c] + eps);
  const float sc = gamma[c] * invstd;
  coef[c] = sc;
  coef[C + c] = beta[c] - running_mean[c] * sc;
  coef[2 * C + c] = running_mean[c];
  coef[3 * C + c] = invstd;
}

void bn_finalize_launch(const double* sums, double count, const float* gamma, const float* beta, float eps,
                        float momentum, float* rm, float* rv, float* coef, int C, bool update_running,
                        hipStream_t s) {
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + 255) / 256), dim3(256), 0, s, sums, count, gamma, beta, eps,
                     momentum, rm, rv, coef, C, (int)update_running);
}

void bn_eval_coef_launch(const float* gamma, const float* beta, const float* rm, const float* rv, float eps,
                         float* coef, int C, hipStream_t s) {
  hipLaunchKernelGGL(bn_eval_coef_kernel, dim3((C + 255) / 256), dim3(256), 0, s, gamma, beta, rm, rv, eps, coef, C);
}

// -------------------------------------------------------------------------------------------------
// out = act(y*scale + shift + R), R = 0 | res | res*rscale + rshift.
// WM: also write the ReLU bitmask (bit e of mask[v] = out[8v+e] > 0) that the backward reads instead of
// re-reading the 16-bit block output (1 bit instead of 16 per element).
//
// Streaming structure (both apply kernels): a block owns U * 256 CONSECUTIVE 16-byte vectors, thread t the vectors
// t, t + 256, ... (each wave-instruction one contiguous KiB), all U loads issued before any math.  256 vectors are
// 2048 elements, so for C | 2048 (every power-of-two width up to 2048: all ResNet / ResNeXt widths) all of a
// thread's vectors hold the SAME 8 channels and the per-channel coefficients are loaded once per thread into
// registers (CH) instead of once per vector -- the coefficient traffic through the vector L1 was 3-6x the
// streamed bytes.  Other widths (CH = false) index the coefficients per vector.
template <int C8, bool CH>
struct ChanCoef {  // C8 coefficient rows of 8 consecutive channels each
  float v[C8][8];
  PDT_DEVICE void load(const float* __restrict__ p, int C, int c0) {
#pragma unroll
    for (int k = 0; k < C8; ++k) {
      const float4 a = *(const float4*)(p + k * C + c0), b = *(const float4*)(p + k * C + c0 + 4);
      v[k][0] = a.x; v[k][1] = a.y; v[k][2] = a.z; v[k][3] = a.w;
      v[k][4] = b.x; v[k][5] = b.y; v[k][6] = b.z; v[k][7] = b.w;
    }
  }
};

template <int DT, int RESMODE, bool RELU, bool WM, bool NT, int U, bool CH>
__global__ __launch_bounds__(256) void bn_apply_kernel(const uint16_t* __restrict__ y, const float* __restrict__ coef,
                                                       const uint16_t* __restrict__ res,
                                                       const float* __restrict__ rcoef, uint16_t* __restrict__ out,
                                                       uint8_t* __restrict__ mask, int64_t n8, int C) {
  using E = E16<DT>;
  const int64_t v0 = (int64_t)blockIdx.x * (256 * U) + threadIdx.x;
  ChanCoef<2, CH> cf;
  ChanCoef<RESMODE == 2 ? 2 : 1, CH> rf;
  if constexpr (CH) {
    const int c0 = (int)((v0 * 8) & (C - 1));
    cf.load(coef, C, c0);
    if constexpr (RESMODE == 2) rf.load(rcoef, C, c0);
  }
  uint4 yy[U], rr[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t v = v0 + u * 256;
    if (v < n8) {
      yy[u] = ld16<NT>(y + v * 8);
      if constexpr (RESMODE != 0) rr[u] = ld16<NT>(res + v * 8);
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t v = v0 + u * 256;
    if (v >= n8) break;
    if constexpr (!CH) {
      const int c0 = (int)((v * 8) % C);
      cf.load(coef, C, c0);
      if constexpr (RESMODE == 2) rf.load(rcoef, C, c0);
    }
    const uint32_t yw[4] = {yy[u].x, yy[u].y, yy[u].z, yy[u].w};
    uint32_t rw[4] = {0, 0, 0, 0};
    if constexpr (RESMODE != 0) { rw[0] = rr[u].x; rw[1] = rr[u].y; rw[2] = rr[u].z; rw[3] = rr[u].w; }
    uint32_t ow[4], bits = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float o2[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int c = 2 * e + h;
        float val = E::to_f((uint16_t)(yw[e] >> (16 * h))) * cf.v[0][c] + cf.v[1][c];
        if constexpr (RESMODE == 1) val += E::to_f((uint16_t)(rw[e] >> (16 * h)));
        if constexpr (RESMODE == 2) val += E::to_f((uint16_t)(rw[e] >> (16 * h))) * rf.v[0][c] + rf.v[1][c];
        if constexpr (RELU) val = fmaxf(val, 0.f);
        o2[h] = val;
      }
      ow[e] = (uint32_t)E::from_f(o2[0]) | ((uint32_t)E::from_f(o2[1]) << 16);
      // the mask tests the ROUNDED output, exactly what a 16-bit re-read would see
      if constexpr (WM) bits |= ((ow[e] & 0x7fffu) != 0 && !(ow[e] & 0x8000u) ? 1u : 0u) << (2 * e) |
                                ((ow[e] & 0x7fff0000u) != 0 && !(ow[e] & 0x80000000u) ? 1u : 0u) << (2 * e + 1);
    }
    st16<NT>(out + v * 8, make_uint4(ow[0], ow[1], ow[2], ow[3]));
    if constexpr (WM) mask[v] = (uint8_t)bits;
  }
}

// Elementwise grids: one block per U * 256 consecutive 16-byte vectors, U = 4 (no grid-stride loop: the in-order
// block dispatch keeps the concurrently streamed window contiguous; capping the grid at a few thousand looping
// blocks cost ~20% of bandwidth, tools/bw_probe.py).  tools/ew_bench.py, ResNet shapes at B = 1200 (round 5):
// U = 1 (one vector per thread, coefficients indexed per vector, the round-4 structure) 5.3-6.1 TB/s, U = 2 and 4
// 6.2-6.7 TB/s (two-branch backward 7.3-7.6), U = 8 a few % below 4.  Streams larger than the L2s and MALL use
// nontemporal loads/stores.
constexpr int kEwU = 4;
static int ew_blocks(int64_t n8, int U) {
  const int64_t b = (n8 + 256 * U - 1) / (256 * U);
  if (b >= (int64_t(1) << 31)) pdt_hip_fail("elementwise pass: tensor too large", hipErrorInvalidValue, __FILE__, __LINE__);
  return (int)(b < 1 ? 1 : b);
}
static bool ew_nt(int64_t bytes) {
  return bytes >= (64ll << 20);  // non-temporal loads / stores from 64 MiB operands on (round-4 sweep)
}
static bool ew_ch(int C) { return C > 0 && C <= 2048 && (C & (C - 1)) == 0 && C % 8 == 0; }

// dispatch an elementwise kernel template K<..., NT, U, CH> over (NT, CH): U = kEwU with hoisted coefficients,
// one vector per thread otherwise
#define PDT_EW_DISPATCH(KERNEL, TARGS, grid_of, nt, ch, ...)                                                     \
  do {                                                                                                           \
    const dim3 b_(256);                                                                                          \
    if (!(ch)) {                                                                                                 \
      if (nt) hipLaunchKernelGGL((KERNEL<TARGS, true, 1, false>), dim3(grid_of(1)), b_, 0, s, __VA_ARGS__);     \
      else hipLaunchKernelGGL((KERNEL<TARGS, false, 1, false>), dim3(grid_of(1)), b_, 0, s, __VA_ARGS__);      \
    } else {                                                                                                     \
      if (nt) hipLaunchKernelGGL((KERNEL<TARGS, true, kEwU, true>), dim3(grid_of(kEwU)), b_, 0, s, __VA_ARGS__); \
      else hipLaunchKernelGGL((KERNEL<TARGS, false, kEwU, true>), dim3(grid_of(kEwU)), b_, 0, s, __VA_ARGS__);  \
    }                                                                                                            \
  } while (0)

template <int DT>
static void bn_apply_dt(const uint16_t* y, const float* coef, const uint16_t* res, const float* rcoef, uint16_t* out,
                        uint8_t* mask, int64_t n, int C, int resmode, bool relu, hipStream_t s) {
  const int64_t n8 = n / 8;
  auto grid = [&](int U) { return ew_blocks(n8, U); };
  const bool wm = mask != nullptr, nt = ew_nt(n * 2), ch = ew_ch(C);
#define PDT_AP(RM, RL, WM)                                                                                       \
  if (resmode == RM && relu == RL && wm == WM) {                                                                 \
    PDT_EW_DISPATCH(bn_apply_kernel, PDT_TARGS(DT, RM, RL, WM), grid, nt, ch, y, coef, res, rcoef, out, mask, n8, C); \
    return;                                                                                                      \
  }
#define PDT_TARGS(...) __VA_ARGS__
  PDT_AP(0, true, false) PDT_AP(1, true, false) PDT_AP(2, true, false) PDT_AP(0, false, false)
  PDT_AP(1, false, false) PDT_AP(2, false, false) PDT_AP(1, true, true) PDT_AP(2, true, true)
#undef PDT_AP
#undef PDT_TARGS
}

void bn_apply_launch(int dtype, const uint16_t* y, const float* coef, const uint16_t* res, const float* rcoef,
                     uint16_t* out, uint8_t* mask, int64_t n, int C, int resmode, bool relu, hipStream_t s) {
  if (dtype == kBF16)
    bn_apply_dt<kBF16>(y, coef, res, rcoef, out, mask, n, C, resmode, relu, s);
  else
    bn_apply_dt<kF16>(y, coef, res, rcoef, out, mask, n, C, resmode, relu, s);
}

// -------------------------------------------------------------------------------------------------
// Backward reduce.  dz = g * mask (ReLU bitmask of the block output, optional).  For branch b in {1,2}:
//   part[blk][c][2b-2] += dz ; part[blk][c][2b-1] += dz * (y_b - mean_b) * invstd_b
// Each thread owns 8 consecutive channels of a row; rows are strided over the grid.
template <int DT, bool MASK, int NBR>
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(const uint16_t* __restrict__ g,
                                                            const uint8_t* __restrict__ mask,
                                                            const uint16_t* __restrict__ y1,
                                                            const float* __restrict__ coef1,
                                                            const uint16_t* __restrict__ y2,
                                                            const float* __restrict__ coef2,
                                                            float* __restrict__ srows, int64_t rows, int C) {
  using E = E16<DT>;
  const int vpr = C / 8;              // 16-byte vectors per row
  const int rpi = 256 / vpr;          // rows per block iteration (C <= 2048)
  const int cv = threadIdx.x % vpr;   // vector (channel group) index
  const int rl = threadIdx.x / vpr;   // row lane
  const int c0 = cv * 8;
  float s[NBR * 2][8];
#pragma unroll
  for (int k = 0; k < NBR * 2; ++k)
#pragma unroll
    for (int e = 0; e < 8; ++e) s[k][e] = 0.f;
  float m1[8], i1[8], m2[8], i2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    m1[e] = coef1[2 * C + c0 + e];
    i1[e] = coef1[3 * C + c0 + e];
    if constexpr (NBR == 2) { m2[e] = coef2[2 * C + c0 + e]; i2[e] = coef2[3 * C + c0 + e]; }
  }
  if (rl < rpi) {
    for (int64_t r = (int64_t)blockIdx.x * rpi + rl; r < rows; r += (int64_t)gridDim.x * rpi) {
      const int64_t off = r * C + c0;
      const uint4 gv = *(const uint4*)(g + off);
      const uint32_t gw[4] = {gv.x, gv.y, gv.z, gv.w};
      uint32_t mb = 0xffu;
      if constexpr (MASK) mb = mask[off >> 3];
      const uint4 y1v = *(const uint4*)(y1 + off);
      const uint32_t y1w[4] = {y1v.x, y1v.y, y1v.z, y1v.w};
      uint32_t y2w[4] = {0, 0, 0, 0};
      if constexpr (NBR == 2) { const uint4 y2v = *(const uint4*)(y2 + off); y2w[0] = y2v.x; y2w[1] = y2v.y; y2w[2] = y2v.z; y2w[3] = y2v.w; }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int sh = 16 * (e & 1);
        float dz = E::to_f((uint16_t)(gw[e >> 1] >> sh));
        if constexpr (MASK) dz = (mb >> e) & 1u ? dz : 0.f;
        const float x1 = (E::to_f((uint16_t)(y1w[e >> 1] >> sh)) - m1[e]) * i1[e];
        s[0][e] += dz;
        s[1][e] += dz * x1;
        if constexpr (NBR == 2) {
          const float x2 = (E::to_f((uint16_t)(y2w[e >> 1] >> sh)) - m2[e]) * i2[e];
          s[2][e] += dz;
          s[3][e] += dz * x2;
        }
      }
    }
  }
  // block reduction over row lanes: LDS [rpi][C][NBR*2]
  extern __shared__ float red[];
  const int K = NBR * 2;
  if (rl < rpi) {
#pragma unroll
    for (int e = 0; e < 8; ++e)
#pragma unroll
      for (int k = 0; k < NBR * 2; ++k) red[((int64_t)rl * C + c0 + e) * K + k] = s[k][e];
  }
  __syncthreads();
  float* dst = srows + (int64_t)blockIdx.x * C * K;  // this block's own partial row
  for (int idx = threadIdx.x; idx < C * K; idx += 256) {
    float t = 0.f;
    for (int r = 0; r < rpi; ++r) t += red[(int64_t)r * C * K + idx];
    dst[idx] = t;
  }
}

int bn_bwd_reduce_blocks(int64_t rows, int C) {
  const int rpi = 256 / (C / 8);
  int64_t b = (rows + rpi * 16 - 1) / (rpi * 16);  // >= 16 rows per thread
  if (b > 1024) b = 1024;
  return (int)(b < 1 ? 1 : b);
}

void bn_bwd_reduce_launch(int dtype, const uint16_t* g, const uint8_t* out, const uint16_t* y1, const float* coef1,
                          const uint16_t* y2, const float* coef2, double* slots, int blocks, int64_t rows, int C,
                          hipStream_t s) {
  const int rpi = 256 / (C / 8);
  const int nbr = y2 ? 2 : 1;
  Scratch part((size_t)blocks * C * nbr * 2 * sizeof(float), s);
  float* srows = part.as<float>();
  const size_t smem = (size_t)rpi * C * nbr * 2 * sizeof(float);
  const bool mask = out != nullptr;
#define PDT_BR(DT_, M_, NB_)                                                                              \
  if (mask == M_ && nbr == NB_) {                                                                         \
    hipLaunchKernelGGL((bn_bwd_reduce_kernel<DT_, M_, NB_>), dim3(blocks), dim3(256), smem, s, g, out, y1, \
                       coef1, y2, coef2, srows, rows, C);                                                  \
    stat_rows_reduce_launch(srows, blocks, C * nbr * 2, slots, s);                                        \
    return;                                                                                               \
  }
  if (dtype == kBF16) {
    PDT_BR(kBF16, true, 1) PDT_BR(kBF16, true, 2) PDT_BR(kBF16, false, 1) PDT_BR(kBF16, false, 2)
  } else {
    PDT_BR(kF16, true, 1) PDT_BR(kF16, true, 2) PDT_BR(kF16, false, 1) PDT_BR(kF16, false, 2)
  }
#undef PDT_BR
}

// -------------------------------------------------------------------------------------------------
// sums[0:C] = sum dz, sums[C:2C] = sum dz*xhat (global over the batch, all ranks for SyncBN).
// Writes dgamma/dbeta (scaled by gscale) into the grad buffer and the elementwise coefficients
//   dy = A*dz + B*y + Cc,   A = gamma*invstd, B = -A*invstd*mean_dzx... (expanded below)
// dy = gamma*invstd*(dz - mean_dz - xhat*mean_dzx) with xhat = (y-mean)*invstd
//    = A*dz + (-A*invstd*mean_dzx)*y + (-A*mean_dz + A*invstd*mean_dzx*mean)
__global__ void bn_bwd_finalize_kernel(const double* __restrict__ sums, double count, const float* __restrict__ coef,
                                       const float* __restrict__ gamma, float* __restrict__ dgamma,
                                       float* __restrict__ dbeta, float gscale, float* __restrict__ bcoef, int C) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const double sdz = sums[c], sdzx = sums[C + c];
  if (dgamma) dgamma[c] = (float)sdzx * gscale;
  if (dbeta) dbeta[c] = (float)sdz * gscale;
  const float mean = coef[2 * C + c], invstd = coef[3 * C + c];
  const float A = gamma[c] * invstd;
  const float mdz = (float)(sdz / count), mdzx = (float)(sdzx / count);
  bcoef[c] = A;
  bcoef[C + c] = -A * invstd * mdzx;
  bcoef[2 * C + c] = -A * mdz + A * invstd * mdzx * mean;
}

void bn_bwd_finalize_launch(const double* sums, double count, const float* coef, const float* gamma, float* dgamma,
                            float* dbeta, float gscale, float* bcoef, int C, hipStream_t s) {
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 255) / 256), dim3(256), 0, s, sums, count, coef, gamma, dgamma,
                     dbeta, gscale, bcoef, C);
}

// Fused (no SyncBN) slot sum + backward finalize for one or two BN branches sharing dz
// (slots [kStatSlots][C][K], K = 2 or 4: sum dz1, sum dz1*x1, sum dz2, sum dz2*x2).
__device__ inline void bn_bwd_coef(double sdz, double sdzx, double count, float mean, float invstd, float gamma,
                                   float* dgamma, float* dbeta, float gscale, float* bcoef, int C, int c) {
  if (dgamma) dgamma[c] = (float)sdzx * gscale;
  if (dbeta) dbeta[c] = (float)sdz * gscale;
  const float A = gamma * invstd;
  const float mdz = (float)(sdz / count), mdzx = (float)(sdzx / count);
  bcoef[c] = A;
  bcoef[C + c] = -A * invstd * mdzx;
  bcoef[2 * C + c] = -A * mdz + A * invstd * mdzx * mean;
}

template <int K>
__global__ __launch_bounds__(256) void bn_bwd_finalize_slots_kernel(const double* __restrict__ slots, double count,
                                             const float* __restrict__ coef1, const float* __restrict__ gamma1,
                                             float* __restrict__ dgamma1, float* __restrict__ dbeta1,
                                             float* __restrict__ bcoef1, const float* __restrict__ coef2,
                                             const float* __restrict__ gamma2, float* __restrict__ dgamma2,
                                             float* __restrict__ dbeta2, float* __restrict__ bcoef2, float gscale,
                                             int C) {
  double s[K];
  int c;
  if (!slot_sum_block<K>(slots, C, s, c)) return;
  bn_bwd_coef(s[0], s[1], count, coef1[2 * C + c], coef1[3 * C + c], gamma1[c], dgamma1, dbeta1, gscale, bcoef1, C, c);
  if constexpr (K == 4)
    bn_bwd_coef(s[2], s[3], count, coef2[2 * C + c], coef2[3 * C + c], gamma2[c], dgamma2, dbeta2, gscale, bcoef2, C, c);
}

void bn_bwd_finalize_slots_launch(const double* slots, int K, double count, const float* coef1, const float* gamma1,
                                  float* dgamma1, float* dbeta1, float* bcoef1, const float* coef2,
                                  const float* gamma2, float* dgamma2, float* dbeta2, float* bcoef2, float gscale,
                                  int C, hipStream_t s) {
  if (K == 4)
    hipLaunchKernelGGL(bn_bwd_finalize_slots_kernel<4>, dim3((C + 63) / 64), dim3(256), 0, s, slots, count, coef1,
                       gamma1, dgamma1, dbeta1, bcoef1, coef2, gamma2, dgamma2, dbeta2, bcoef2, gscale, C);
  else
    hipLaunchKernelGGL(bn_bwd_finalize_slots_kernel<2>, dim3((C + 63) / 64), dim3(256), 0, s, slots, count, coef1,
                       gamma1, dgamma1, dbeta1, bcoef1, coef2, gamma2, dgamma2, dbeta2, bcoef2, gscale, C);
}

// dy_b = A_b*dz + B_b*y_b + C_b for b = 1 (and 2); optionally also writes dz (identity branch grad).
// Streaming structure and coefficient hoisting (CH) as bn_apply_kernel.
template <int DT, bool MASK, int NBR, bool WDZ, bool NT, int U, bool CH>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const uint16_t* __restrict__ g,
                                                           const uint8_t* __restrict__ mask,
                                                           const uint16_t* __restrict__ y1,
                                                           const float* __restrict__ b1, uint16_t* __restrict__ dy1,
                                                           const uint16_t* __restrict__ y2,
                                                           const float* __restrict__ b2, uint16_t* __restrict__ dy2,
                                                           uint16_t* __restrict__ dz_out, int64_t n8, int C) {
  using E = E16<DT>;
  const int64_t v0 = (int64_t)blockIdx.x * (256 * U) + threadIdx.x;
  ChanCoef<3, CH> f1;
  ChanCoef<NBR == 2 ? 3 : 1, CH> f2;
  if constexpr (CH) {
    const int c0 = (int)((v0 * 8) & (C - 1));
    f1.load(b1, C, c0);
    if constexpr (NBR == 2) f2.load(b2, C, c0);
  }
  uint4 gv[U], y1v[U], y2v[U];
  uint32_t mb[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t v = v0 + u * 256;
    if (v < n8) {
      gv[u] = ld16<NT>(g + v * 8);
      mb[u] = 0xffu;
      if constexpr (MASK) mb[u] = mask[v];
      y1v[u] = ld16<NT>(y1 + v * 8);
      if constexpr (NBR == 2) y2v[u] = ld16<NT>(y2 + v * 8);
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t v = v0 + u * 256;
    if (v >= n8) break;
    if constexpr (!CH) {
      const int c0 = (int)((v * 8) % C);
      f1.load(b1, C, c0);
      if constexpr (NBR == 2) f2.load(b2, C, c0);
    }
    const uint32_t gw[4] = {gv[u].x, gv[u].y, gv[u].z, gv[u].w};
    const uint32_t y1w[4] = {y1v[u].x, y1v[u].y, y1v[u].z, y1v[u].w};
    uint32_t y2w[4] = {0, 0, 0, 0};
    if constexpr (NBR == 2) { y2w[0] = y2v[u].x; y2w[1] = y2v[u].y; y2w[2] = y2v[u].z; y2w[3] = y2v[u].w; }
    uint32_t o1[4], o2[4], oz[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      uint16_t r1[2], r2[2], rz[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int c = 2 * e + h;
        float dz = E::to_f((uint16_t)(gw[e] >> (16 * h)));
        if constexpr (MASK) dz = (mb[u] >> (2 * e + h)) & 1u ? dz : 0.f;
        rz[h] = E::from_f(dz);
        r1[h] = E::from_f(f1.v[0][c] * dz + f1.v[1][c] * E::to_f((uint16_t)(y1w[e] >> (16 * h))) + f1.v[2][c]);
        if constexpr (NBR == 2)
          r2[h] = E::from_f(f2.v[0][c] * dz + f2.v[1][c] * E::to_f((uint16_t)(y2w[e] >> (16 * h))) + f2.v[2][c]);
      }
      o1[e] = (uint32_t)r1[0] | ((uint32_t)r1[1] << 16);
      if constexpr (NBR == 2) o2[e] = (uint32_t)r2[0] | ((uint32_t)r2[1] << 16);
      oz[e] = (uint32_t)rz[0] | ((uint32_t)rz[1] << 16);
    }
    st16<NT>(dy1 + v * 8, make_uint4(o1[0], o1[1], o1[2], o1[3]));
    if constexpr (NBR == 2) st16<NT>(dy2 + v * 8, make_uint4(o2[0], o2[1], o2[2], o2[3]));
    if constexpr (WDZ) st16<NT>(dz_out + v * 8, make_uint4(oz[0], oz[1], oz[2], oz[3]));
  }
}

void bn_bwd_apply_launch(int dtype, const uint16_t* g, const uint8_t* out, const uint16_t* y1, const float* b1,
                         uint16_t* dy1, const uint16_t* y2, const float* b2, uint16_t* dy2, uint16_t* dz_out, int64_t n,
                         int C, hipStream_t s) {
  const int64_t n8 = n / 8;
  auto grid = [&](int U) { return ew_blocks(n8, U); };
  const bool mask = out != nullptr, wdz = dz_out != nullptr, nt = ew_nt(n * 2), ch = ew_ch(C);
  const int nbr = y2 ? 2 : 1;
#define PDT_TARGS(...) __VA_ARGS__
#define PDT_BA(DT_, M_, NB_, WZ_)                                                                                \
  if (mask == M_ && nbr == NB_ && wdz == WZ_) {                                                                  \
    PDT_EW_DISPATCH(bn_bwd_apply_kernel, PDT_TARGS(DT_, M_, NB_, WZ_), grid, nt, ch, g, out, y1, b1, dy1, y2, b2, \
                    dy2, dz_out, n8, C);                                                                         \
    return;                                                                                                      \
  }
  if (dtype == kBF16) {
    PDT_BA(kBF16, true, 1, false) PDT_BA(kBF16, true, 1, true) PDT_BA(kBF16, true, 2, false)
    PDT_BA(kBF16, false, 1, false) PDT_BA(kBF16, false, 2, false) PDT_BA(kBF16, false, 1, true)
  } else {
    PDT_BA(kF16, true, 1, false) PDT_BA(kF16, true, 1, true) PDT_BA(kF16, true, 2, false)
    PDT_BA(kF16, false, 1, false) PDT_BA(kF16, false, 2, false) PDT_BA(kF16, false, 1, true)
  }
#undef PDT_BA
#undef PDT_TARGS
  pdt_hip_fail("bn_bwd_apply: unsupported variant", hipErrorInvalidValue, __FILE__, __LINE__);
}

}  // namespace pdt
