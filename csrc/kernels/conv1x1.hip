// 1x1 / stride-1 "expanding" convolution, 64 -> 256 channels (ResNet-50 layer1: each block's conv3 and the
// downsample), as a persistent, store-overlapped kernel.
//
// With K = 64 a 1x1 conv is one MFMA K-step per output tile: the implicit-GEMM kernels spend a block's life in
// load latency -> a few MFMAs -> an epilogue that writes 2-4x the bytes it read, and the next tile's load waits
// for the store queue too (vmcnt counts stores): 777 us (512 x 128 ping-pong) against ~350 us for writing the
// 1.93 GB output at ResNet-50 B = 1200 (profiles/r2c_resnet50_1x1_write_bound.md).  Here:
//   * the whole weight matrix (256 x 64, 32 KB) stays in registers as MFMA A fragments (8 per wave) after one
//     LDS-DMA; each wave owns 64 output channels of every tile;
//   * blocks are persistent (2 per CU) and walk 128-pixel tiles; a tile's 16 KB input is DMA'd into a 2-deep LDS
//     ring one tile ahead;
//   * the per-tile wait is COUNTED: the next tile's DMA is issued before this tile's 16 stores, so waiting for it
//     (s_waitcnt vmcnt(16)) leaves the stores in flight -- the store stream of tile t overlaps tile t+1;
//   * BN statistics of the rounded outputs accumulate in registers across all of a block's tiles and are reduced
//     once (16-lane DPP sums) into the block's partial row (deterministic, conv_fwd.h).
//   * PRE: x is the RAW output of the producer conv (a bottleneck's conv2) and its BatchNorm + ReLU is applied to
//     each input fragment after the LDS read (pre_act8, bit-identical to bn_apply): the activation is never
//     written.  A lane's fragment channels are fixed (kk * 32 + fq * 8 + [0, 8)), so its 16 scale / shift pairs
//     live in registers for the whole kernel.
#include <cstdlib>

#include "../common.h"
#include "conv1x1.h"
#include "conv_fwd.h"

namespace pdt {

namespace {
constexpr int kC = 64, kK = 256;
constexpr int kBM = 128;               // pixels per tile
constexpr int kRowB = kC * 2;          // 128 B per pixel row / weight row
constexpr int kTileB = kBM * kRowB;    // 16 KB
constexpr int kWB = kK * kRowB;        // 32 KB
constexpr int kStoresPerTile = 16;     // global stores per wave per full tile: 8 pixel x 2 channel-fragment pairs
static_assert(kStoresPerTile == 16, "the per-tile s_waitcnt vmcnt(16) literal below");
}  // namespace

template <int DT, bool STATS, bool PRE>
__global__ __launch_bounds__(256, 2) void conv1x1_c64_kernel(const uint16_t* __restrict__ x,
                                                             const uint16_t* __restrict__ w,
                                                             uint16_t* __restrict__ y, float* __restrict__ srows,
                                                             const float* __restrict__ pre_coef, int64_t M) {
  using E = E16<DT>;
  typedef typename E::vec8 vec8;
  __shared__ __attribute__((aligned(1024))) char smem[kWB + 2 * kTileB];
  char* const wl = smem;
  char* const xl = smem + kWB;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int lrow = lane >> 3, pchunk = lane & 7;
  const int sw = (fr >> 1) & 7;  // fragment rows start at multiples of 16: row swizzle (row >> 1) & 7 == sw
  const int tiles = (int)((M + kBM - 1) / kBM);
  const int G = gridDim.x;
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(x, (uint32_t)(M * kRowB));
  const __amdgpu_buffer_rsrc_t rw = make_rsrc(w, (uint32_t)kWB);

  // LDS row images: LDS chunk p of row r holds source chunk p ^ ((r >> 1) & 7) (conflict-free ds_read_b128)
  // resident weights: 32 DMA instructions of 8 rows x 8 chunks, 8 per wave
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int ins = wave * 8 + j;
    const int row = ins * 8 + lrow;
    buf_lds16_asm(rw, wl + ins * 1024, (uint32_t)(row * kRowB + ((pchunk ^ ((row >> 1) & 7)) << 4)));
  }
  // one tile's input: 16 instructions, 4 per wave; rows past M read zeros (their results are not stored)
  auto stage_x = [&](int t, int buf) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int ins = wave * 4 + j;
      const int row = ins * 8 + lrow;
      const int64_t m = (int64_t)t * kBM + row;
      const uint32_t off = m < M ? (uint32_t)(m * kRowB + ((pchunk ^ ((row >> 1) & 7)) << 4)) : kOOB;
      buf_lds16_asm(rx, xl + buf * kTileB + ins * 1024, off);
    }
  };

  int t = blockIdx.x;
  if (t < tiles) stage_x(t, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // this wave's 64 output channels as resident MFMA A fragments: [cout fragment i][K half kk].  Fragment rows are
  // permuted (wave_ch below) so that fragments 2p and 2p+1 give a lane 8 CONSECUTIVE channels of its pixel: one
  // 16-byte store per pixel and fragment pair, 64 contiguous bytes per pixel per store instruction.
  auto wave_ch = [](int i, int row) { return (i >> 1) * 32 + (row >> 2) * 8 + (i & 1) * 4 + (row & 3); };
  vec8 af[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int wr = wave * 64 + wave_ch(i, fr);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
      af[i][kk] = *(const vec8*)(wl + wr * kRowB + (((kk * 4 + fq) ^ ((wr >> 1) & 7)) << 4));
  }

  float ssum[4][4], ssq[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) { ssum[i][r] = 0.f; ssq[i][r] = 0.f; }
  // PRE: scale / shift of this lane's fragment channels kk * 32 + fq * 8 + e
  float psc[2][8], psh[2][8];
  if constexpr (PRE) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        psc[kk][e] = pre_coef[kk * 32 + fq * 8 + e];
        psh[kk][e] = pre_coef[kC + kk * 32 + fq * 8 + e];
      }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the loop's counted waits must not see these loads
  }

  int buf = 0;
  bool first = true;
  for (; t < tiles; t += G) {
    if (!first) {
      // tile t's DMA was issued before the previous tile's 16 stores (the previous tile was a full one: only a
      // block's last tile can be the partial M tail); vector-memory ops retire in order, so waiting down to 16
      // outstanding retires the DMA and leaves the stores in flight.  Raw barrier (no vmcnt(0) drain): every
      // wave's part of the DMA landed and every wave finished reading the other ring slot.
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
    first = false;
    if (t + G < tiles) stage_x(t + G, buf ^ 1);

    const char* xb = xl + buf * kTileB;
    const int64_t mt = (int64_t)t * kBM;
    // two 64-pixel halves (64 accumulators each, no spills): half 1's MFMAs run behind half 0's stores
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      f32x4_t acc[4][4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        vec8 bf[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          bf[j] = *(const vec8*)(xb + ((h * 4 + j) * 16 + fr) * kRowB + (((kk * 4 + fq) ^ sw) << 4));
          if constexpr (PRE)
            bf[j] = __builtin_bit_cast(vec8, pre_act8<DT>(__builtin_bit_cast(uint4, bf[j]), psc[kk], psh[kk]));
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = E::mfma16x16x32(af[i][kk], bf[j], acc[i][j]);
      }
      // epilogue: fragment pair p gives the lane channels wave*64 + p*32 + 8*fq + [0, 8) of pixel
      // t*128 + (h*4 + j)*16 + fr
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t m = mt + (h * 4 + j) * 16 + fr;
        uint16_t* yp = y + m * kK + wave * 64 + 8 * fq;
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          uint4 pk;  // one v_cvt_pk_bf16_f32 per pair (E16::pack2)
          pk.x = E::pack2(acc[2 * p][j][0], acc[2 * p][j][1]);
          pk.y = E::pack2(acc[2 * p][j][2], acc[2 * p][j][3]);
          pk.z = E::pack2(acc[2 * p + 1][j][0], acc[2 * p + 1][j][1]);
          pk.w = E::pack2(acc[2 * p + 1][j][2], acc[2 * p + 1][j][3]);
          uint16_t o[8];
          unpack8(pk, o);
          if (m < M) {
            *(uint4*)(yp + p * 32) = pk;
            if constexpr (STATS) {
#pragma unroll
              for (int r = 0; r < 8; ++r) {
                const float q = E::to_f(o[r]);
                ssum[2 * p + (r >> 2)][r & 3] += q;
                ssq[2 * p + (r >> 2)][r & 3] += q * q;
              }
            }
          }
        }
      }
    }
    buf ^= 1;
  }

  if constexpr (STATS) {
    // reduce over the 16 pixel lanes; lane fr == 15 owns channel wave*64 + wave_ch(i, 4*fq + r) of the block's row
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        ssum[i][r] = row16_sum(ssum[i][r]);
        ssq[i][r] = row16_sum(ssq[i][r]);
      }
    if (fr == 15) {
      float* dst = srows + (int64_t)blockIdx.x * kK * 2;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int c = wave * 64 + wave_ch(i, 4 * fq + r);
          *(float2*)(dst + c * 2) = make_float2(ssum[i][r], ssq[i][r]);
        }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// The same GEMM as the backward-data pass of ResNet-50 layer1's REDUCING 1x1 conv (256 -> 64 forward: dX[M][256] =
// dY[M][64] x W^T), with the dgrad epilogue of a block-output BatchNorm fused (conv_fwd.h EPI 3): v = acc + res,
// dz = v where the block output's ReLU bit is set (else 0), stored rounded, and per channel sum(dz) and
// sum(dz * (y1 - mean1) * invstd1) into the block's statistics row; BR = 2 (EPI 4): a second BatchNorm branch on
// the same block input (a downsample block's main and shortcut BN) adds sum(dz * (y2 - mean2) * invstd2).  The generic path runs this as the 512 x 128
// ping-pong kernel with ONE K-step per tile (1.5-1.7 ms per call at B = 1200).
// Tiles are 64 pixels (two 32-pixel sub-tiles): per tile and wave 24 epilogue operand loads (residual, y1: 16 B;
// mask: 1 B per 8 channels; BR = 2: 8 more for y2) and 8 stores follow the next tile's input DMA, so the loop-top
// wait is vmcnt(32) (BR = 2: vmcnt(40)).
namespace {
constexpr int kBMb = 64;
constexpr int kTileBb = kBMb * kRowB;  // 8 KB
constexpr int kOpsPerTileB = 32;       // vector-memory ops per wave after the next tile's DMA (24 loads + 8 stores; +8)
}  // namespace

template <int DT, int BR, int KH>
__global__ __launch_bounds__(256, 2) void conv1x1_c64_bnb_kernel(const uint16_t* __restrict__ x,
                                                                 const uint16_t* __restrict__ w,
                                                                 uint16_t* __restrict__ y,
                                                                 const uint16_t* __restrict__ res,
                                                                 const uint16_t* __restrict__ y1,
                                                                 const float* __restrict__ coef1,
                                                                 const uint16_t* __restrict__ y2,
                                                                 const float* __restrict__ coef2,
                                                                 const uint8_t* __restrict__ mask,
                                                                 float* __restrict__ srows, int64_t M) {
  static_assert(BR == 1 || BR == 2, "one or two BatchNorm branches");
  static_assert(KH == 1 || KH == 2, "64 or 128 reduction channels");
  static_assert(kOpsPerTileB == 32, "the loop-top s_waitcnt vmcnt(32 | 40) literals below");
  using E = E16<DT>;
  typedef typename E::vec8 vec8;
  // KH 64-channel halves of the reduction, each in the 128-B-row layout of the K = 64 kernel.  KH = 2: the 64 KB of
  // weights pass through LDS once (into registers) and the input ring then reuses that area (2 workgroups per CU)
  constexpr int kXOff = KH == 1 ? kWB : 0;
  constexpr int kCfOff = KH == 1 ? kWB + 2 * kTileBb : 2 * kWB;
  static_assert(KH == 1 || 2 * KH * kTileBb <= KH * kWB, "input ring inside the weight staging area");
  __shared__ __attribute__((aligned(1024))) char smem[kCfOff + BR * 2 * kK * 4];
  char* const wl = smem;
  char* const xl = smem + kXOff;
  // per-branch BN mean / invstd of all 256 channels: cf[(branch * 2 + 0 | 1) * 256 + c]
  float* const cf = (float*)(smem + kCfOff);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int lrow = lane >> 3, pchunk = lane & 7;
  const int sw = (fr >> 1) & 7;
  const int tiles = (int)((M + kBMb - 1) / kBMb);
  const int G = gridDim.x;
  constexpr int kSrcRow = KH * kRowB;  // bytes per source row (x: pixel, w: output channel)
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(x, (uint32_t)(M * kSrcRow));
  const __amdgpu_buffer_rsrc_t rw = make_rsrc(w, (uint32_t)(KH * kWB));
  auto wave_ch = [](int i, int row) { return (i >> 1) * 32 + (row >> 2) * 8 + (i & 1) * 4 + (row & 3); };

#pragma unroll
  for (int hh = 0; hh < KH; ++hh)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int ins = wave * 8 + j;
      const int row = ins * 8 + lrow;
      buf_lds16_asm(rw, wl + hh * kWB + ins * 1024,
                    (uint32_t)(row * kSrcRow + hh * kRowB + ((pchunk ^ ((row >> 1) & 7)) << 4)));
    }
  // one tile's input: 8 instructions per half, 2 per wave
  auto stage_x = [&](int t, int buf) {
#pragma unroll
    for (int hh = 0; hh < KH; ++hh)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int ins = wave * 2 + j;
        const int row = ins * 8 + lrow;
        const int64_t m = (int64_t)t * kBMb + row;
        const uint32_t off =
            m < M ? (uint32_t)(m * kSrcRow + hh * kRowB + ((pchunk ^ ((row >> 1) & 7)) << 4)) : kOOB;
        buf_lds16_asm(rx, xl + (buf * KH + hh) * kTileBb + ins * 1024, off);
      }
  };

  int t = blockIdx.x;
  if constexpr (KH == 1) {
    if (t < tiles) stage_x(t, 0);
  }
  cf[tid] = coef1[2 * kK + tid];
  cf[kK + tid] = coef1[3 * kK + tid];
  if constexpr (BR == 2) {
    cf[2 * kK + tid] = coef2[2 * kK + tid];
    cf[3 * kK + tid] = coef2[3 * kK + tid];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  vec8 af[4][2 * KH];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int wr = wave * 64 + wave_ch(i, fr);
#pragma unroll
    for (int kq = 0; kq < 2 * KH; ++kq)
      af[i][kq] = *(const vec8*)(wl + (kq >> 1) * kWB + wr * kRowB + ((((kq & 1) * 4 + fq) ^ ((wr >> 1) & 7)) << 4));
  }
  if constexpr (KH == 2) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();  // every wave holds its weight fragments: the area becomes the input ring
    if (t < tiles) stage_x(t, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  // statistics of this lane's 16 output channels: pair p, element e -> channel wave*64 + p*32 + 8*fq + e
  float s0[2][8], s1[2][8], s2[BR == 2 ? 2 : 1][8];
#pragma unroll
  for (int p = 0; p < 2; ++p)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      s0[p][e] = 0.f;
      s1[p][e] = 0.f;
      if constexpr (BR == 2) s2[p][e] = 0.f;
    }

  int buf = 0;
  bool first = true;
  for (; t < tiles; t += G) {
    if (!first) {
      // tile t's DMA was issued before the previous (full) tile's 24 | 32 operand loads and 8 stores: waiting down to
      // that many outstanding retires it and leaves the stores in flight
      if constexpr (BR == 1)
        asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(40)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
    first = false;
    if (t + G < tiles) stage_x(t + G, buf ^ 1);

    const char* xb = xl + buf * KH * kTileBb;
    const int64_t mt = (int64_t)t * kBMb;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      // epilogue operands first (independent of the MFMAs); rows past M load row M-1 and are not stored
      uint4 rr[2][2], yy[2][2], yz[BR == 2 ? 2 : 1][2];
      uint32_t mb[2][2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        int64_t m = mt + (h * 2 + j) * 16 + fr;
        m = m < M ? m : M - 1;
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const int64_t o = m * kK + wave * 64 + p * 32 + 8 * fq;
          rr[j][p] = *(const uint4*)(res + o);
          yy[j][p] = *(const uint4*)(y1 + o);
          if constexpr (BR == 2) yz[j][p] = *(const uint4*)(y2 + o);
          mb[j][p] = mask[o >> 3];
        }
      }
      f32x4_t acc[4][2];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kq = 0; kq < 2 * KH; ++kq) {
        vec8 bf[2];
#pragma unroll
        for (int j = 0; j < 2; ++j)
          bf[j] = *(const vec8*)(xb + (kq >> 1) * kTileBb + ((h * 2 + j) * 16 + fr) * kRowB +
                                 ((((kq & 1) * 4 + fq) ^ sw) << 4));
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = E::mfma16x16x32(af[i][kq], bf[j], acc[i][j]);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int64_t m = mt + (h * 2 + j) * 16 + fr;
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const uint32_t rw4[4] = {rr[j][p].x, rr[j][p].y, rr[j][p].z, rr[j][p].w};
          const uint32_t yw4[4] = {yy[j][p].x, yy[j][p].y, yy[j][p].z, yy[j][p].w};
          float vv[8], q1[8], q2[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            float v = acc[2 * p + (e >> 2)][j][e & 3] + E::to_f((uint16_t)(rw4[e >> 1] >> (16 * (e & 1))));
            if (!((mb[j][p] >> e) & 1u)) v = 0.f;
            vv[e] = v;
            q1[e] = E::to_f((uint16_t)(yw4[e >> 1] >> (16 * (e & 1))));
          }
          if constexpr (BR == 2) {
            const uint32_t zw4[4] = {yz[j][p].x, yz[j][p].y, yz[j][p].z, yz[j][p].w};
#pragma unroll
            for (int e = 0; e < 8; ++e) q2[e] = E::to_f((uint16_t)(zw4[e >> 1] >> (16 * (e & 1))));
          }
          uint4 pk;  // one v_cvt_pk_bf16_f32 per pair (E16::pack2)
          pk.x = E::pack2(vv[0], vv[1]);
          pk.y = E::pack2(vv[2], vv[3]);
          pk.z = E::pack2(vv[4], vv[5]);
          pk.w = E::pack2(vv[6], vv[7]);
          uint16_t o[8];
          unpack8(pk, o);
          if (m < M) {
            const int c0 = wave * 64 + p * 32 + 8 * fq;
            *(uint4*)(y + m * kK + c0) = pk;
            const float4 ma = *(const float4*)(cf + c0), mb4 = *(const float4*)(cf + c0 + 4);
            const float4 ia = *(const float4*)(cf + kK + c0), ib = *(const float4*)(cf + kK + c0 + 4);
            const float mu[8] = {ma.x, ma.y, ma.z, ma.w, mb4.x, mb4.y, mb4.z, mb4.w};
            const float is[8] = {ia.x, ia.y, ia.z, ia.w, ib.x, ib.y, ib.z, ib.w};
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float dz = E::to_f(o[e]);
              s0[p][e] += dz;
              s1[p][e] += dz * (q1[e] - mu[e]) * is[e];
            }
            if constexpr (BR == 2) {
              const float4 na = *(const float4*)(cf + 2 * kK + c0), nb = *(const float4*)(cf + 2 * kK + c0 + 4);
              const float4 ja = *(const float4*)(cf + 3 * kK + c0), jb = *(const float4*)(cf + 3 * kK + c0 + 4);
              const float mu2[8] = {na.x, na.y, na.z, na.w, nb.x, nb.y, nb.z, nb.w};
              const float is2[8] = {ja.x, ja.y, ja.z, ja.w, jb.x, jb.y, jb.z, jb.w};
#pragma unroll
              for (int e = 0; e < 8; ++e) s2[p][e] += E::to_f(o[e]) * (q2[e] - mu2[e]) * is2[e];
            }
          }
        }
      }
    }
    buf ^= 1;
  }

  // reduce over the 16 pixel lanes; lane fr == 15 owns channels wave*64 + p*32 + 8*fq + e of the block's row
  // ([256][2] = (sum dz, sum dz*xhat1); two branches: [256][4] = (sum dz, sum dz*xhat1, sum dz, sum dz*xhat2))
#pragma unroll
  for (int p = 0; p < 2; ++p)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      s0[p][e] = row16_sum(s0[p][e]);
      s1[p][e] = row16_sum(s1[p][e]);
      if constexpr (BR == 2) s2[p][e] = row16_sum(s2[p][e]);
    }
  if (fr == 15) {
    constexpr int KO = BR == 2 ? 4 : 2;
    float* dst = srows + (int64_t)blockIdx.x * kK * KO;
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = wave * 64 + p * 32 + 8 * fq + e;
        if constexpr (BR == 2)
          *(float4*)(dst + c * 4) = make_float4(s0[p][e], s1[p][e], s0[p][e], s2[p][e]);
        else
          *(float2*)(dst + c * 2) = make_float2(s0[p][e], s1[p][e]);
      }
  }
}

void conv1x1_c64_bnb_launch(const uint16_t* x, const uint16_t* w, uint16_t* y, const uint16_t* res,
                            const uint16_t* y1, const float* coef1, const uint16_t* y2, const float* coef2,
                            const uint8_t* mask, double* slots, int64_t M, int cin, int dtype, hipStream_t s) {
  if (cin != 64 && !(cin == 128 && y2 == nullptr))
    pdt_hip_fail("conv1x1_c64_bnb: 64 reduction channels, or 128 with one BN branch", hipErrorInvalidValue, __FILE__,
                 __LINE__);
  if (M <= 0) return;
  if (M * kK >= (int64_t(1) << 31))
    pdt_hip_fail("conv1x1_c64_bnb: operands exceed 32-bit offsets", hipErrorInvalidValue, __FILE__, __LINE__);
  static const int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      n = 256;
    return n > 0 ? n : 256;
  }();
  const int tiles = (int)((M + kBMb - 1) / kBMb);
  const int G = tiles < 2 * cus ? tiles : 2 * cus;
  const int KO = y2 ? 4 : 2;
  Scratch part((size_t)G * kK * KO * sizeof(float), s);
  float* srows = part.as<float>();
  PDT_COUNT("conv1x1_c64_bnb");
  if (cin == 128)
    PDT_COUNT("conv1x1_c64_bnb_c128");
  else if (y2)
    PDT_COUNT("conv1x1_c64_bnb_2br");
  else
    PDT_COUNT("conv1x1_c64_bnb_1br");
#define PDT_CB(DT_, BR_, KH_)                                                                                     \
  hipLaunchKernelGGL((conv1x1_c64_bnb_kernel<DT_, BR_, KH_>), dim3(G), dim3(256), 0, s, x, w, y, res, y1, coef1, y2,  \
                     coef2, mask, srows, M)
  if (dtype == kBF16) {
    if (cin == 128) PDT_CB(kBF16, 1, 2); else if (y2) PDT_CB(kBF16, 2, 1); else PDT_CB(kBF16, 1, 1);
  } else {
    if (cin == 128) PDT_CB(kF16, 1, 2); else if (y2) PDT_CB(kF16, 2, 1); else PDT_CB(kF16, 1, 1);
  }
#undef PDT_CB
  stat_rows_reduce_launch(srows, G, kK * KO, slots, s);
}

int conv1x1_c64_mode(int set) {
  // PDT_CONV1X1=0: the generic implicit-GEMM kernels (A/B); set >= 0 switches at run time (tests)
  static int on = [] {
    const char* e = getenv("PDT_CONV1X1");
    return e && e[0] == '0' ? 0 : 1;
  }();
  const int prev = on;
  if (set >= 0) on = set;
  return prev;
}

bool conv1x1_c64_supported(int C, int Kout) { return conv1x1_c64_mode(-1) && C == kC && Kout == kK; }

void conv1x1_c64_launch(const uint16_t* x, const uint16_t* w, uint16_t* y, double* stats, int64_t M, int dtype,
                        hipStream_t s, const float* pre_coef) {
  if (M <= 0) return;
  if (M * kRowB >= (int64_t(1) << 31) || M * kK >= (int64_t(1) << 31))
    pdt_hip_fail("conv1x1_c64: operands exceed 32-bit offsets", hipErrorInvalidValue, __FILE__, __LINE__);
  static const int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      n = 256;
    return n > 0 ? n : 256;
  }();
  const int tiles = (int)((M + kBM - 1) / kBM);
  const int G = tiles < 2 * cus ? tiles : 2 * cus;
  Scratch part(stats ? (size_t)G * kK * 2 * sizeof(float) : 0, s);
  float* srows = part.as<float>();
  PDT_COUNT("conv1x1_c64");
  if (pre_coef && !stats)
    pdt_hip_fail("conv1x1_c64: the fused producer BN (pre_coef) runs in training forwards (with statistics)",
                 hipErrorInvalidValue, __FILE__, __LINE__);
  if (pre_coef) PDT_COUNT("conv1x1_c64_fused_bn_relu");
#define PDT_C1(DT_, ST_, PR_)                                                                                  \
  hipLaunchKernelGGL((conv1x1_c64_kernel<DT_, ST_, PR_>), dim3(G), dim3(256), 0, s, x, w, y, srows, pre_coef, M)
  if (dtype == kBF16) {
    if (pre_coef) PDT_C1(kBF16, true, true); else if (stats) PDT_C1(kBF16, true, false); else PDT_C1(kBF16, false, false);
  } else {
    if (pre_coef) PDT_C1(kF16, true, true); else if (stats) PDT_C1(kF16, true, false); else PDT_C1(kF16, false, false);
  }
#undef PDT_C1
  if (stats) stat_rows_reduce_launch(srows, G, kK * 2, stats, s);
}

}  // namespace pdt
