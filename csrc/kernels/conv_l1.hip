// 3x3 / stride 1 / pad 1 convolution with 64 input and 64 output channels on 56-wide images (ResNet
// layer1, the most expensive convolutions of ResNet-18/34), forward and backward-data.
//
// The generic implicit-GEMM kernel (conv_fwd.hip) streams a 256-pixel x 64-channel activation tile and
// a weight tile per (tap, channel) K-step: every activation is fetched 9 times (once per tap) and the
// L2 -> LDS stream, not the MFMAs, bounds it (~570 TF/s).  This kernel is built around the data reuse:
//   * the whole weight tensor (64 x 9 x 64 bf16 = 72 KB) stays resident in LDS for the block's life;
//   * a block tile is 4 output rows x 56 columns of one image; its input halo (6 rows x 58 columns x 64
//     channels, zero padding from the buffer range check) is staged ONCE by LDS-DMA into a 2-deep ring
//     (tile i+1 streams in while tile i computes) and all 9 taps read shifted windows of it;
//   * MFMA B fragments (8 consecutive channels of one pixel) are single ds_read_b128s of the halo
//     (rows XOR-swizzled by row & 7 with a matching lane -> pixel order: conflict-free);
//     A fragments come from the resident weights (chunks swizzled by (cout >> 1) & 7);
//   * persistent blocks (one per CU: 72 + 2 x 43.5 KB of LDS), XCD-contiguous tile ranges;
//   * the epilogues of conv_fwd.hip: residual add, forward BN statistics, or the fused BN-backward
//     reduce (ReLU mask from the BN input or from the block output), statistics accumulated in
//     registers across all of a block's tiles.
// Backward-data is the same convolution of dY with the transposed, 180-degree-rotated weights
// ([C][3][3][K] with taps reversed): ``flip`` reads tap 8 - t of the derived dgrad weights.
#include <cstdlib>
#include <type_traits>

#include "../common.h"
#include "conv_fwd.h"
#include "conv_l1.h"

namespace pdt {

namespace {
constexpr int kW = 56;                     // image width
constexpr int kXP = kW + 2;                // halo row pitch (pixels)
constexpr int kXRows = 6 * kXP;            // 348 halo pixels per tile
constexpr int kStageB = kXRows * 128;      // 44544 B
constexpr int kWB = 64 * 9 * 64 * 2;       // 73728 B of resident weights
constexpr int kLds = kWB + 2 * kStageB;    // 162816 B, plus 1 KiB of BN coefficients = the whole 160 KiB
constexpr int kGroups = 4 * kW / 16;       // 14 groups of 16 pixels per tile

// Halo row swizzle: 16-B chunk p of LDS row R holds logical chunk p ^ (R & 7).  ds_read_b128 serves a
// wave in 4 groups of 16 lanes; each group reads chunk c for 8 pixels and chunk c ^ 1 for 8 others.
// With the lane -> pixel map pix_of_lane() below, each set of 8 is 8 consecutive halo rows of one image
// row (56 is a multiple of 8), so (R & 1, c ^ (R & 7)) is distinct across the whole group: conflict-free
// for every tap shift (tools/lds_sim.py).
PDT_DEVICE int hswz(int R) { return R & 7; }
// MFMA column (lane & 15) -> pixel within a 16-pixel group: lanes {0-3, 12-15} -> pixels 0..7,
// lanes 4..11 -> pixels 8..15 (matches the ds_read_b128 lane groups {0-3,12-15,20-27}, ...)
PDT_DEVICE int pix_of_lane(int fr) { return fr < 4 ? fr : (fr >= 12 ? fr - 8 : fr + 4); }
PDT_DEVICE int wswz(int co, int c) { return (c & ~7) | ((c & 7) ^ ((co >> 1) & 7)); }  // weight chunk
// conv_l1pp_kernel's weight rows are read permuted (A fragment i row fr = output channel 8 * (fr >> 2) + 4 * i +
// (fr & 3) of the wave's 32): its swizzle is the same function of the READING lane's fr as wswz's, so the fragment
// reads stay conflict-free
PDT_DEVICE int wswz_pp(int co, int c) { return (c & ~7) | ((c & 7) ^ ((((co >> 3) & 3) << 1) | ((co & 3) >> 1))); }
}  // namespace

// PRE: the input is the raw output of the block's first conv; its BatchNorm + ReLU is applied to each staged
// halo in LDS (one pass per tile, padding rows / columns left zero) instead of by a separate bn_apply pass.
template <int DT, int EPI, bool RES, bool PRE = false>
__global__ __launch_bounds__(256) void conv_l1_kernel(ConvFwdArgs a, int flip) {
  using E = E16<DT>;
  typedef typename E::vec8 vec8;
  __shared__ __attribute__((aligned(1024))) char smem[kLds + 1024];
  char* const wl = smem;
  char* const stage0 = smem + kWB;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;

  const int TH = (a.H + 3) / 4;
  const int tiles = a.N * TH;
  const int G = gridDim.x;
  const int xcd = blockIdx.x & 7, lb = blockIdx.x >> 3, per_x = G >> 3;
  const int t_per = (tiles + 7) >> 3;
  const int t_begin = xcd * t_per, t_end = min(tiles, t_begin + t_per);

  const uint32_t img_bytes = (uint32_t)a.N * a.H * kW * 128u;
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(a.x, img_bytes);
  const __amdgpu_buffer_rsrc_t rw = make_rsrc(a.w, (uint32_t)kWB);
  const int lrow = lane >> 3, pch = lane & 7;

  // ---- resident weights by LDS-DMA: 72 instructions of 8 rows x 8 chunks (18 per wave) ----
  // LDS row co has 72 chunks; LDS chunk p of row co holds source chunk wswz(co, p) (an involution)
#pragma unroll
  for (int m = 0; m < 18; ++m) {
    const int ii = wave + 4 * m;
    const int L = ii * 64 + lrow * 8 + pch;  // LDS chunk index 0..4607
    const int co = L / 72, p = L - co * 72;
    buf_lds16(rw, wl + ii * 1024, (uint32_t)(co * 72 + wswz(co, p)) * 16u);
  }

  // ---- halo DMA: 348 rows of 128 B (44 instructions, 11 per wave; the last one half-masked) ----
  auto stage_tile = [&](int t, int buf) {
    const int n = t / TH, h0 = (t - n * TH) * 4;
    char* sb = stage0 + buf * kStageB;
#pragma unroll
    for (int m = 0; m < 11; ++m) {
      const int ii = wave + 4 * m;
      const int R = ii * 8 + lrow;
      if (R < kXRows) {
        const int hr = R / kXP, wc = R - (R / kXP) * kXP;
        const int h = h0 - 1 + hr, w = wc - 1;
        const bool ok = (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)kW;
        const uint32_t off = ok ? (uint32_t)((((n * a.H + h) * kW + w) * 64 + (pch ^ hswz(R)) * 8) * 2) : kOOB;
        // PRE: opaque DMA, or the compiler drains it (vmcnt(0)) before the in-LDS transform of the other buffer
        if constexpr (PRE)
          buf_lds16_asm(rx, sb + ii * 1024, off);
        else
          buf_lds16(rx, sb + ii * 1024, off);
      }
    }
  };

  // pixel groups of this wave: 14 groups over 4 waves -> 4, 4, 3, 3
  const int g0 = wave < 2 ? wave * 4 : 8 + (wave - 2) * 3;
  const int ng = wave < 2 ? 4 : 3;
  // per group: halo row (tap 0,0) of this lane's pixel
  int R0[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int px = (g0 + j) * 16 + pix_of_lane(fr);
    const int r = px / kW, w = px - (px / kW) * kW;
    R0[j] = r * kXP + w;
  }

  constexpr int KS = EPI == 0 ? 1 : 2;
  float sacc[4][4][KS];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int k = 0; k < KS; ++k) sacc[i][r][k] = 0.f;

  // BN coefficients of the fused BN-backward epilogues ([scale, shift, mean, invstd] x 64 channels) in the
  // last KiB of LDS, read per channel fragment in the epilogue: held in registers across the MFMA loop they
  // cost 32-64 VGPRs per lane, which this kernel (one wave per SIMD, 18 unrolled K-steps) does not have.
  float* const cfl = (float*)(smem + kLds);
  if constexpr (EPI >= 2) cfl[tid] = a.bn_coef1[tid];  // published by the first tile's barrier
  auto coef = [&](int q, int i) { return *(const float4*)(cfl + q * 64 + i * 16 + 4 * fq); };

  // PRE: thread tid transforms halo rows R = tid/8 + 32k at physical chunk tid%8, which always holds logical
  // chunk (tid ^ (tid >> 3)) & 7 (the row swizzle is R & 7 and 32k keeps it): 8 fixed channels per thread
  float pre_sc[8], pre_sh[8];
  if constexpr (PRE) {
    const int lc = (tid ^ (tid >> 3)) & 7;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      pre_sc[e] = a.pre_coef[lc * 8 + e];
      pre_sh[e] = a.pre_coef[64 + lc * 8 + e];
    }
  }

  int t = t_begin + lb;
  int buf = 0;
  // Stores this wave issued in the previous tile's epilogue: they are the only vector-memory operations
  // younger than the halo DMA of the tile about to be computed, and vmcnt retires in issue order, so
  // vmcnt(n_st) proves the DMA landed without also waiting out the store latency (vmcnt(0) here used to
  // expose ~1-2 us of store drain per tile: one wave per SIMD, nothing else to cover it).  Every live
  // pixel group issues exactly 4 stores (H % 4 == 0: no partial row tiles), so n_st = 4 * ng.
  int n_st = 0;
  if (t < t_end) stage_tile(t, 0);
  for (; t < t_end; t += per_x) {
    if (n_st == 16)
      __builtin_amdgcn_s_waitcnt((16 & 0xF) | ((16 >> 4) << 14) | (0x7 << 4) | (0xF << 8));
    else if (n_st == 12)
      __builtin_amdgcn_s_waitcnt((12 & 0xF) | ((12 >> 4) << 14) | (0x7 << 4) | (0xF << 8));
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA (and the weights, first time)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (t + per_x < t_end) stage_tile(t + per_x, buf ^ 1);
    // PRE: transform this tile's halo while the next tile's DMA (into the other buffer) is in flight
    if constexpr (PRE) {
      const int n = t / TH, h0 = (t - n * TH) * 4;
      char* sbw = stage0 + buf * kStageB;
      // two batches (6 + 5 chunks): all of a batch's LDS reads in flight together, register budget kept
#pragma unroll
      for (int k0 = 0; k0 < 11; k0 += 6) {
        int off[6];
        bool ok[6];
#pragma unroll
        for (int k = 0; k < 6; ++k) {
          const int R = min((tid >> 3) + 32 * (k0 + k), kXRows - 1);
          const int hr = R / kXP, wc = R - (R / kXP) * kXP;
          const int h = h0 - 1 + hr, w = wc - 1;
          ok[k] = k0 + k < 11 && (tid >> 3) + 32 * (k0 + k) < kXRows && (unsigned)h < (unsigned)a.H &&
                  (unsigned)w < (unsigned)kW;
          off[k] = R * 128 + (tid & 7) * 16;
        }
        pre_act_chunks<DT, 6>(sbw, off, ok, pre_sc, pre_sh);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
    const char* sb = stage0 + buf * kStageB;

    // epilogue operands (residual, BN input, block output) of this tile, loaded now so their latency
    // hides under the MFMA loop (one block per CU: nothing else would cover an exposed epilogue)
    const int n = t / TH, h0 = (t - n * TH) * 4;
    int64_t obase[4];
    uint2 pre_res[RES ? 4 : 1][RES ? 4 : 1], pre_y1[EPI >= 2 ? 4 : 1][EPI >= 2 ? 4 : 1];
    uint64_t pre_m[EPI == 3 ? 4 : 1];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      // a 3-group wave's 4th group re-reads group 0 (unused): every wave issues the same loads, unconditionally
      const int px = (g0 + (j < ng ? j : 0)) * 16 + pix_of_lane(fr);
      const int r = px / kW, w = px - (px / kW) * kW;
      obase[j] = ((int64_t)(n * a.H + h0 + r) * kW + w) * 64;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c0 = i * 16 + 4 * fq;
        if constexpr (RES) pre_res[j][i] = *(const uint2*)(a.res + obase[j] + c0);
        if constexpr (EPI >= 2) pre_y1[j][i] = *(const uint2*)(a.bn_y1 + obase[j] + c0);
      }
      if constexpr (EPI == 3) pre_m[j] = *(const uint64_t*)(a.bn_mask + (obase[j] >> 3));
    }

    f32x4_t acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    // 18 K-steps (9 taps x 2 channel halves), fully unrolled so the LDS reads of a step can be issued
    // ahead of the previous step's MFMAs; the group count is a wave-uniform branch outside the loop
    auto run = [&](auto NGc) {
      constexpr int NG = decltype(NGc)::value;
      // Fragments of step st+1 are read while step st's MFMAs run: an explicit register double buffer,
      // pinned with scheduling barriers (left alone, hipcc sinks each ds_read to ~3 MFMAs before its use,
      // which exposes the LDS latency on every fragment -- one wave per SIMD, nothing else covers it).
      vec8 af[2][4], bf[2][NG];
      auto load = [&](int st, int sl) {
        const int tap = st >> 1, kk = st & 1;
        const int tr = tap / 3, tu = tap % 3;
        const int wtap = flip ? 8 - tap : tap;
        const int dR = tr * kXP + tu;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int co = i * 16 + fr;
          const int c = wtap * 8 + kk * 4 + fq;
          af[sl][i] = *(const vec8*)(wl + co * 1152 + wswz(co, c) * 16);
        }
#pragma unroll
        for (int j = 0; j < NG; ++j) {
          const int R = R0[j] + dR;
          bf[sl][j] = *(const vec8*)(sb + R * 128 + (((kk * 4 + fq) ^ hswz(R)) << 4));
        }
      };
      load(0, 0);
#pragma unroll
      for (int st = 0; st < 18; ++st) {
        if (st + 1 < 18) load(st + 1, (st + 1) & 1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < NG; ++j) acc[i][j] = E::mfma16x16x32(af[st & 1][i], bf[st & 1][j], acc[i][j]);
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    if (ng == 4)
      run(std::integral_constant<int, 4>{});
    else
      run(std::integral_constant<int, 3>{});

    // ---- epilogue: lane holds couts n = i*16 + 4*fq + r of pixel (g0+j)*16 + fr ----
    // H % 4 == 0 (conv_l1_eligible): every pixel of a live group is in range, so the epilogue is straight-line
    // code -- a branch around the stores would leave the waitcnt pass unsure how many were issued, and it
    // then waited vmcnt(0) (the previous group's store latency) in front of every group.
    n_st = 4 * ng;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (j >= ng) break;  // wave-uniform
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c0 = i * 16 + 4 * fq;
        float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
        if constexpr (RES) {
          const uint2 rr = pre_res[j][i];
          v[0] += E::to_f((uint16_t)(rr.x & 0xffff));
          v[1] += E::to_f((uint16_t)(rr.x >> 16));
          v[2] += E::to_f((uint16_t)(rr.y & 0xffff));
          v[3] += E::to_f((uint16_t)(rr.y >> 16));
        }
        float y1[4];
        if constexpr (EPI >= 2) {
          const uint2 q1 = pre_y1[j][i];
          y1[0] = E::to_f((uint16_t)(q1.x & 0xffff)); y1[1] = E::to_f((uint16_t)(q1.x >> 16));
          y1[2] = E::to_f((uint16_t)(q1.y & 0xffff)); y1[3] = E::to_f((uint16_t)(q1.y >> 16));
          if constexpr (EPI == 2) {
            const float4 sc = coef(0, i), sh = coef(1, i);
            if (!(y1[0] * sc.x + sh.x > 0.f)) v[0] = 0.f;
            if (!(y1[1] * sc.y + sh.y > 0.f)) v[1] = 0.f;
            if (!(y1[2] * sc.z + sh.z > 0.f)) v[2] = 0.f;
            if (!(y1[3] * sc.w + sh.w > 0.f)) v[3] = 0.f;
          } else {
            const uint32_t mb = (uint32_t)(pre_m[j] >> c0);
            if (!(mb & 1u)) v[0] = 0.f;
            if (!(mb & 2u)) v[1] = 0.f;
            if (!(mb & 4u)) v[2] = 0.f;
            if (!(mb & 8u)) v[3] = 0.f;
          }
        }
        uint2 packed;  // one v_cvt_pk_bf16_f32 per pair (E16::pack2)
        packed.x = E::pack2(v[0], v[1]);
        packed.y = E::pack2(v[2], v[3]);
        const uint16_t o[4] = {(uint16_t)packed.x, (uint16_t)(packed.x >> 16), (uint16_t)packed.y,
                               (uint16_t)(packed.y >> 16)};
        *(uint2*)(a.y + obase[j] + c0) = packed;
        if constexpr (EPI == 1) {
#pragma unroll
          for (int r2 = 0; r2 < 4; ++r2) {
            const float q = E::to_f(o[r2]);
            sacc[i][r2][0] += q;
            sacc[i][r2][1] += q * q;
          }
        } else if constexpr (EPI >= 2) {
          const float4 mu = coef(2, i), is = coef(3, i);
          const float m1[4] = {mu.x, mu.y, mu.z, mu.w}, i1[4] = {is.x, is.y, is.z, is.w};
#pragma unroll
          for (int r2 = 0; r2 < 4; ++r2) {
            const float dz = E::to_f(o[r2]);
            sacc[i][r2][0] += dz;
            sacc[i][r2][1] += dz * (y1[r2] - m1[r2]) * i1[r2];
          }
        }
      }
    }
    buf ^= 1;
  }

  if constexpr (EPI > 0) {
    // block totals: DPP row scan over the 16 pixel lanes, then the 4 waves through LDS (stage 0 is
    // free once every wave passed the barrier below), stored to this block's own partial row (conv_fwd.h)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int k = 0; k < KS; ++k) sacc[i][r][k] = row16_sum(sacc[i][r][k]);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();
    float* red = (float*)stage0;  // [4 waves][64][2]
    if (fr == 15) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int c = i * 16 + 4 * fq + r;
          red[(wave * 64 + c) * 2 + 0] = sacc[i][r][0];
          red[(wave * 64 + c) * 2 + 1] = sacc[i][r][1];
        }
    }
    __syncthreads();
    if (tid < 128) a.srows[(int64_t)blockIdx.x * 128 + tid] = red[tid] + red[128 + tid] + red[256 + tid] + red[384 + tid];
  }
}

// ------------------------------------------------------------------------------------------------
// 8-wave "ping-pong" variant of the kernel above (the default; PDT_CONV_L1_PP=0 selects the 4-wave one):
// ResNet-18 bs1200 bf16 layer1 forward / backward-data 3.2 -> 2.5 ms of kernel time, 21.34 -> 21.04 ms/step (same box).
//
// The 4-wave kernel runs one wave per SIMD, so everything that is not an MFMA -- the epilogue (16-bit
// conversion, statistics, 14-16 scattered stores per lane), the fused producer-BN transform of the halo
// (PRE), the barrier at every tile -- leaves the matrix pipe idle, and its 14 pixel groups split 4/4/3/3
// over the waves (two SIMDs idle a quarter of every tile).  Here two groups of 4 waves (one wave of each
// group per SIMD) work on alternate tiles of the block one phase apart:
//     phase A: group 0 computes tile 2i        | group 1: epilogue of tile 2i-1, DMA (+ PRE transform) of 2i+1
//     phase B: group 0: epilogue 2i, DMA 2i+2   | group 1 computes tile 2i+1
// so on every SIMD one wave's MFMAs run while its partner does the memory / VALU work of the other tile.
// LDS: the resident weights (72 KB, shared) + ONE halo buffer per group (2 x 43.5 KB) = the same 160 KB.
// A group's buffer is refilled in its memory phase right after its compute phase read it (the phase
// barrier orders the two), and each wave waits for its own DMA pieces (counted vmcnt) and -- PRE --
// transforms exactly the halo chunks it DMA'd itself, so no extra barrier is needed before the next
// compute phase's barrier.  Work split inside a group: 2 (32 output channels) x 2 (7 pixel groups) --
// balanced, 14 MFMAs per 9 LDS reads per K-step.
// SL: a 64-channel slice of wider tensors (grouped convs, ResNeXt stage 1): input pixel stride a.cs, output / BN-input
// pixel stride a.ldy, BN coefficient quantity stride a.coef_ld (forward with statistics and backward data with the
// inner-BN reduce only: no residual, no producer BN)
template <int DT, int EPI, bool RES, bool PRE, bool FLIP, bool SL = false>
__global__ __launch_bounds__(512) void conv_l1pp_kernel(ConvFwdArgs a) {
  static_assert(!SL || (!RES && !PRE && EPI <= 2), "sliced layer1 kernel: EPI 0-2 without residual / producer BN");
  using E = E16<DT>;
  typedef typename E::vec8 vec8;
  constexpr int NJ = 7;  // pixel groups per wave
  __shared__ __attribute__((aligned(1024))) char smem[kLds + 1024];
  char* const wl = smem;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave >> 2, gw = wave & 3;
  const int wn = gw & 1, wm = gw >> 1;
  const int fr = lane & 15, fq = lane >> 4;
  const int lrow = lane >> 3, pch = lane & 7;
  char* const sbuf = smem + kWB + grp * kStageB;  // this group's halo buffer

  const int TH = (a.H + 3) / 4;
  const int tiles = a.N * TH;
  const int G = gridDim.x;
  const int xcd = blockIdx.x & 7, lb = blockIdx.x >> 3, per_x = G >> 3;
  const int t_per = (tiles + 7) >> 3;
  const int t_begin = xcd * t_per, t_end = min(tiles, t_begin + t_per);
  const int first = t_begin + lb;
  const int nk = first < t_end ? (t_end - first + per_x - 1) / per_x : 0;  // this block's tiles (block-uniform)

  const int xcs = SL ? a.cs : 64, ldo = SL ? a.ldy : 64;  // pixel strides (elements) of x / of y, res, bn_y1
  const uint32_t img_bytes = (uint32_t)a.N * a.H * kW * (uint32_t)ldo * 2u;
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(a.x, (uint32_t)a.N * a.H * kW * (uint32_t)xcs * 2u);
  const __amdgpu_buffer_rsrc_t rw = make_rsrc(a.w, (uint32_t)kWB);
  const __amdgpu_buffer_rsrc_t ry1 = make_rsrc(EPI >= 2 ? a.bn_y1 : a.x, img_bytes);
  const __amdgpu_buffer_rsrc_t rres = make_rsrc(RES ? a.res : a.x, img_bytes);
  const __amdgpu_buffer_rsrc_t rmask = make_rsrc(EPI == 3 ? (const void*)a.bn_mask : (const void*)a.x, img_bytes / 16u);

  // ---- resident weights: 72 DMA instructions, 9 per wave (all DMA here is asm: explicitly counted) ----
#pragma unroll
  for (int m = 0; m < 9; ++m) {
    const int ii = wave + 8 * m;
    const int L = ii * 64 + lrow * 8 + pch;
    const int co = L / 72, p = L - co * 72;
    buf_lds16_asm(rw, wl + ii * 1024, (uint32_t)(co * 72 + wswz_pp(co, p)) * 16u);
  }
  // ---- a group's halo DMA: 44 instructions, 11 per wave, the last one half-masked ----
  auto stage_tile = [&](int t) {
    const int n = t / TH, h0 = (t - n * TH) * 4;
    int lr = lrow;
    asm volatile("" : "+v"(lr));  // per-call row decode: hoisted out of the tile loop it is ~40 live registers
#pragma unroll
    for (int m = 0; m < 11; ++m) {
      const int ii = gw + 4 * m;
      const int R = ii * 8 + lr;
      if (R < kXRows) {
        const int hr = R / kXP, wc = R - (R / kXP) * kXP;
        const int h = h0 - 1 + hr, w = wc - 1;
        const bool ok = (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)kW;
        buf_lds16_asm(rx, sbuf + ii * 1024,
                      ok ? (uint32_t)((((n * a.H + h) * kW + w) * xcs + (pch ^ (wc & 7)) * 8) * 2) : kOOB);
      }
    }
    asm volatile("" ::: "memory");  // no later store may be scheduled ahead of the DMA (counted waits below)
  };
  // PRE: this lane's halo chunks are row (gw + 4m) * 8 + lrow, physical chunk pch = logical chunk pch ^ (column & 7);
  // the BN coefficients of each chunk's 8 channels come from the LDS coefficient block (registers are short here)
  auto transform = [&](int t) {  // after this wave's own DMA of tile t landed
    const int n = t / TH, h0 = (t - n * TH) * 4;
    const float* cpre = (const float*)(smem + kLds);
#pragma unroll
    for (int m = 0; m < 11; ++m) {
      const int R = (gw + 4 * m) * 8 + lrow;
      const bool live = R < kXRows;
      const int Rc = live ? R : 0;
      const int hr = Rc / kXP, wc = Rc - (Rc / kXP) * kXP;
      const int h = h0 - 1 + hr, w = wc - 1;
      const bool ok = live && (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)kW;
      const float* cp = cpre + (pch ^ (wc & 7)) * 8;
      float sc[8], sh[8];
      *(float4*)&sc[0] = *(const float4*)(cp);
      *(float4*)&sc[4] = *(const float4*)(cp + 4);
      *(float4*)&sh[0] = *(const float4*)(cp + 64);
      *(float4*)&sh[4] = *(const float4*)(cp + 68);
      char* q = sbuf + Rc * 128 + pch * 16;
      const uint4 v = *(const uint4*)q;
      if (ok) *(uint4*)q = pre_act8<DT>(v, sc, sh);
    }
  };

  // per pixel group: halo row (tap 0,0) of this lane's pixel; groups wm*7 .. wm*7+6 of the tile
  // Fragment addresses without per-read arithmetic.  This kernel swizzles a halo row by its COLUMN (physical
  // chunk = logical chunk ^ (column & 7); conflict-free like the row swizzle, tools/lds_sim.py): a tap (tr, tu)
  // shifts the row by dR = 58 tr + tu but the column only by tu, so baddr[j][tu] -- the LDS byte address of
  // group j's kk = 0 fragment at column shift tu -- plus the immediate dR * 128 addresses every tap; kk = 1 flips
  // address bit 6 (its chunk is the kk = 0 chunk ^ 4).  The weight address is one base per kk plus immediates
  // (cout block i, tap): 23 address registers in all, one VALU op (the xor) per fragment read at kk = 1.
  uint32_t baddr[NJ][3];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int px = (wm * NJ + j) * 16 + pix_of_lane(fr);
    const int r = px / kW, w = px - (px / kW) * kW;
    const int R0 = r * kXP + w;  // halo column of tap (., 0) is w
#pragma unroll
    for (int tu = 0; tu < 3; ++tu)
      baddr[j][tu] = (uint32_t)(kWB + grp * kStageB + R0 * 128 + ((fq ^ ((w + tu) & 7)) << 4));
  }
  // permuted weight rows: fragment i row fr = channel wn*32 + 8*(fr >> 2) + 4*i + (fr & 3), so a lane's two fragments
  // hold the 8 CONSECUTIVE channels wn*32 + 8*fq .. +7 of its pixel: one 16-byte store / operand load per pixel group
  // (round 5, same box: ResNet-18 20.32/20.31/20.28 -> 20.15/20.16/20.14 ms, ResNet-50 73.07/73.15 -> 72.94/72.92 ms)
  const uint32_t abase0 = (uint32_t)((wn * 32 + 8 * (fr >> 2) + (fr & 3)) * 1152 + ((fq ^ ((fr >> 1) & 7)) << 4));
  const uint32_t abase1 = abase0 ^ 64u;
  auto xor64 = [](uint32_t x) {
    uint32_t r;
    asm volatile("v_xor_b32 %0, 64, %1" : "=v"(r) : "v"(x));
    return r;
  };

  constexpr int KS = EPI == 0 ? 1 : 2;
  float sacc[2][4][KS];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int k = 0; k < KS; ++k) sacc[i][r][k] = 0.f;

  float* const cfl = (float*)(smem + kLds);
  if constexpr (EPI >= 2) {  // published by the prologue barrier
    if (tid < 256) cfl[tid] = a.bn_coef1[SL ? (tid >> 6) * a.coef_ld + (tid & 63) : tid];
  }
  if constexpr (PRE) {
    if (tid < 128) cfl[tid] = a.pre_coef[tid];  // scale[64] | shift[64]
    __syncthreads();                            // the prologue transform reads them
  }
  // coefficient q of channels wn*32 + 8*fq + 4*h .. +3
  auto coef = [&](int q, int h) { return *(const float4*)(cfl + q * 64 + wn * 32 + 8 * fq + 4 * h); };

  f32x4_t acc[2][NJ];
  // epilogue operands of the tile being computed: loaded at the start of its compute phase (latency hidden
  // under the MFMAs), pinned complete at its end
  // epilogue operands (residual, BN input, ReLU mask) are loaded at the start of the memory phase, see memphase
  // EPI 3 (block-output BN-backward: residual + BN input + ReLU mask, 5 operand loads per pixel group) holds the
  // operands of at most NJO = 4 groups at once: all 7 would spill (~70 registers beside the accumulators), so its
  // epilogue runs in two halves (groups 0-3, then 4-6), each with its own operand loads (see memphase)
  constexpr int NJO = EPI == 3 ? 4 : NJ;
  u32x4v pre_res[RES ? NJO : 1], pre_y1[EPI >= 2 ? NJO : 1];
  u32x2v pre_m[EPI == 3 ? NJO : 1];
  // a tile's 4 x 56 output pixels are one contiguous block: pixel px of tile t is element (t's first pixel + px) * ldo
  const int lpx0 = pix_of_lane(fr) * ldo;
  int lpx = lpx0;  // re-opaqued per use site (see stage_tile)
  auto obase_of = [&](int t, int j) {
    const int n = t / TH, h0 = (t - n * TH) * 4;
    return (int64_t)(n * a.H + h0) * (kW * ldo) + (lpx + (wm * NJ + j) * 16 * ldo);
  };

  auto compute = [&](int t) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    vec8 af[2][2], bf[2][NJ];
    auto load = [&](int st, int sl) {
      const int tap = st >> 1, kk = st & 1;
      const int tr = tap / 3, tu = tap % 3;
      const int wtap = FLIP ? 8 - tap : tap;
      const int dR = tr * kXP + tu;
#pragma unroll
      for (int i = 0; i < 2; ++i)
        af[sl][i] = *(const vec8*)(smem + (kk ? abase1 : abase0) + i * 4 * 1152 + wtap * 128);
      // (volatile xor: computed here, not hoisted out of the tile loop as 49 more live registers)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        bf[sl][j] = *(const vec8*)(smem + (kk ? xor64(baddr[j][tu]) : baddr[j][tu]) + dR * 128);
    };
    __builtin_amdgcn_s_setprio(1);
    load(0, 0);
#pragma unroll
    for (int st = 0; st < 18; ++st) {
      if (st + 1 < 18) load(st + 1, (st + 1) & 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = E::mfma16x16x32(af[st & 1][i], bf[st & 1][j], acc[i][j]);
      __builtin_amdgcn_sched_barrier(0);
    }
    __builtin_amdgcn_s_setprio(0);
  };

  // epilogue: lane holds couts wn*32 + 8*fq + 4*i + r of pixel (wm*7 + j)*16 + pix_of_lane(fr); exactly
  // NJ = 7 16-byte stores per lane (every pixel of a tile is in range: H % 4 == 0)
  constexpr int kStores = NJ;
  // HOLD: the packed outputs go to held[j - J0] instead of memory (stored later by store_held)
  uint4 held[NJO];
  auto epilogue = [&](int t, auto J0c, auto J1c, auto HOLDc) {  // pixel groups [J0, J1); operands in pre_*[j - J0]
    constexpr int J0 = decltype(J0c)::value, J1 = decltype(J1c)::value;
    constexpr bool HOLD = decltype(HOLDc)::value;
    (void)held;
    (void)pre_m; (void)pre_res; (void)pre_y1;
    lpx = lpx0;
    asm volatile("" : "+v"(lpx));
    const int c0 = wn * 32 + 8 * fq;
#pragma unroll
    for (int j = J0; j < J1; ++j) {
      const int jo = j - J0;
      const int64_t ob = obase_of(t, j);
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = acc[e >> 2][j][e & 3];
      if constexpr (RES) {
        const u32x4v rr = pre_res[jo];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += E::to_f((uint16_t)(rr[e >> 1] >> (16 * (e & 1))));
      }
      float y1[8];
      if constexpr (EPI >= 2) {
        const u32x4v q1 = pre_y1[jo];
#pragma unroll
        for (int e = 0; e < 8; ++e) y1[e] = E::to_f((uint16_t)(q1[e >> 1] >> (16 * (e & 1))));
        if constexpr (EPI == 2) {
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const float4 sc = coef(0, h), sh = coef(1, h);
            const float scv[4] = {sc.x, sc.y, sc.z, sc.w}, shv[4] = {sh.x, sh.y, sh.z, sh.w};
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (!(y1[4 * h + r] * scv[r] + shv[r] > 0.f)) v[4 * h + r] = 0.f;
          }
        } else {
          const uint32_t mb = c0 < 32 ? pre_m[jo][0] >> c0 : pre_m[jo][1] >> (c0 - 32);
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (!((mb >> e) & 1u)) v[e] = 0.f;
        }
      }
      uint4 packed;  // one v_cvt_pk_bf16_f32 per pair (E16::pack2)
      packed.x = E::pack2(v[0], v[1]);
      packed.y = E::pack2(v[2], v[3]);
      packed.z = E::pack2(v[4], v[5]);
      packed.w = E::pack2(v[6], v[7]);
      uint16_t o[8];
      unpack8(packed, o);
      if constexpr (HOLD)
        held[jo] = packed;
      else
        *(uint4*)(a.y + ob + c0) = packed;
      if constexpr (EPI == 1) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float q = E::to_f(o[e]);
          sacc[e >> 2][e & 3][0] += q;
          sacc[e >> 2][e & 3][1] += q * q;
        }
      } else if constexpr (EPI >= 2) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const float4 mu = coef(2, h), is = coef(3, h);
          const float m1[4] = {mu.x, mu.y, mu.z, mu.w}, i1[4] = {is.x, is.y, is.z, is.w};
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float dz = E::to_f(o[4 * h + r]);
            sacc[h][r][0] += dz;
            sacc[h][r][1] += dz * (y1[4 * h + r] - m1[r]) * i1[r];
          }
        }
      }
      __builtin_amdgcn_sched_barrier(0);  // one pixel group at a time: bounded epilogue temporaries
    }
  };

  auto store_held = [&](int t, auto J0c, auto J1c) {
    constexpr int J0 = decltype(J0c)::value, J1 = decltype(J1c)::value;
    lpx = lpx0;
    asm volatile("" : "+v"(lpx));
#pragma unroll
    for (int j = J0; j < J1; ++j) {
      const int64_t ob = obase_of(t, j);
      *(uint4*)(a.y + ob + wn * 32 + 8 * fq) = held[j - J0];
    }
  };

  // memory phase of a group: DMA of tile k_dma into its (just read) buffer first, then the epilogue of tile
  // k_epi under it, then wait for this wave's DMA only (the epilogue's stores are the kStores youngest
  // vector-memory operations) and, PRE, transform the chunks this wave DMA'd.
  // Epilogue operands of tile k_epi: asm buffer loads (uncounted by the compiler), waited for with counted vmcnt and
  // pinned by "+v" operands; one 32-bit offset per pixel group (the channel block is an immediate), not 14 pointers.
  auto load_ops = [&](int t, auto J0c, auto J1c) {
    constexpr int J0 = decltype(J0c)::value, J1 = decltype(J1c)::value;
    (void)pre_m; (void)rmask; (void)pre_res; (void)rres; (void)pre_y1; (void)ry1;  // (generic lambda: capture them)
    const int n = t / TH, h0 = (t - n * TH) * 4;
    const uint32_t tb = (uint32_t)(n * a.H + h0) * (kW * (uint32_t)ldo);  // tile's first element (< 2^31: 4 GB)
    lpx = lpx0;
    asm volatile("" : "+v"(lpx));
#pragma unroll
    for (int j = J0; j < J1; ++j) {
      const int jo = j - J0;
      const uint32_t e = tb + (uint32_t)(lpx + (wm * NJ + j) * 16 * ldo);
      const uint32_t yo = (e + wn * 32 + 8 * fq) * 2u;
      if constexpr (RES)
        asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(pre_res[jo]) : "v"(yo), "s"(rres));
      if constexpr (EPI >= 2)
        asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(pre_y1[jo]) : "v"(yo), "s"(ry1));
      if constexpr (EPI == 3)
        asm volatile("buffer_load_dwordx2 %0, %1, %2, 0 offen" : "=v"(pre_m[jo]) : "v"(e >> 3), "s"(rmask));
    }
  };
  auto pin_ops = [&](auto NOc) {  // after the covering wait: no use of the operands may be scheduled ahead of it
    constexpr int NO = decltype(NOc)::value;
    (void)pre_m; (void)pre_res; (void)pre_y1;
#pragma unroll
    for (int jo = 0; jo < NO; ++jo) {
      if constexpr (RES) asm volatile("" : "+v"(pre_res[jo]));
      if constexpr (EPI >= 2) asm volatile("" : "+v"(pre_y1[jo]));
      if constexpr (EPI == 3) asm volatile("" : "+v"(pre_m[jo]));
    }
  };
  using I0 = std::integral_constant<int, 0>;
  using IH = std::integral_constant<int, NJO>;
  using IN = std::integral_constant<int, NJ>;
  auto memphase = [&](int k_epi, int k_dma) {
    constexpr bool OPS = RES || EPI >= 2;
    const int te = first + k_epi * per_x;
    if constexpr (OPS) {
      if (k_epi >= 0) load_ops(te, I0{}, IH{});  // ahead of the DMA: waited for with the DMA still in flight
    }
    if (k_dma >= 0) stage_tile(first + k_dma * per_x);
    if constexpr (OPS) {
      if (k_epi >= 0) {
        if (k_dma >= 0)
          asm volatile("s_waitcnt vmcnt(11)" ::: "memory");  // the 11 DMA pieces are the youngest
        else
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        pin_ops(IH{});
      }
    }
    if constexpr (NJO < NJ) {
      // EPI 3, two halves: groups 0-3 computed into registers (held, not stored yet), the operands of groups 4-6
      // loaded into the freed operand registers, THEN the first half's 4 stores: the second half's loads are older
      // than those stores, so vmcnt(4) waits for the loads (and the DMA) without draining the stores
      if (k_epi >= 0) {
        epilogue(te, I0{}, IH{}, std::true_type{});
        load_ops(te, IH{}, IN{});
        __builtin_amdgcn_sched_barrier(0);
        store_held(te, I0{}, IH{});
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        pin_ops(std::integral_constant<int, NJ - NJO>{});
        epilogue(te, IH{}, IN{}, std::false_type{});
      }
      if (k_dma >= 0 && k_epi < 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      // (PRE never combines with EPI 3)
    } else {
      if (k_epi >= 0) epilogue(te, I0{}, IN{}, std::false_type{});
      if (k_dma >= 0) {
        if (k_epi >= 0)
          __builtin_amdgcn_s_waitcnt((kStores & 0xF) | ((kStores >> 4) << 14) | (0x7 << 4) | (0xF << 8));
        else
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if constexpr (PRE) transform(first + k_dma * per_x);
      }
    }
  };
  auto phase_barrier = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  // prologue: group g stages the block's tile g
  if (grp < nk) stage_tile(first + grp * per_x);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's weight pieces and halo pieces
  if constexpr (PRE) {
    if (grp < nk) transform(first + grp * per_x);
  }
  phase_barrier();
  // phase p: the group with grp == p & 1 computes tile p; the other one finishes tile p - 1 and stages tile p + 1
  // (tile 1 was staged by the prologue).  The phase count is block-uniform: every wave passes the same barriers.
  const int nphase = 2 * ((nk + 1) >> 1) + 1;
  for (int p = 0; p < nphase; ++p) {
    if ((p & 1) == grp) {
      if (p < nk) compute(first + p * per_x);
    } else {
      const int ke = p - 1 < nk ? p - 1 : -1;  // p - 1 < 0 -> -1 as well
      const int kd = p >= 1 && p + 1 < nk ? p + 1 : -1;
      if (ke >= 0 || kd >= 0) memphase(ke, kd);
    }
    if (p + 1 < nphase) phase_barrier();
  }

  if constexpr (EPI > 0) {
    // block totals: DPP row scan over the 16 pixel lanes, then the 8 waves through LDS (group 0's halo
    // buffer is free once every wave passed the barrier below), summed in a fixed order per channel
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int k = 0; k < KS; ++k) sacc[i][r][k] = row16_sum(sacc[i][r][k]);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();
    float* red = (float*)(smem + kWB);  // [8 waves][32 channels][2]
    if (fr == 15) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int lc = 8 * fq + 4 * i + r;
          red[(wave * 32 + lc) * 2 + 0] = sacc[i][r][0];
          red[(wave * 32 + lc) * 2 + 1] = sacc[i][r][1];
        }
    }
    __syncthreads();
    if (tid < 128) {
      const int c = tid >> 1, k = tid & 1, cn = c >> 5, lc = c & 31;
      float s = 0.f;
#pragma unroll
      for (int g = 0; g < 2; ++g)
#pragma unroll
        for (int m = 0; m < 2; ++m) s += red[((g * 4 + m * 2 + cn) * 32 + lc) * 2 + k];
      a.srows[(int64_t)blockIdx.x * 128 + tid] = s;
    }
  }
}

static int g_conv_l1_pp = -1;  // -1: PDT_CONV_L1_PP decides; 0 / 1: set by conv_l1_set_pp (tests, A/B)
// PDT_CONV_L1_PP=0: the 4-wave kernel everywhere (A/B)
static bool conv_l1_pp_on() {
  static const bool pp_env = [] {
    const char* e = getenv("PDT_CONV_L1_PP");
    return !(e && e[0] == '0');
  }();
  return g_conv_l1_pp >= 0 ? g_conv_l1_pp != 0 : pp_env;
}

// strided operands (a channel slice of a grouped conv's wider tensors)
static bool conv_l1_sliced(const ConvFwdArgs& a) {
  return a.cs != 64 || (a.ldy && a.ldy != 64) || (a.coef_ld && a.coef_ld != 64) || a.stats_ld;
}

bool conv_l1_eligible(const ConvFwdArgs& a, int* flip) {
  // H % 4 == 0: whole 4-row tiles only (the epilogue has no per-pixel range checks; see conv_l1_kernel)
  if (a.C != 64 || a.Kout != 64 || a.W != kW || a.OW != kW || a.bnb == 3 || a.H % 4 != 0) return false;
  if (conv_l1_sliced(a)) {
    // a 64-channel slice of wider tensors (grouped convs): the 8-wave kernel's SL form -- forward (with or without
    // statistics) or backward data (with or without the inner-BN reduce), no residual / producer BN
    if (!conv_l1_pp_on() || a.res || a.pre_coef || a.nslice > 1 || a.bnb > 1) return false;
    if (a.cs % 8 != 0 || a.ldy % 8 != 0 || a.cs < 64 || a.ldy < 64) return false;
  }
  if (a.nphase == 0) {
    if (a.T == 3 && a.U == 3 && a.ist_h == 1 && a.ist_w == 1 && a.ioff_h == -1 && a.ioff_w == -1 &&
        a.tstep_h == 1 && a.tstep_w == 1 && a.ost_h == 1 && a.ost_w == 1 && a.ooff_h == 0 && a.ooff_w == 0 &&
        a.Pm == a.H && a.Qm == kW && a.OH == a.H) {
      *flip = 0;
      return true;
    }
    return false;
  }
  // single-phase backward-data of a stride-1 3x3 conv: in = i + 1 - t (taps flipped)
  if (a.nphase == 1 && a.pT[0] == 3 && a.pU[0] == 3 && a.pioff_h[0] == 1 && a.pioff_w[0] == 1 &&
      a.tstep_h == -1 && a.tstep_w == -1 && a.ist_h == 1 && a.ist_w == 1 && a.ost_h == 1 && a.ost_w == 1 &&
      a.pooff_h[0] == 0 && a.pooff_w[0] == 0 && a.pPm[0] == a.H && a.pQm[0] == kW && a.OH == a.H) {
    *flip = 1;
    return true;
  }
  return false;
}


int conv_l1_set_pp(int mode) {
  const int old = g_conv_l1_pp;
  g_conv_l1_pp = mode;
  return old;
}

void conv_l1_launch(const ConvFwdArgs& args, int flip, int dtype, hipStream_t s) {
  ConvFwdArgs a = args;
  if (a.nphase == 1) a.w = args.w + args.pwoff[0];
  int dev = 0, cus = 256;
  PDT_HIP_CHECK(hipGetDevice(&dev));
  PDT_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const int tiles = a.N * ((a.H + 3) / 4);
  int G = (cus + 7) / 8 * 8;
  const int cap = (tiles + 7) / 8 * 8;
  if (G > cap) G = cap;
  const bool rs = a.res != nullptr;
  const int epi = a.bnb ? a.bnb + 1 : (a.stats != nullptr ? 1 : 0);
  if (a.pre_coef && (epi != 1 || rs || flip))
    pdt_hip_fail("conv_l1: the fused producer BN (pre_coef) needs a forward conv with statistics, no residual",
                 hipErrorInvalidValue, __FILE__, __LINE__);
  if (a.pre_coef) PDT_COUNT("conv_l1_fwd_fused_bn_relu");
  // The 8-wave ping-pong kernel takes every variant except the block-output BN-backward epilogue (EPI 3: residual +
  // BN input + ReLU mask operands do not fit its 256 registers without spilling), which stays on the 4-wave kernel.
  const bool pp_on = conv_l1_pp_on();
  const bool pp = pp_on && (epi == 0 || (epi == 1 && !rs && !flip) || (epi == 2 && !rs) || (epi == 3 && rs));
  if (pp) PDT_COUNT("conv_l1_pp");
  const bool sl = conv_l1_sliced(a);
  if (sl && !(pp && !rs && !a.pre_coef && epi <= 2))
    pdt_hip_fail("conv_l1: sliced operands need the 8-wave kernel, EPI 0-2, no residual", hipErrorInvalidValue,
                 __FILE__, __LINE__);
  if (sl) PDT_COUNT("conv_l1_sliced");
  Scratch part(a.stats ? (size_t)G * 128 * sizeof(float) : 0, s);
  a.srows = part.as<float>();
  const dim3 grid(G);
#define PDT_L1OLD(DT_, E_, R_, P_) hipLaunchKernelGGL((conv_l1_kernel<DT_, E_, R_, P_>), grid, dim3(256), 0, s, a, flip)
#define PDT_L1PP(DT_, E_, R_, P_, F_) hipLaunchKernelGGL((conv_l1pp_kernel<DT_, E_, R_, P_, F_>), grid, dim3(512), 0, s, a)
#define PDT_L1SL(DT_, E_, F_) hipLaunchKernelGGL((conv_l1pp_kernel<DT_, E_, false, false, F_, true>), grid, dim3(512), 0, s, a)
#define PDT_L1_DT(DT_)                                                                                   \
  if (sl) {                                                                                              \
    if (epi == 0) { if (flip) PDT_L1SL(DT_, 0, true); else PDT_L1SL(DT_, 0, false); }                    \
    else if (epi == 1) PDT_L1SL(DT_, 1, false);                                                          \
    else if (flip) PDT_L1SL(DT_, 2, true);                                                               \
    else PDT_L1SL(DT_, 2, false);                                                                        \
  } else if (pp) {                                                                                       \
    if (epi == 0 && !rs) { if (flip) PDT_L1PP(DT_, 0, false, false, true); else PDT_L1PP(DT_, 0, false, false, false); } \
    else if (epi == 0) { if (flip) PDT_L1PP(DT_, 0, true, false, true); else PDT_L1PP(DT_, 0, true, false, false); }    \
    else if (epi == 1) { if (a.pre_coef) PDT_L1PP(DT_, 1, false, true, false); else PDT_L1PP(DT_, 1, false, false, false); } \
    else if (epi == 2) { if (flip) PDT_L1PP(DT_, 2, false, false, true); else PDT_L1PP(DT_, 2, false, false, false); } \
    else { if (flip) PDT_L1PP(DT_, 3, true, false, true); else PDT_L1PP(DT_, 3, true, false, false); }                  \
  } else if (epi == 0 && !rs) PDT_L1OLD(DT_, 0, false, false);                                            \
  else if (epi == 0 && rs) PDT_L1OLD(DT_, 0, true, false);                                               \
  else if (epi == 1 && !rs && a.pre_coef) PDT_L1OLD(DT_, 1, false, true);                                \
  else if (epi == 1 && !rs) PDT_L1OLD(DT_, 1, false, false);                                             \
  else if (epi == 2 && !rs) PDT_L1OLD(DT_, 2, false, false);                                             \
  else if (epi == 3 && rs) PDT_L1OLD(DT_, 3, true, false);                                               \
  else pdt_hip_fail("conv_l1: unsupported epilogue variant", hipErrorInvalidValue, __FILE__, __LINE__);
  if (dtype == kBF16) {
    PDT_L1_DT(kBF16)
  } else {
    PDT_L1_DT(kF16)
  }
#undef PDT_L1_DT
#undef PDT_L1SL
#undef PDT_L1PP
#undef PDT_L1OLD
  if (a.stats) stat_rows_reduce_launch(a.srows, G, 128, a.stats, s, a.stats_ld);
}

}  // namespace pdt
