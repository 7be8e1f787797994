// Implicit-GEMM convolution on MFMA (gfx950), NHWC activations, [Cout][taps][Cin] weights.
//
// One kernel serves three roles:
//   * forward conv:        out(n,i,j,k) = sum_{t,u,c} X(n, i*s-p+t, j*s-p+u, c) * W(k,t,u,c)
//   * backward-data conv:  one launch per sub-pixel phase of the stride; the phase's taps form a
//                          small stride-1 conv over dY with flipped weights, written to the
//                          phase's output sub-grid (no MFMA work is wasted on structural zeros)
//   * linear layers:       a 1x1 "conv" over [B,1,1,K]
// ``cs`` is the element stride between input pixels (== C, except for the ResNet stem's "window" mode,
// where X is the zero-padded NHWC4 image and one 32-wide reduction chunk spans 8 pixels x 4 channels
// of a kernel row, so the 7x7/2 stem runs with no im2col buffer).  With C == 64 ("window-pair" mode)
// one 64-wide chunk covers TWO consecutive kernel rows (chunks 0..3 row h, chunks 4..7 row h+1), so the
// stem runs 4 BK=64 steps instead of 7 BK=32 steps.
// The generalised geometry is
//   in_h  = i*ist_h + ioff_h + t*tstep_h      (t in [0,T)),  same for w / u
//   out_h = i*ost_h + ooff_h
// GEMM view: D[n=cout][m=pixel] = sum_k Wt[n][k] * X[m][k]; MFMA A = weights, B = activations, so a
// lane's accumulator holds 4 consecutive output channels of one pixel (8-byte NHWC stores).
//
// Tiles are staged global->LDS with LDS-DMA (global_load_lds_dwordx4, 16 B/lane) into two LDS
// buffers (buffer_load ... lds); out-of-bounds rows (padding, M tail) read zeros through the buffer
// resource range check.  The LDS image is linear per
// wave-instruction and XOR-swizzled through the SOURCE address (chunk ^= (row>>1)&(chunks-1)), which
// makes the ds_read_b128 fragment reads bank-conflict free.  Optional epilogues: residual add (used
// to fuse the identity-gradient add of a residual block into dgrad) and per-channel BatchNorm
// statistics (sum, sum of squares of the rounded outputs), reduced per block and written with plain stores to
// the block's own partial row, then summed in a fixed order by stat_rows_reduce into kStatSlots slots
// (deterministic, no atomics; conv_fwd.h) -- so no separate statistics pass over the output.
#include <cstdlib>

#include "../common.h"
#include "conv_fwd.h"
#include "conv_l1.h"

namespace pdt {

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void glb_void;

template <int CHUNKS>
PDT_DEVICE int swz(int row) { return (row >> 1) & (CHUNKS - 1); }

// Shared epilogue of the implicit-GEMM conv kernels: the wave's accumulators acc[i][j] hold output
// channels n = n0 + wn*WN + i*16 + 4*fq + r of pixel m = m0 + wm*WM + j*16 + fr.
// RES: 0 no residual | 1 residual in the output's layout | 2 compact residual of sub-pixel phase a.res_phase
// (ConvFwdArgs::res_phase), indexed by GEMM row; its loads stay unconditional (in range on every phase) and
// only the add is selected, so the hoisted-load structure of the RES == 1 path is kept.
// SMEM > 0 (the kernel's LDS bytes): with a.stage_out the output tile is staged in LDS and written back as
// whole 16-byte-per-lane rows; a lane's accumulators otherwise hold 4 channels of one pixel, so every store
// instruction writes 16 rows x 32 B.
// PERM (conv_pp_kernel: its weight rows are staged permuted): fragment i row 4*fq + r is channel
// wn*WN + (i >> 1)*32 + 8*fq + 4*(i & 1) + r, so fragments 2p and 2p+1 give a lane 8 CONSECUTIVE channels of its pixel
// -- one 16-byte operand load / store (staged or not) per pair instead of two 8-byte ones.  Round 5, same box:
// ResNet-18 20.66/20.69/20.68 -> 20.53/20.58/20.51 ms, ResNet-50 74.05/74.04 -> 73.64/73.42 ms (an earlier variant
// with 8-byte staged writes at the permuted offsets was 0.1 ms SLOWER on ResNet-18: LDS write conflicts).
template <int DT, int EPI, int RES, int FN, int FM, int WN, int WM, int BN, int WAVES_M, int NW_, int SMEM = 0,
          bool PERM = false>
PDT_DEVICE void conv_epilogue(const ConvFwdArgs& a, f32x4_t (&acc)[FN][FM], int64_t m0, int n0, int tile_m, int wn,
                              int wm, int tid, int lane, char* smem) {
  using E = E16<DT>;
  const int fr = lane & 15, fq = lane >> 4;
  const int PQ = a.Pm * a.Qm;
  const FastDiv fd_pq{a.pq_mul, a.pq_shift}, fd_q{a.q_mul, a.q_shift};
  // ---- epilogue: lane holds channels n = n0 + wn*WN + i*16 + 4*fq + r of pixel m ----
  // EPI: 0 plain | 1 forward BN statistics (sum, sumsq of the rounded outputs) | 2..4 BN-backward
  // reduce of the consumer BatchNorm fused into this (backward-data) conv: the output written is
  // dz = v * relu'(.), and per channel sum(dz), sum(dz * xhat) accumulate (2: ReLU mask recomputed from
  // the BN input y1 and its forward coefficients; 3: mask = (block output > 0); 4: as 3 plus a second
  // BN branch y2 sharing dz, e.g. a residual block's downsample BN).
  constexpr int KS = EPI == 0 ? 0 : (EPI == 4 ? 3 : 2);  // accumulated quantities per channel
  float sacc[FN][4][KS > 0 ? KS : 1];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int k = 0; k < (KS > 0 ? KS : 1); ++k) sacc[i][r][k] = 0.f;

  // Per-channel BN coefficients of the fused BN-backward epilogues, staged once per block in LDS (free after
  // the main loop; placed behind the statistics scratch) and read back as float4 per channel fragment:
  // registers would cost 32-64 VGPRs per lane, global reloads would be serialised behind the stores.
  // Layout [quantity][BN]: 0 scale, 1 shift, 2 mean, 3 invstd (branch 1); 4 mean, 5 invstd (branch 2).
  constexpr int RED_BYTES = WAVES_M * BN * 3 * 4;
  float* cf = (float*)(smem + RED_BYTES);
  const int64_t LDY = a.ldy ? a.ldy : a.Kout;  // output pixel stride (channel slices of a wider tensor)
  if constexpr (EPI >= 2) {
    const int CL = a.coef_ld ? a.coef_ld : a.Kout;
    for (int c = tid; c < BN; c += NW_ * 64) {
      const int n = n0 + c;
      cf[0 * BN + c] = a.bn_coef1[n];
      cf[1 * BN + c] = a.bn_coef1[CL + n];
      cf[2 * BN + c] = a.bn_coef1[2 * CL + n];
      cf[3 * BN + c] = a.bn_coef1[3 * CL + n];
      if constexpr (EPI == 4) {
        cf[4 * BN + c] = a.bn_coef2[2 * CL + n];
        cf[5 * BN + c] = a.bn_coef2[3 * CL + n];
      }
    }
    __syncthreads();
  }
  // channel of fragment i, row 4*fq + r, within the wave's WN (PERM: see above)
  auto chan = [&](int i, int r) { return PERM ? (i >> 1) * 32 + 8 * fq + 4 * (i & 1) + r : i * 16 + 4 * fq + r; };
  static_assert(!PERM || FN % 2 == 0, "PERM pairs fragments");
  auto coef4 = [&](int q, int i) { return *(const float4*)(cf + q * BN + wn * WN + chan(i, 0)); };

  // Two-phase chunks of JC pixel fragments: every epilogue operand load of the chunk (residual, BN input(s),
  // ReLU mask) is issued before any arithmetic or store, so the chunk pays ONE memory latency instead of
  // one per (pixel fragment, channel fragment) -- the stores could alias the operands as far as the
  // compiler knows, so it would not hoist them itself.  Out-of-range pixels (M tail) load from pixel 0.
  constexpr bool LY1 = EPI >= 2, LY2 = EPI == 4, LM = EPI == 3 || EPI == 4;
  // ReLU bitmask: one 8-byte load per pixel and 64 channels (the wave's WN channels are whole 64-bit words);
  // a byte load per fragment, shifted right away, made the compiler wait for each one as it was issued
  static_assert(!LM || WN % 64 == 0, "bitmask epilogue needs 64-channel wave columns");
  constexpr int MW = LM ? WN / 64 : 1;
  // registers per pixel fragment of hoisted operands; chunk size keeps them within the budget left
  // beside the accumulators (FN*FM*4) and the statistics accumulators (beyond two per channel: EPI 4
  // keeps three) so no variant spills or loses occupancy
  constexpr int PER_J = FN * (2 * (RES != 0) + 2 * LY1 + 2 * LY2) + (LM ? 2 * MW : 0);
  constexpr int BUDGET = (FN * FM * 4 >= 128 ? 64 : 96) - (KS > 2 ? FN * 4 * (KS - 2) * 2 : 0);
  constexpr int JC = PER_J == 0 ? FM
                     : (8 * PER_J <= BUDGET && FM % 8 == 0) ? 8
                     : (4 * PER_J <= BUDGET && FM % 4 == 0) ? 4
                     : (2 * PER_J <= BUDGET && FM % 2 == 0) ? 2 : 1;
  static_assert(FM % JC == 0, "epilogue chunking");
  constexpr int BM_T = WAVES_M * WM;
  constexpr int SPITCH = BN * 2 + 16;  // staged row pitch (+16 B: consecutive rows rotate by 4 banks)
  constexpr int STG_OFF = 16384;       // behind the statistics scratch and the BN coefficients
  // the whole tile staged at once, or -- when only one wave row-group's WM x BN slice fits (the 256 x 256 ping-pong
  // tile: 128 KB of LDS) -- one pass per wave row-group: its waves stage, then every wave writes those rows back
  constexpr bool FULL = SMEM >= STG_OFF + BM_T * SPITCH;
  constexpr bool PERGRP = !FULL && WAVES_M > 1 && EPI != 2 && SMEM >= STG_OFF + WM * SPITCH;  // (EPI 2: spills)
  constexpr bool CAN_STAGE = FULL || PERGRP;
  static_assert(!CAN_STAGE || RED_BYTES + 6 * BN * 4 <= STG_OFF, "epilogue LDS regions overlap");
  const bool stage = CAN_STAGE && a.stage_out;
  char* stg = smem + STG_OFF;
  const int srow0 = FULL ? wm * WM : 0;  // this wave's first row in the staging buffer
  constexpr bool RC = RES == 2;
  const bool res_on = !RC || (int)blockIdx.y == a.res_phase;  // compact: this block's phase owns the residual
  // write the staged rows of wave row-group g (PERGRP) or of the whole tile (FULL) back: 16 B per lane, whole
  // BN-channel rows per pixel
  auto copy_rows = [&](int g) {
    constexpr int CPR = BN / 8;
    constexpr int SROWS = FULL ? BM_T : WM;
    for (int q = tid; q < SROWS * CPR; q += NW_ * 64) {
      const int row = q / CPR, ch = q - row * CPR;
      const int64_t m = m0 + (FULL ? 0 : g * WM) + row;
      if (m < a.M) {
        const int mm = (int)m;
        const int nimg = (int)fdiv((uint32_t)mm, fd_pq);
        const int rem = mm - nimg * PQ;
        const int i_ = (int)fdiv((uint32_t)rem, fd_q), j_ = rem - i_ * a.Qm;
        const int oh = i_ * a.ost_h + a.ooff_h, ow = j_ * a.ost_w + a.ooff_w;
        const int64_t ob = (((int64_t)nimg * a.OH + oh) * a.OW + ow) * LDY + n0 + ch * 8;
        *(uint4*)(a.y + ob) = *(const uint4*)(stg + row * SPITCH + ch * 16);
      }
    }
  };
  // PERGRP: row-group g stages its slice while the groups before it are written back (each wave runs its own
  // fragment loop once, and every wave passes 2 x WAVES_M barriers)
  if constexpr (PERGRP) {
    if (stage)
      for (int g = 0; g < wm; ++g) {
        __syncthreads();
        copy_rows(g);
        __syncthreads();
      }
  }
#pragma unroll
  for (int jc = 0; jc < FM; jc += JC) {
    int64_t obase[JC];
    uint32_t rbase[RC ? JC : 1];
    bool valid[JC];
#pragma unroll
    for (int jj = 0; jj < JC; ++jj) {
      const int64_t m = m0 + wm * WM + (jc + jj) * 16 + fr;
      valid[jj] = m < a.M;
      const int mm = valid[jj] ? (int)m : 0;
      const int nimg = (int)fdiv((uint32_t)mm, fd_pq);
      const int rem = mm - nimg * PQ;
      const int i_ = (int)fdiv((uint32_t)rem, fd_q), j_ = rem - i_ * a.Qm;
      const int oh = i_ * a.ost_h + a.ooff_h, ow = j_ * a.ost_w + a.ooff_w;
      obase[jj] = (((int64_t)nimg * a.OH + oh) * a.OW + ow) * LDY;
      if constexpr (RC) rbase[jj] = (uint32_t)mm * (uint32_t)LDY;
    }
    uint2 p_res[RES ? JC : 1][RES ? FN : 1], p_y1[LY1 ? JC : 1][LY1 ? FN : 1], p_y2[LY2 ? JC : 1][LY2 ? FN : 1];
    uint64_t p_m[LM ? JC : 1][MW];
#pragma unroll
    for (int jj = 0; jj < JC; ++jj) {
      if constexpr (PERM) {  // one 16-byte load per fragment pair
#pragma unroll
        for (int i = 0; i < FN; i += 2) {
          const int64_t o = obase[jj] + n0 + wn * WN + chan(i, 0);
          auto split = [&](uint2 (&dst)[FN], const uint4 v) {
            dst[i] = make_uint2(v.x, v.y);
            dst[i + 1] = make_uint2(v.z, v.w);
          };
          if constexpr (RES == 1) split(p_res[jj], *(const uint4*)(a.res + o));
          if constexpr (RC) split(p_res[jj], *(const uint4*)(a.res + rbase[jj] + (uint32_t)(n0 + wn * WN + chan(i, 0))));
          if constexpr (LY1) split(p_y1[jj], *(const uint4*)(a.bn_y1 + o));
          if constexpr (LY2) split(p_y2[jj], *(const uint4*)(a.bn_y2 + o));
        }
      } else {
#pragma unroll
        for (int i = 0; i < FN; ++i) {
          const int64_t o = obase[jj] + n0 + wn * WN + i * 16 + 4 * fq;
          if constexpr (RES == 1) p_res[jj][i] = *(const uint2*)(a.res + o);
          if constexpr (RC) p_res[jj][i] = *(const uint2*)(a.res + rbase[jj] + (uint32_t)(n0 + wn * WN + i * 16 + 4 * fq));
          if constexpr (LY1) p_y1[jj][i] = *(const uint2*)(a.bn_y1 + o);
          if constexpr (LY2) p_y2[jj][i] = *(const uint2*)(a.bn_y2 + o);
        }
      }
      if constexpr (LM) {
#pragma unroll
        for (int g = 0; g < MW; ++g)
          p_m[jj][g] = *(const uint64_t*)(a.bn_mask + ((obase[jj] + n0 + wn * WN + g * 64) >> 3));
      }
    }
#pragma unroll
    for (int jj = 0; jj < JC; ++jj) {
      if (!valid[jj]) continue;
      const int j = jc + jj;
      uint2 held = make_uint2(0u, 0u);  // PERM: fragment 2p's packed output, stored with 2p + 1's
#pragma unroll
      for (int i = 0; i < FN; ++i) {
        const int n = n0 + wn * WN + chan(i, 0);
        const int64_t o = obase[jj] + n;
        float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
        if constexpr (RES) {
          uint2 rr = p_res[jj][i];
          if constexpr (RC) {
            rr.x = res_on ? rr.x : 0u;
            rr.y = res_on ? rr.y : 0u;
          }
          v[0] += E::to_f((uint16_t)(rr.x & 0xffff));
          v[1] += E::to_f((uint16_t)(rr.x >> 16));
          v[2] += E::to_f((uint16_t)(rr.y & 0xffff));
          v[3] += E::to_f((uint16_t)(rr.y >> 16));
        }
        float y1[4], y2[4];
        if constexpr (LY1) {
          const uint2 q1 = p_y1[jj][i];
          y1[0] = E::to_f((uint16_t)(q1.x & 0xffff)); y1[1] = E::to_f((uint16_t)(q1.x >> 16));
          y1[2] = E::to_f((uint16_t)(q1.y & 0xffff)); y1[3] = E::to_f((uint16_t)(q1.y >> 16));
          if constexpr (EPI == 2) {
            const float4 sc = coef4(0, i), sh = coef4(1, i);
            if (!(y1[0] * sc.x + sh.x > 0.f)) v[0] = 0.f;
            if (!(y1[1] * sc.y + sh.y > 0.f)) v[1] = 0.f;
            if (!(y1[2] * sc.z + sh.z > 0.f)) v[2] = 0.f;
            if (!(y1[3] * sc.w + sh.w > 0.f)) v[3] = 0.f;
          } else {
            const uint32_t mb = (uint32_t)(p_m[jj][chan(i, 0) >> 6] >> (chan(i, 0) & 63));
            if (!(mb & 1u)) v[0] = 0.f;
            if (!(mb & 2u)) v[1] = 0.f;
            if (!(mb & 4u)) v[2] = 0.f;
            if (!(mb & 8u)) v[3] = 0.f;
          }
        }
        if constexpr (LY2) {
          const uint2 q2 = p_y2[jj][i];
          y2[0] = E::to_f((uint16_t)(q2.x & 0xffff)); y2[1] = E::to_f((uint16_t)(q2.x >> 16));
          y2[2] = E::to_f((uint16_t)(q2.y & 0xffff)); y2[3] = E::to_f((uint16_t)(q2.y >> 16));
        }
        uint2 packed;  // one v_cvt_pk_bf16_f32 per pair (E16::pack2)
        packed.x = E::pack2(v[0], v[1]);
        packed.y = E::pack2(v[2], v[3]);
        const uint16_t ov[4] = {(uint16_t)packed.x, (uint16_t)(packed.x >> 16), (uint16_t)packed.y,
                                (uint16_t)(packed.y >> 16)};
        if (CAN_STAGE && stage) {
          if constexpr (PERM) {  // 16 B per pair: a pixel's 4 fq lanes write 64 contiguous bytes
            if (i & 1)
              *(uint4*)(stg + (srow0 + j * 16 + fr) * SPITCH + (wn * WN + chan(i, 0) - 4) * 2) =
                  make_uint4(held.x, held.y, packed.x, packed.y);
            else
              held = packed;
          } else {
            *(uint2*)(stg + (srow0 + j * 16 + fr) * SPITCH + (wn * WN + chan(i, 0)) * 2) = packed;
          }
        } else if constexpr (PERM) {
          if (i & 1)
            *(uint4*)(a.y + o - 4) = make_uint4(held.x, held.y, packed.x, packed.y);
          else
            held = packed;
        } else {
          *(uint2*)(a.y + o) = packed;
        }
        if constexpr (EPI == 1) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float q = E::to_f(ov[r]);
            sacc[i][r][0] += q;
            sacc[i][r][1] += q * q;
          }
        } else if constexpr (EPI >= 2) {
          const float4 mu = coef4(2, i), is = coef4(3, i);
          const float m1[4] = {mu.x, mu.y, mu.z, mu.w}, i1[4] = {is.x, is.y, is.z, is.w};
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float dz = E::to_f(ov[r]);
            sacc[i][r][0] += dz;
            sacc[i][r][1] += dz * (y1[r] - m1[r]) * i1[r];
          }
          if constexpr (EPI == 4) {
            const float4 mu2 = coef4(4, i), is2 = coef4(5, i);
            const float m2[4] = {mu2.x, mu2.y, mu2.z, mu2.w}, i2[4] = {is2.x, is2.y, is2.z, is2.w};
#pragma unroll
            for (int r = 0; r < 4; ++r) sacc[i][r][2] += E::to_f(ov[r]) * (y2[r] - m2[r]) * i2[r];
          }
        }
      }
    }
  }

  if constexpr (CAN_STAGE) {
    if (stage) {
      if constexpr (PERGRP) {
        for (int g = wm; g < WAVES_M; ++g) {
          __syncthreads();
          copy_rows(g);
          __syncthreads();
        }
      } else {
        __syncthreads();
        copy_rows(0);
      }
    }
  }

  if constexpr (KS > 0) {
    // reduce over the 16 lanes (pixels) that share fq (DPP row scan: lane fr == 15 holds the total),
    // then over the WAVES_M waves through LDS, then plain stores into this block's own partial row
    // (phase, M tile) of [rows][Kout][KO] (deterministic statistics, conv_fwd.h).
    constexpr int KO = EPI == 4 ? 4 : 2;  // stored quantities (EPI 4: sum dz is stored twice)
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int k = 0; k < KS; ++k) sacc[i][r][k] = row16_sum(sacc[i][r][k]);
    float* red = (float*)smem;  // [WAVES_M][BN][KS]
    __syncthreads();
    if (fr == 15) {
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int nl = wn * WN + chan(i, r);
#pragma unroll
          for (int k = 0; k < KS; ++k) red[(wm * BN + nl) * KS + k] = sacc[i][r][k];
        }
    }
    __syncthreads();
    if (tid < BN) {
      float t[KS];
#pragma unroll
      for (int k = 0; k < KS; ++k) t[k] = 0.f;
#pragma unroll
      for (int w = 0; w < WAVES_M; ++w)
#pragma unroll
        for (int k = 0; k < KS; ++k) t[k] += red[(w * BN + tid) * KS + k];
      const int64_t row = (a.nphase > 0 ? (int64_t)blockIdx.y * a.srows_pp : 0) + tile_m;
      const int64_t sld = a.nslice > 1 ? (int64_t)a.nslice * a.Kout : a.Kout;
      float* dst = a.srows + (row * sld + a.srows_coff + n0 + tid) * KO;
      if constexpr (EPI == 4)
        *(float4*)dst = make_float4(t[0], t[1], t[0], t[2]);
      else
        *(float2*)dst = make_float2(t[0], t[1]);
    }
  }
}

// Multi-phase launches size the grid for the largest phase; a block beyond its phase's tiles writes zeros
// into the statistics row slice it owns (row = phase * srows_pp + M tile), so the fixed-order row reduction
// never reads unwritten memory.
template <int EPI, int BN_>
PDT_DEVICE void zero_stat_row(const ConvFwdArgs& a, int nthreads) {
  if constexpr (EPI != 0) {
    constexpr int KO = EPI == 4 ? 4 : 2;
    const int tm = (int)blockIdx.x / a.n_tiles, tn = (int)blockIdx.x - tm * a.n_tiles;
    const int64_t sld = a.nslice > 1 ? (int64_t)a.nslice * a.Kout : a.Kout;
    float* dst = a.srows + (((int64_t)blockIdx.y * a.srows_pp + tm) * sld + a.srows_coff) * KO + (int64_t)tn * BN_ * KO;
    for (int i = threadIdx.x; i < BN_ * KO; i += nthreads) dst[i] = 0.f;
  }
}

template <int DT, int BM, int BN, int BK, int WAVES_N, int EPI, int RES, int STAGES, int NW>
// min 2 waves per SIMD where LDS allows two workgroups per CU: the BN-backward epilogue variants otherwise
// took > 256 registers and ran one workgroup per CU (half the 2-stage kernel's latency hiding)
__global__ __launch_bounds__(NW * 64, (STAGES * (BN + BM) * BK * 2 <= 81920 || NW == 8) ? 2 : 1)
void conv_fwd_kernel(ConvFwdArgs args) {
  ConvFwdArgs a = args;
  // (the kernel-argument struct itself is never written: a write makes the compiler copy it, with its dynamically
  // indexed phase arrays, to scratch -- 528 bytes per lane of spills, measured 65 % slower)
  const uint16_t* wbase = args.w;
  if (args.nslice > 1) {  // one launch over every channel slice of a grouped conv: this block's slice
    const int sl = blockIdx.z;
    a.x += (int64_t)sl * a.Kout;
    a.y += (int64_t)sl * a.Kout;
    wbase += (int64_t)sl * args.slice_wstride;
    a.w = wbase;
    if (a.bn_y1 != nullptr) a.bn_y1 += (int64_t)sl * a.Kout;
    if (a.bn_coef1 != nullptr) a.bn_coef1 += sl * a.Kout;
    a.srows_coff = sl * a.Kout;
  }
  if (args.nphase > 0) {  // multi-phase launch: this block's phase geometry (wave-uniform)
    const int ph = blockIdx.y;
    a.T = args.pT[ph]; a.U = args.pU[ph];
    a.ioff_h = args.pioff_h[ph]; a.ioff_w = args.pioff_w[ph];
    a.Pm = args.pPm[ph]; a.Qm = args.pQm[ph];
    a.ooff_h = args.pooff_h[ph]; a.ooff_w = args.pooff_w[ph];
    a.m_tiles = args.pmt[ph];
    a.M = (int64_t)a.N * a.Pm * a.Qm;
    a.w = wbase + args.pwoff[ph];
    a.pq_mul = args.ppq_mul[ph]; a.pq_shift = args.ppq_shift[ph];
    a.q_mul = args.pq1_mul[ph]; a.q_shift = args.pq1_shift[ph];
    if ((int)blockIdx.x >= a.m_tiles * a.n_tiles) {
      zero_stat_row<EPI, BN>(a, NW * 64);
      return;
    }
  }
  using E = E16<DT>;
  typedef typename E::vec8 vec8;
  constexpr int WAVES_M = NW / WAVES_N;
  constexpr int WN = BN / WAVES_N;
  constexpr int WM = BM / WAVES_M;
  constexpr int FN = WN / 16, FM = WM / 16;
  constexpr int ROWB = BK * 2;
  constexpr int CHUNKS = ROWB / 16;
  constexpr int RPI = 1024 / ROWB;               // rows per wave LDS-DMA instruction
  constexpr int A_INSTR = BN / RPI / NW;         // weight-tile instructions per wave
  constexpr int B_INSTR = BM / RPI / NW;         // activation-tile instructions per wave
  constexpr int A_BYTES = BN * ROWB;
  constexpr int STAGE = (BN + BM) * ROWB;
  static_assert(A_INSTR * RPI * NW == BN && B_INSTR * RPI * NW == BM, "tile/instr mismatch");
  __shared__ __attribute__((aligned(1024))) char smem[STAGES * STAGE];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wave % WAVES_N, wm = wave / WAVES_N;

  const int nwg = a.m_tiles * a.n_tiles;
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int tile_m = bid / a.n_tiles, tile_n = bid % a.n_tiles;
  const int64_t m0 = (int64_t)tile_m * BM;
  const int n0 = tile_n * BN;

  const int PQ = a.Pm * a.Qm;
  const FastDiv fd_pq{a.pq_mul, a.pq_shift}, fd_q{a.q_mul, a.q_shift};
  const int TU = a.T * a.U;
  const int csteps = a.C / BK;
  const int ksteps = TU * csteps;

  // ---- LDS-DMA sources: buffer resources over x and w; out-of-range byte offsets read zeros ----
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(a.x, (uint32_t)a.N * a.H * a.W * a.cs * 2u);
  const __amdgpu_buffer_rsrc_t rw = make_rsrc(a.w, (uint32_t)a.Kout * TU * a.C * 2u);

  // activation rows: per-lane (h0, w0) and byte offset of (image, h0, w0, chunk); the per-K-step
  // tap/channel displacement is wave-uniform and added per step
  const int lrow = lane / CHUNKS;      // row within one DMA instruction
  const int pchunk = lane % CHUNKS;    // physical (LDS) chunk this lane writes
  int brow_h[B_INSTR], brow_w[B_INSTR], brow_off[B_INSTR];
#pragma unroll
  for (int j = 0; j < B_INSTR; ++j) {
    const int row = (wave * B_INSTR + j) * RPI + lrow;
    const int64_t m = m0 + row;
    const int bch = pchunk ^ swz<CHUNKS>(row);
    if (m < a.M) {
      const int nimg = (int)fdiv((uint32_t)m, fd_pq);
      const int rem = (int)m - nimg * PQ;
      const int i = (int)fdiv((uint32_t)rem, fd_q), jj = rem - i * a.Qm;
      brow_h[j] = i * a.ist_h + a.ioff_h;
      brow_w[j] = jj * a.ist_w + a.ioff_w;
      const int pair = (CHUNKS == 8 && bch >= 4) ? a.pair_skip : 0;
      brow_off[j] = (((nimg * a.H + brow_h[j]) * a.W + brow_w[j]) * a.cs + bch * 8 + pair) * 2;
    } else {
      brow_h[j] = -(1 << 29);
      brow_w[j] = 0;
      brow_off[j] = 0;
    }
  }
  // PERM (conv_epilogue): LDS weight row wn*WN + 16*i + m holds channel wn*WN + (i >> 1)*32 + (m >> 2)*8 + 4*(i & 1) +
  // (m & 3), so fragment pairs give a lane 8 consecutive channels; the row swizzle stays a function of the LDS row
  constexpr bool PERM = WN % 32 == 0;
  uint32_t arow_off[A_INSTR];
#pragma unroll
  for (int j = 0; j < A_INSTR; ++j) {
    const int row = (wave * A_INSTR + j) * RPI + lrow;
    const int lw = row % WN, fi = lw >> 4, fm = lw & 15;
    const int ch = PERM ? row - lw + (fi >> 1) * 32 + (fm >> 2) * 8 + (fi & 1) * 4 + (fm & 3) : row;
    arow_off[j] = (uint32_t)(((n0 + ch) * TU * a.C + (pchunk ^ swz<CHUNKS>(row)) * 8) * 2);
  }

  // load cursor over (t, u, c0) in K-step order: advanced incrementally (no per-step divisions)
  int cur_t = 0, cur_u = 0, cur_c = 0;
  auto stage_load = [&](int buf) {
    const int t = cur_t, u = cur_u, c0 = cur_c;
    const int tap = t * a.U + u;
    cur_c += BK;
    if (cur_c == a.C) {
      cur_c = 0;
      if (++cur_u == a.U) { cur_u = 0; ++cur_t; }
    }
    char* sbase = smem + buf * STAGE;
    const uint32_t a_delta = (uint32_t)(tap * a.C + c0) * 2u;
#pragma unroll
    for (int j = 0; j < A_INSTR; ++j) buf_lds16(rw, sbase + (wave * A_INSTR + j) * 1024, arow_off[j] + a_delta);
    const int dh = t * a.tstep_h, dw = u * a.tstep_w;
    const int b_delta = ((dh * a.W + dw) * a.cs + c0) * 2;
#pragma unroll
    for (int j = 0; j < B_INSTR; ++j) {
      const int h = brow_h[j] + dh, w = brow_w[j] + dw;
      const bool ok = (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W;
      const uint32_t voff = ok ? (uint32_t)(brow_off[j] + b_delta) : kOOB;
      buf_lds16(rx, sbase + A_BYTES + (wave * B_INSTR + j) * 1024, voff);
    }
  };

  f32x4_t acc[FN][FM];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // fragment read offsets (bytes within a stage), per kk-independent part
  const int fr = lane & 15, fq = lane >> 4;
  int a_off[FN], b_off[FM];
#pragma unroll
  for (int i = 0; i < FN; ++i) a_off[i] = (wn * WN + i * 16 + fr) * ROWB;
#pragma unroll
  for (int j = 0; j < FM; ++j) b_off[j] = A_BYTES + (wm * WM + j * 16 + fr) * ROWB;

  auto compute_stage = [&](const char* sb) {
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      vec8 af[FN], bfr[FM];
#pragma unroll
      for (int i = 0; i < FN; ++i) {
        const int row = wn * WN + i * 16 + fr;
        const int ch = (kk * 4 + fq) ^ swz<CHUNKS>(row);
        af[i] = *(const vec8*)(sb + a_off[i] + ch * 16);
      }
#pragma unroll
      for (int j = 0; j < FM; ++j) {
        const int row = wm * WM + j * 16 + fr;
        const int ch = (kk * 4 + fq) ^ swz<CHUNKS>(row);
        bfr[j] = *(const vec8*)(sb + b_off[j] + ch * 16);
      }
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j) acc[i][j] = E::mfma16x16x32(af[i], bfr[j], acc[i][j]);
    }
  };

  if constexpr (STAGES == 2) {
    if (ksteps > 0) {
      stage_load(0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      for (int ks = 0; ks < ksteps; ++ks) {
        const int cur = ks & 1;
        if (ks + 1 < ksteps) stage_load(cur ^ 1);
        compute_stage(smem + cur * STAGE);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      }
    }
  } else {
    // S-stage LDS ring (S = 3 or 4): S-2 K-steps of LDS-DMA stay in flight across every barrier; each
    // iteration waits (counted vmcnt, never 0 while more are queued) only for the stage it is about to
    // read, then a raw s_barrier publishes it to all waves.  The buffer refilled in iteration ks was last
    // read in iteration ks-1, which every wave finished before passing this iteration's barrier.
    // MFMA clusters run at raised wave priority (s_setprio) so the issue of the next DMA / reads
    // interleaves with them instead of starving them.
    constexpr int S = STAGES;
    constexpr int PER_STAGE = A_INSTR + B_INSTR;  // LDS-DMA instructions per wave per stage
    auto wait_ahead = [&](int ahead) {             // vmcnt(ahead * PER_STAGE), immediate operands only
      constexpr int W1 = PER_STAGE, W2 = 2 * PER_STAGE;
      if (ahead >= 2)
        __builtin_amdgcn_s_waitcnt((W2 & 0xF) | ((W2 >> 4) << 14) | (0x7 << 4) | (0xF << 8));
      else if (ahead == 1)
        __builtin_amdgcn_s_waitcnt((W1 & 0xF) | ((W1 >> 4) << 14) | (0x7 << 4) | (0xF << 8));
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    };
    static_assert(S <= 4, "wait_ahead covers at most two stages in flight");
    if (ksteps > 0) {
#pragma unroll
      for (int p = 0; p < S - 1; ++p)
        if (p < ksteps) stage_load(p);
      int buf = 0;
      for (int ks = 0; ks < ksteps; ++ks) {
        const int ahead = min(S - 2, ksteps - 1 - ks);
        wait_ahead(ahead);
        __builtin_amdgcn_s_barrier();
        if (ks + S - 1 < ksteps) stage_load(buf == 0 ? S - 1 : buf - 1);
        __builtin_amdgcn_s_setprio(1);
        compute_stage(smem + buf * STAGE);
        __builtin_amdgcn_s_setprio(0);
        buf = buf == S - 1 ? 0 : buf + 1;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
  }

  conv_epilogue<DT, EPI, RES, FN, FM, WN, WM, BN, WAVES_M, NW, STAGES * STAGE, PERM>(a, acc, m0, n0, tile_m, wn, wm, tid,
                                                                             lane, smem);
}

// ----------------------------------------------------------------------------------------------
// "Ping-pong" implicit-GEMM conv: 8 waves, one workgroup per CU, BK = 64, two LDS buffers.
//
// The 2-stage kernel above waits vmcnt(0) + barrier every K-step; with its DMA in flight only for one
// K-step the MFMA pipe idles whenever both waves of a SIMD wait at once (PMC: 42-46 % MFMA busy).
// Here every K-step runs as 4 phases, each a LOAD segment (LDS fragment reads + the next DMA piece)
// and a COMPUTE segment (16 MFMAs) separated by workgroup barriers, and waves 4-7 start one barrier
// late, so on every SIMD one wave computes while its partner loads.  The DMA of K-step k+1 is issued
// in four pieces during K-step k and waited with COUNTED vmcnt (never 0 in the loop), each piece
// having 2-4 phases to land.
//
// Geometry: tile BM pixels x BN output channels; each wave owns 128 pixels x 64 channels (8 x 4
// MFMA 16x16 fragments, 128 fp32 accumulators per lane).  BN = 256: waves 2 (px) x 4 (ch), 64 KB per
// LDS buffer; BN = 128: BM = 512, waves 4 x 2, 80 KB per buffer (2 x 80 KB = the whole 160 KB LDS).
// The operand images are split in halves: X half h holds, for every pixel group g of 128, pixels
// g*128 + h*64 .. +64; W half h holds channels g*64 + h*32 .. +32.  Phase p reads (X half, W half):
//   p1: X0 (8 b128) + W0 (4)   compute X0 x W0
//   p2: W1 (4)                 compute X0 x W1
//   p3: X1 (8)                 compute X1 x W1
//   p4: -                      compute X1 x W0
// and issues the DMA of the next K-step's X0, W0, W1, X1 (in that order).  A half is refilled four
// phases after its last read (WAR safe for both wave groups) and read 3-4 phases after its DMA
// (RAW: each wave waits for its own pieces with a counted vmcnt before a barrier the readers pass).
template <int N>
PDT_DEVICE void vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}

template <int DT, int BM, int BN, int EPI, int RES, bool PP_STAGE = (EPI != 2)>  // (EPI 2 + staging spills)
__global__ __launch_bounds__(512) void conv_pp_kernel(ConvFwdArgs args) {
  ConvFwdArgs a = args;
  if (args.nphase > 0) {  // multi-phase launch (strided backward-data): this block's phase geometry
    const int ph = blockIdx.y;
    a.T = args.pT[ph]; a.U = args.pU[ph];
    a.ioff_h = args.pioff_h[ph]; a.ioff_w = args.pioff_w[ph];
    a.Pm = args.pPm[ph]; a.Qm = args.pQm[ph];
    a.ooff_h = args.pooff_h[ph]; a.ooff_w = args.pooff_w[ph];
    a.m_tiles = args.pmt[ph];
    a.M = (int64_t)a.N * a.Pm * a.Qm;
    a.w = args.w + args.pwoff[ph];
    a.pq_mul = args.ppq_mul[ph]; a.pq_shift = args.ppq_shift[ph];
    a.q_mul = args.pq1_mul[ph]; a.q_shift = args.pq1_shift[ph];
    if ((int)blockIdx.x >= a.m_tiles * a.n_tiles) {
      zero_stat_row<EPI, BN>(a, 512);
      return;
    }
  }
  using E = E16<DT>;
  typedef typename E::vec8 vec8;
  constexpr int NW = 8, WN = 64, WM = 128;
  constexpr int WAVES_N = BN / WN, WAVES_M = NW / WAVES_N;
  static_assert(WAVES_N * WAVES_M == NW && WAVES_M * WM == BM, "pp tile geometry");
  constexpr int FN = 4, FM = 8;           // channel / pixel fragments per wave
  constexpr int ROWB = 128;               // 64 16-bit elements per LDS row
  constexpr int XH = (BM / 2) * ROWB;     // bytes of one X half
  constexpr int WH = (BN / 2) * ROWB;     // bytes of one W half
  constexpr int NX = XH / 1024 / NW;      // DMA instructions per wave per X half
  constexpr int NWI = WH / 1024 / NW;     // ... per W half
  static_assert(NX * 1024 * NW == XH && NWI * 1024 * NW == WH, "pp DMA split");
  constexpr int BUF = 2 * XH + 2 * WH;
  constexpr int OX0 = 0, OX1 = XH, OW0 = 2 * XH, OW1 = 2 * XH + WH;
  __shared__ __attribute__((aligned(1024))) char smem[2 * BUF];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave >> 2;  // waves w and w+4 share a SIMD: they run one barrier apart
  const int wn = wave % WAVES_N, wm = wave / WAVES_N;

  const int nwg = a.m_tiles * a.n_tiles;
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int tile_m = bid / a.n_tiles, tile_n = bid % a.n_tiles;
  const int64_t m0 = (int64_t)tile_m * BM;
  const int n0 = tile_n * BN;

  const int PQ = a.Pm * a.Qm;
  const FastDiv fd_pq{a.pq_mul, a.pq_shift}, fd_q{a.q_mul, a.q_shift};
  const int TU = a.T * a.U;
  const int csteps = a.C >> 6;
  const int ksteps = TU * csteps;

  const __amdgpu_buffer_rsrc_t rx = make_rsrc(a.x, (uint32_t)a.N * a.H * a.W * a.cs * 2u);
  const __amdgpu_buffer_rsrc_t rw = make_rsrc(a.w, (uint32_t)a.Kout * TU * a.C * 2u);

  // DMA lane geometry: 8 rows x 8 chunks of 16 B per 1 KiB instruction; the source chunk is XOR
  // swizzled by the LDS row so the ds_read_b128 fragment reads are conflict free
  const int lrow = lane >> 3, pchunk = lane & 7;
  // X rows: packed (h << 16 | w & 0xffff) input position and byte offset, per half and instruction
  int xhw[2][NX], xoff[2][NX];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      const int hr = (wave * NX + j) * 8 + lrow;  // row of the half image
      const int64_t m = m0 + (hr >> 6) * 128 + h * 64 + (hr & 63);
      const int bch = pchunk ^ ((hr >> 1) & 7);
      if (m < a.M) {
        const int nimg = (int)fdiv((uint32_t)m, fd_pq);
        const int rem = (int)m - nimg * PQ;
        const int i = (int)fdiv((uint32_t)rem, fd_q), jj = rem - i * a.Qm;
        const int ih = i * a.ist_h + a.ioff_h, iw = jj * a.ist_w + a.ioff_w;
        xhw[h][j] = (ih << 16) | (iw & 0xffff);
        xoff[h][j] = (((nimg * a.H + ih) * a.W + iw) * a.cs + bch * 8) * 2;
      } else {
        xhw[h][j] = (int)0xC0000000;  // h = -16384: always out of range
        xoff[h][j] = 0;
      }
    }
  uint32_t woff[2][NWI];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int j = 0; j < NWI; ++j) {
      const int hr = (wave * NWI + j) * 8 + lrow;
      // permuted channel order inside each 32-row half (conv_epilogue PERM): LDS row f2*16 + m of the half holds
      // channel (m >> 2)*8 + f2*4 + (m & 3) -- the row swizzle stays a function of the LDS row, conflict-free as before
      const int lr = hr & 31;
      const int n = n0 + (hr >> 5) * 64 + h * 32 + ((lr & 15) >> 2) * 8 + (lr >> 4) * 4 + (lr & 3);
      woff[h][j] = (uint32_t)((n * TU * a.C + (pchunk ^ ((hr >> 1) & 7)) * 8) * 2);
    }

  // K-step cursor (tap, channel block) of the K-step whose DMA is being issued
  int cur_t = 0, cur_u = 0, cur_c = 0;
  uint32_t s_adelta = 0;
  int s_dh = 0, s_dw = 0, s_bdelta = 0;
  auto advance = [&]() {  // latch the cursor's K-step deltas, then step the cursor
    s_adelta = (uint32_t)((cur_t * a.U + cur_u) * a.C + cur_c) * 2u;
    s_dh = cur_t * a.tstep_h;
    s_dw = cur_u * a.tstep_w;
    s_bdelta = ((s_dh * a.W + s_dw) * a.cs + cur_c) * 2;
    cur_c += 64;
    if (cur_c == a.C) {
      cur_c = 0;
      if (++cur_u == a.U) { cur_u = 0; ++cur_t; }
    }
  };
  auto dma_x = [&](char* buf, int h) {
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      const int ih = (xhw[h][j] >> 16) + s_dh, iw = (int)(short)(xhw[h][j] & 0xffff) + s_dw;
      const bool ok = (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
      buf_lds16(rx, buf + (h ? OX1 : OX0) + (wave * NX + j) * 1024, ok ? (uint32_t)(xoff[h][j] + s_bdelta) : kOOB);
    }
  };
  auto dma_w = [&](char* buf, int h) {
#pragma unroll
    for (int j = 0; j < NWI; ++j)
      buf_lds16(rw, buf + (h ? OW1 : OW0) + (wave * NWI + j) * 1024, woff[h][j] + s_adelta);
  };

  f32x4_t acc[FN][FM];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  // fragment rows within the half images (the swizzle depends on the row only through bits 1..3,
  // which fr determines: every fragment base is a multiple of 16)
  const int xrow0 = wm * 64 + fr, wrow0 = wn * 32 + fr;
  const int sw = (fr >> 1) & 7;
  vec8 xs[4][2], w0r[2][2], w1r[2][2];
  auto read_x = [&](const char* base) {
#pragma unroll
    for (int f = 0; f < 4; ++f)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        xs[f][kk] = *(const vec8*)(base + (xrow0 + f * 16) * ROWB + (((kk * 4 + fq) ^ sw) << 4));
  };
  auto read_w = [&](vec8 (&wr)[2][2], const char* base) {
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        wr[f][kk] = *(const vec8*)(base + (wrow0 + f * 16) * ROWB + (((kk * 4 + fq) ^ sw) << 4));
  };
  auto mma = [&](const vec8 (&wr)[2][2], int xh, int wh) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int f2 = 0; f2 < 2; ++f2)
#pragma unroll
        for (int f = 0; f < 4; ++f)
          acc[wh * 2 + f2][xh * 4 + f] = E::mfma16x16x32(wr[f2][kk], xs[f][kk], acc[wh * 2 + f2][xh * 4 + f]);
  };
  auto compute = [&](const vec8 (&wr)[2][2], int xh, int wh) {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    mma(wr, xh, wh);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  if (ksteps > 0) {
    // prologue: all of K-step 0, then wait for its X0 / W0 (W1 and X1 may still fly)
    advance();
    dma_x(smem, 0);
    dma_w(smem, 0);
    dma_w(smem, 1);
    dma_x(smem, 1);
    vm_wait<NWI + NX>();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    if (grp == 1) __builtin_amdgcn_s_barrier();  // stagger: waves 4-7 run one barrier behind
    for (int ks = 0; ks < ksteps; ++ks) {
      const char* cb = smem + (ks & 1) * BUF;
      char* nb = smem + ((ks + 1) & 1) * BUF;
      const bool more = ks + 1 < ksteps;
      if (more) advance();
      // phase 1: DMA X0(k+1); wait W1(k); read X0, W0; compute X0 x W0
      if (more) { dma_x(nb, 0); vm_wait<2 * NX>(); } else { vm_wait<NX>(); }
      read_x(cb + OX0);
      read_w(w0r, cb + OW0);
      compute(w0r, 0, 0);
      // phase 2: DMA W0(k+1); wait X1(k); read W1; compute X0 x W1
      if (more) { dma_w(nb, 0); vm_wait<NX + NWI>(); } else { vm_wait<0>(); }
      read_w(w1r, cb + OW1);
      compute(w1r, 0, 1);
      // phase 3: DMA W1(k+1); read X1; compute X1 x W1
      if (more) dma_w(nb, 1);
      read_x(cb + OX1);
      compute(w1r, 1, 1);
      // phase 4: DMA X1(k+1); wait X0(k+1), W0(k+1); compute X1 x W0
      if (more) { dma_x(nb, 1); vm_wait<NWI + NX>(); }
      compute(w0r, 1, 0);
    }
    if (grp == 0) __builtin_amdgcn_s_barrier();  // re-align the two wave groups
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }

  conv_epilogue<DT, EPI, RES, FN, FM, WN, WM, BN, WAVES_M, NW, PP_STAGE ? 2 * BUF : 0, true>(a, acc, m0, n0, tile_m, wn,
                                                                                        wm, tid, lane, smem);
}

template <int DT, int BM, int BN>
static void launch_pp(const ConvFwdArgs& args, hipStream_t s) {
  // the ping-pong kernel stores straight from the accumulators: with the PERM epilogue the direct stores are 16 bytes
  // per lane, and LDS-staged row stores (one wave row-group at a time) measured slower on the same box in round 5
  // (ResNet-18 20.45/20.43 -> 20.33/20.32 ms, ResNet-50 73.23/73.36 -> 73.09/73.19); that knob was removed in round 6
  ConvFwdArgs a = args;
  a.stage_out = 0;
  if (a.nslice > 1)
    pdt_hip_fail("conv_pp: slice-batched (grouped) launches run on the generic kernel", hipErrorInvalidValue, __FILE__,
                 __LINE__);
  int gx = a.m_tiles * a.n_tiles;
  if (a.nphase > 0) {
    gx = 0;
    for (int p = 0; p < a.nphase; ++p) gx = gx > a.pmt[p] * a.n_tiles ? gx : a.pmt[p] * a.n_tiles;
  }
  dim3 grid(gx, a.nphase > 0 ? a.nphase : 1), block(512);
  const int rs = a.res == nullptr ? 0 : (a.res_phase >= 0 && a.nphase > 0 ? 2 : 1);
  const int epi = a.bnb ? a.bnb + 1 : (a.stats != nullptr ? 1 : 0);
#define PDT_K(E_, R_) hipLaunchKernelGGL((conv_pp_kernel<DT, BM, BN, E_, R_>), grid, block, 0, s, a)
  if (epi == 0) {
    if (rs == 1) PDT_K(0, 1); else if (rs == 2) PDT_K(0, 2); else PDT_K(0, 0);
  } else if (epi == 1 && rs != 2) {
    if (rs) PDT_K(1, 1); else PDT_K(1, 0);
  } else if (epi == 2 && !rs) {
    PDT_K(2, 0);
  } else if (epi == 3 && rs) {
    if (rs == 2) PDT_K(3, 2); else PDT_K(3, 1);
  } else if (epi == 4 && rs) {
    if (rs == 2) PDT_K(4, 2); else PDT_K(4, 1);
  } else {
    pdt_hip_fail("conv_pp: unsupported epilogue variant", hipErrorInvalidValue, __FILE__, __LINE__);
  }
#undef PDT_K
}

// ----------------------------------------------------------------------------------------------
template <int DT, int BM, int BN, int BK, int WAVES_N, int STAGES, int NW>
static void launch_cfg(const ConvFwdArgs& a, hipStream_t s) {
  int gx = a.m_tiles * a.n_tiles;
  if (a.nphase > 0) {
    gx = 0;
    for (int p = 0; p < a.nphase; ++p) gx = gx > a.pmt[p] * a.n_tiles ? gx : a.pmt[p] * a.n_tiles;
  }
  dim3 grid(gx, a.nphase > 0 ? a.nphase : 1, a.nslice > 1 ? a.nslice : 1), block(NW * 64);
  const int rs = a.res == nullptr ? 0 : (a.res_phase >= 0 && a.nphase > 0 ? 2 : 1);
  const int epi = a.bnb ? a.bnb + 1 : (a.stats != nullptr ? 1 : 0);
#define PDT_K(E_, R_) hipLaunchKernelGGL((conv_fwd_kernel<DT, BM, BN, BK, WAVES_N, E_, R_, STAGES, NW>), grid, block, 0, s, a)
  if (epi == 0) {
    if (rs == 1) PDT_K(0, 1); else if (rs == 2) PDT_K(0, 2); else PDT_K(0, 0);
  } else if (epi == 1 && rs != 2) {
    if (rs) PDT_K(1, 1); else PDT_K(1, 0);
  } else if constexpr ((((BK == 64 && STAGES == 2) || (BK == 32 && STAGES == 3)) && (BN == 128 || BN == 64) &&
                        (BM * BN == 4096 * NW || (BM == 256 && BN == 128 && NW == 4))) ||
                       (BM == 256 && BN == 256)) {
    // fused BN-backward epilogues: only on the backward-data tiles (128x128, 256x64: BK = 64 on the 2-stage ring,
    // BK = 32 on the 3-stage ring for short sub-pixel-phase reductions)
    if (epi == 2 && !rs) PDT_K(2, 0);
    else if (epi == 3 && rs) { if (rs == 2) PDT_K(3, 2); else PDT_K(3, 1); }
    else if (epi == 4 && rs) { if (rs == 2) PDT_K(4, 2); else PDT_K(4, 1); }
    else pdt_hip_fail("conv_fwd: unsupported BN-backward epilogue variant", hipErrorInvalidValue, __FILE__, __LINE__);
  } else {
    pdt_hip_fail("conv_fwd: BN-backward epilogue needs a 128x128 or 256x64 tile", hipErrorInvalidValue,
                 __FILE__, __LINE__);
  }
#undef PDT_K
}

template <int DT>
static void launch_tile(const ConvFwdArgs& a, int bm, int bn, int bk, hipStream_t s);

template <int DT>
static void launch_dt(ConvFwdArgs a, int bm, int bn, int bk, hipStream_t s) {
  // no LDS-staged output write-back: the PERM epilogue's direct stores are 16 bytes per lane; staging measured slower
  // on the same box in round 5 (ResNet-18 20.33/20.32 -> 20.23/20.23 ms, ResNet-50 73.09/73.19 -> 73.05/73.00 ms
  // with it off); the knob was removed in round 6
  a.stage_out = 0;
  a.m_tiles = (int)((a.M + bm - 1) / bm);
  a.n_tiles = a.Kout / bn;
  {
    const FastDiv f1 = make_fastdiv((uint32_t)(a.Pm * a.Qm)), f2 = make_fastdiv((uint32_t)a.Qm);
    a.pq_mul = f1.mul; a.pq_shift = f1.shift; a.q_mul = f2.mul; a.q_shift = f2.shift;
  }
  int srows = 0;  // statistics rows: one per (phase, M tile)
  if (a.nphase > 0) {
    int any = 0, maxmt = 0;
    for (int p = 0; p < a.nphase; ++p) {
      a.pmt[p] = (int)(((int64_t)a.N * a.pPm[p] * a.pQm[p] + bm - 1) / bm);
      any |= a.pmt[p];
      maxmt = maxmt > a.pmt[p] ? maxmt : a.pmt[p];
      if (a.pPm[p] > 0 && a.pQm[p] > 0) {
        const FastDiv f1 = make_fastdiv((uint32_t)(a.pPm[p] * a.pQm[p])), f2 = make_fastdiv((uint32_t)a.pQm[p]);
        a.ppq_mul[p] = f1.mul; a.ppq_shift[p] = f1.shift; a.pq1_mul[p] = f2.mul; a.pq1_shift[p] = f2.shift;
      }
    }
    if (!any || a.n_tiles == 0) return;
    a.srows_pp = maxmt;
    srows = a.nphase * maxmt;
  } else if (a.m_tiles * a.n_tiles == 0) {
    return;
  } else {
    a.srows_pp = a.m_tiles;
    srows = a.m_tiles;
  }
  const int KO = a.bnb == 3 ? 4 : 2;
  const int nsl = a.nslice > 1 ? a.nslice : 1;  // slice-batched grouped conv: rows span every slice's channels
  Scratch part(a.stats ? (size_t)srows * a.Kout * nsl * KO * sizeof(float) : 0, s);
  a.srows = part.as<float>();
  launch_tile<DT>(a, bm, bn, bk, s);
  if (a.stats) stat_rows_reduce_launch(a.srows, srows, a.Kout * nsl * KO, a.stats, s, a.stats_ld);
}

template <int DT>
static void launch_tile(const ConvFwdArgs& a, int bm, int bn, int bk, hipStream_t s) {
  // LDS ring depth: 2 for BK=64, 3 for BK=32 (round-3/4 sweeps)
#define PDT_CFGN(BM_, BN_, BK_, WN_, ST_, NW_)            \
  if (bm == BM_ && bn == BN_ && bk == BK_) {               \
    launch_cfg<DT, BM_, BN_, BK_, WN_, ST_, NW_>(a, s);    \
    return;                                                \
  }
#define PDT_CFG(BM_, BN_, BK_, WN_, ST_) PDT_CFGN(BM_, BN_, BK_, WN_, ST_, 4)
  {
    const bool dg = a.nphase > 0;  // backward-data (sub-pixel phases)
    const bool pp = bk == 64 && a.C % 64 == 0 && ((bm == 256 && bn == 256) || (bm == 512 && bn == 128));
    if (pp && dg)
      PDT_COUNT("conv_pp_dgrad");
    else if (pp)
      PDT_COUNT("conv_pp_fwd");
    else if (dg && a.nphase > 1)
      PDT_COUNT("conv_generic_dgrad_phased");
    else if (dg)
      PDT_COUNT("conv_generic_dgrad");
    else if (a.cs != a.C)
      PDT_COUNT("conv_generic_fwd_window");
    else
      PDT_COUNT("conv_generic_fwd");
    if (pp && bm == 512) PDT_COUNT("conv_pp_512x128");
    if (dg && a.res_phase >= 0) PDT_COUNT("conv_dgrad_compact_residual");
    if (dg && a.bnb) PDT_COUNT("conv_dgrad_bn_reduce_epilogue");
  }
  // BK = 64 tiles: 2-stage ring; BK = 32 tiles: 3-stage ring (counted vmcnt, more latency hiding)
  PDT_CFG(128, 128, 64, 2, 2)
  PDT_CFG(256, 64, 64, 1, 2)
  PDT_CFG(128, 64, 64, 1, 2)
  PDT_CFG(128, 128, 32, 2, 3)
  PDT_CFG(256, 64, 32, 1, 3)
  PDT_CFG(128, 64, 32, 1, 3)
  PDT_CFG(64, 128, 64, 4, 2)
  // 256 x 128: 4 waves of 128 x 64 (the ping-pong kernel's wave tile) on a 3-stage BK=32 ring (72 KB: 2 workgroups
  // per CU, two K-steps of LDS-DMA in flight) -- for BK = 64 callers too (C % 64 == 0 implies C % 32 == 0).  Round 6,
  // tools/conv_bench.py at B = 1200: ResNet-18 layer2 3x3 128 -> 128 forward 812 -> 872 TF/s, backward-data
  // 910 -> 925 TF/s, 3x3/2 64 -> 128 forward 521 -> 572, against the 128 x 128 2-stage tile; the 8-wave 2-stage
  // 256 x 128 kernel this replaces ran 750 / 441 on the same shapes.  Outputs are bit-identical to the 128 x 128
  // tile (same K order); the BN statistics differ in the order the per-tile partial rows are summed.
  if (bm == 256 && bn == 128 && (bk == 32 || bk == 64)) {
    launch_cfg<DT, 256, 128, 32, 2, 3, 4>(a, s);
    return;
  }
  const bool sliced = (a.ldy && a.ldy != a.Kout) || a.cs != a.C;
  if (bk == 64 && bm == 256 && bn == 256 && a.C % 64 == 0 && !sliced) {
    launch_pp<DT, 256, 256>(a, s);
    return;
  }
  if (bk == 64 && bm == 512 && bn == 128 && a.C % 64 == 0 && !sliced) {
    launch_pp<DT, 512, 128>(a, s);
    return;
  }
  PDT_CFGN(256, 256, 32, 4, 4, 8)  // 8 waves (2 x 4 of 128 x 64), 4-stage BK=32 ring (128 KB), 2 steps in flight
#undef PDT_CFG
#undef PDT_CFGN
  pdt_hip_fail("conv_fwd: unsupported tile config", hipErrorInvalidValue, __FILE__, __LINE__);
}

void conv_fwd_launch(const ConvFwdArgs& a, int dtype, int bm, int bn, int bk, hipStream_t s) {
  // ResNet layer1 geometry (3x3/s1/p1, 64 -> 64, W = 56): halo-reuse kernel (conv_l1.hip);
  // PDT_CONV_L1=0 forces the generic path
  static const bool l1_on = [] {
    const char* e = getenv("PDT_CONV_L1");
    return !(e && e[0] == '0');
  }();
  int flip = 0;
  if (l1_on && a.nslice > 1) {
    // grouped conv, every slice in one call: slices of the layer1 geometry (ResNeXt stage 1) run one halo-kernel
    // launch each (its persistent grid already fills the GPU), with the slice offsets of conv_fwd_kernel's nslice path
    ConvFwdArgs b = a;
    b.nslice = 0;
    if (conv_l1_eligible(b, &flip)) {
      if (b.nphase > 0)
        PDT_COUNT("conv_l1_dgrad");
      else
        PDT_COUNT("conv_l1_fwd");
      const int KO = a.bnb == 3 ? 4 : 2;
      for (int sl = 0; sl < a.nslice; ++sl) {
        b.x = a.x + (int64_t)sl * a.Kout;
        b.y = a.y + (int64_t)sl * a.Kout;
        b.w = a.w + (int64_t)sl * a.slice_wstride;
        b.bn_y1 = a.bn_y1 ? a.bn_y1 + (int64_t)sl * a.Kout : nullptr;
        b.bn_coef1 = a.bn_coef1 ? a.bn_coef1 + sl * a.Kout : nullptr;
        b.stats = a.stats ? a.stats + (int64_t)sl * a.Kout * KO : nullptr;
        conv_l1_launch(b, flip, dtype, s);
      }
      return;
    }
  }
  if (l1_on && conv_l1_eligible(a, &flip)) {
    if (a.nphase > 0)
      PDT_COUNT("conv_l1_dgrad");
    else
      PDT_COUNT("conv_l1_fwd");
    conv_l1_launch(a, flip, dtype, s);
    return;
  }
  if (a.pre_coef)
    pdt_hip_fail("conv_fwd: a fused producer BN (pre_coef) is only supported by the layer1 halo kernel",
                 hipErrorInvalidValue, __FILE__, __LINE__);
  if (dtype == kBF16)
    launch_dt<kBF16>(a, bm, bn, bk, s);
  else
    launch_dt<kF16>(a, bm, bn, bk, s);
}

int conv_fwd_m_tiles(int64_t M, int bm) { return (int)((M + bm - 1) / bm); }

}  // namespace pdt
