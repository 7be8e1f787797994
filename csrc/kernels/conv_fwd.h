#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pdt {

constexpr int kStatSlots = 64;  // slot copies of per-channel statistics accumulators

// Deterministic per-channel statistics (BN forward sums, BN-backward sums): every producing block writes
// its fp32 partials to its OWN row of rows[R][CK] with plain stores (no atomics, so no order-dependent
// rounding: fp64 atomics of cancelling partials made BN-backward sums -- and, through the chaotic 16-bit
// backward of a random-init ResNet, whole gradients -- depend on block scheduling), then
// stat_rows_reduce sums the rows in a FIXED order (slot s <- contiguous row range s*R/64.., fp64)
// into slots[kStatSlots][CK], the layout the finalize kernels and the SyncBN all-reduce read.  Every slot
// is written, so the slots need no zeroing.
void stat_rows_reduce_launch(const float* rows, int R, int CK, double* slots, hipStream_t s, int slots_ld = 0);


// Generalised implicit-GEMM convolution (see conv_fwd.hip for the geometry contract).
struct ConvFwdArgs {
  const uint16_t* x;    // [N][H][W][C] input activations
  const uint16_t* w;    // [Kout][T*U][C] weights (taps already ordered/flipped for the role)
  uint16_t* y;          // [N][OH][OW][Kout] output
  const uint16_t* res;  // optional: residual in y's layout, added before rounding (nullptr = none)
  double* stats;        // optional: [kStatSlots][Kout][2] fp64 (sum, sumsq) BN statistics (nullptr = none);
                        // with bnb != 0: [kStatSlots][Kout][2 or 4] BN-backward sums (sum dz, sum dz*xhat ...)
  float* srows;         // per-block partial rows [R][Kout][2 or 4] behind ``stats`` (set by the launcher)
  int srows_pp;         // rows per phase (multi-phase launches: row = phase * srows_pp + M tile)
  // Fused BN-backward reduce (backward-data use): 0 none | 1 mask from bn_y1 * coef1 (inner BN + ReLU)
  // | 2 mask from bn_mask (ReLU bitmask of the block output, bit e of byte v = element 8v+e > 0)
  // | 3 as 2 with a second BN branch bn_y2 / bn_coef2.
  int bnb;
  const uint16_t* bn_y1;
  const float* bn_coef1;  // forward coefficients [scale | shift | mean | invstd] x Kout
  const uint16_t* bn_y2;
  const float* bn_coef2;
  const uint8_t* bn_mask;
  int N, H, W, C, Kout, T, U;
  int cs;                                              // elements per input pixel (normally == C)
  int pair_skip;  // window-pair mode (stem, BK=64): chunks 4..7 read the NEXT image row (+pair_skip elements)
  int Pm, Qm;                                          // GEMM-M sub-grid (M = N*Pm*Qm)
  int ist_h, ist_w, ioff_h, ioff_w, tstep_h, tstep_w;  // in = i*ist + ioff + t*tstep
  int OH, OW, ost_h, ost_w, ooff_h, ooff_w;            // out = i*ost + ooff
  int64_t M;                                           // < 2^31 (32-bit fast division of pixel indices)
  int m_tiles, n_tiles;                                // filled by the launcher
  uint32_t pq_mul, pq_shift, q_mul, q_shift;           // FastDiv by Pm*Qm and Qm (filled by the launcher)
  // Multi-phase launch (backward-data of strided convs): blockIdx.y selects a phase whose geometry
  // overrides T, U, ioff, Pm, Qm, ooff and the weight offset.  nphase == 0: single-phase launch.
  int nphase;
  // res_phase >= 0: the residual exists only for phase res_phase and is COMPACT, indexed by that phase's GEMM
  // row ([N*Pm*Qm][Kout]: e.g. the 1x1/2 downsample's data gradient, which is zero on the other 3 phases of
  // a 3x3/2 dgrad and so is neither written nor read there).  -1: residual in dx's layout on every phase.
  int res_phase = -1;
  int stage_out = 0;  // epilogue writes the output tile through LDS as whole rows (set by the launcher)
  // pre_coef != nullptr: x is the RAW output of a producer conv and the kernel applies that BatchNorm + ReLU
  // (scale[C] | shift[C]) to the staged input tile itself (conv_l1 forward only; zero padding stays zero)
  const float* pre_coef = nullptr;
  // Channel slices of wider tensors (grouped convolution, models/executor.py): output pixel stride ``ldy`` (y, res,
  // bn_y1/bn_y2 and the ReLU mask are [pixels][ldy] with this conv's Kout channels at the caller's pointer offset),
  // stride ``coef_ld`` of the bn_coef1/bn_coef2 quantity rows, and row stride ``stats_ld`` of the fp64 statistics
  // slots ([kStatSlots][stats_ld]); 0 = Kout / Kout / Kout * quantities (dense tensors).  The input's pixel stride
  // is ``cs``.
  int ldy = 0, coef_ld = 0, stats_ld = 0;
  // nslice > 1: ONE launch over all channel slices of a grouped conv (blockIdx.z = slice s): x, y, bn_y1 and bn_coef1
  // advance by s * Kout elements, w by s * slice_wstride, and the statistics partial rows are [rows][nslice * Kout]
  // (every slice's columns of one row reduced together); 0 / 1: a single slice at the caller's pointers.
  int nslice = 0;
  int64_t slice_wstride = 0;
  int srows_coff = 0;  // kernel-local: this block's column offset (channels) in the statistics partial rows
  int pT[4], pU[4], pioff_h[4], pioff_w[4], pPm[4], pQm[4], pooff_h[4], pooff_w[4], pmt[4];
  int64_t pwoff[4];
  uint32_t ppq_mul[4], ppq_shift[4], pq1_mul[4], pq1_shift[4];
};

void conv_fwd_launch(const ConvFwdArgs& a, int dtype, int bm, int bn, int bk, hipStream_t s);
int conv_fwd_m_tiles(int64_t M, int bm);

}  // namespace pdt
