// fp32 compute path: the precision of the reference's `distributed.py` / `dataparallel.py` (plain fp32, no
// autocast; SURVEY K1 "fp32 path via v_mfma_f32_16x16x4_f32").  Storage, products and accumulation are all
// fp32; the matrix work runs on the CDNA4 fp32 MFMA (v_mfma_f32_16x16x4f32, 32 cycles per 16x16x4 on one
// SIMD: 1/16 of the bf16 rate, so an fp32 step is MFMA-bound by construction).
//
//   * conv32: implicit GEMM, NHWC x KRSC, the geometry contract of conv_fwd.hip (forward, multi-phase strided
//     backward-data with one launch for every sub-pixel phase, 1x1 / linear).  Tiles of 32 fp32 K-elements
//     (128-byte LDS rows, 8 16-byte chunks, source-side XOR swizzle: conflict-free ds_read_b128) are staged by
//     LDS-DMA into a 2-deep ring.  A lane's b128 fragment holds 4 consecutive K-elements of one row; MFMA e
//     (e = 0..3) consumes element e of every lane, i.e. the 16 K-elements of a fragment pair are split across
//     4 MFMAs by residue -- any permutation of K is valid as long as A and B use the same one -- so every
//     fragment is ONE ds_read_b128 instead of four ds_read_b32.  Epilogues: residual add and BN statistics
//     (per-block partial rows, fixed-order reduction: deterministic, conv_fwd.h).
//   * wgrad32: split-K weight gradient over 64-pixel chunks; the [pixel][channel] tiles are DMA'd with the
//     16-byte chunk index XOR-ed by (row & 3) << 2 so that the four pixel rows one MFMA reads (lane / 16) hit
//     four different bank groups (ds_read_b32, conflict free).
//   * BN apply / backward reduce / backward apply, stem BN+ReLU+max-pool and its backward, average pool,
//     softmax cross-entropy + accuracy, bias column sums, stem im2col: float4-vectorised NHWC kernels.
#include <cstdlib>

#include "../common.h"
#include "conv_fwd.h"
#include "fp32.h"

namespace pdt {

typedef float f32x4v __attribute__((ext_vector_type(4)));

PDT_DEVICE f32x4_t mfma4(float a, float b, f32x4_t c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }

static int ew_blocks(int64_t n) {
  int64_t b = (n + 255) / 256;
  if (b > 16384) b = 16384;
  return (int)(b < 1 ? 1 : b);
}

// ------------------------------------------------------------------------------------------------ conv32
template <int EPI, int BN_>
PDT_DEVICE void zero_stat_row32(const Conv32Args& a) {
  if constexpr (EPI != 0) {
    constexpr int KO = EPI == 3 ? 4 : 2;
    const int tm = (int)blockIdx.x / a.n_tiles, tn = (int)blockIdx.x - tm * a.n_tiles;
    float* dst = a.srows + ((int64_t)blockIdx.y * a.srows_pp + tm) * a.Kout * KO + (int64_t)tn * BN_ * KO;
    for (int i = threadIdx.x; i < BN_ * KO; i += blockDim.x) dst[i] = 0.f;
  }
}

// Shared epilogue of the fp32 implicit-GEMM kernels (conv32_kernel, conv32_halo_kernel): acc[i][j] holds
// output channels n0 + wn*WN + i*16 + 4*(lane>>4) + r of pixel m0 + wm*WM + j*16 + (lane&15).
template <int BM, int BN, int WAVES_M, int WAVES_N, int EPI, bool RES>
PDT_DEVICE void conv32_epilogue(const Conv32Args& a, f32x4_t (&acc)[BN / WAVES_N / 16][BM / WAVES_M / 16],
                                int64_t m0, int n0, int tile_m, int wn, int wm, int tid, int lane, char* smem) {
  constexpr int NW = WAVES_M * WAVES_N;
  constexpr int WN = BN / WAVES_N, WM = BM / WAVES_M;
  constexpr int FN = WN / 16, FM = WM / 16;
  const int fr = lane & 15, fq = lane >> 4;
  const int PQ = a.Pm * a.Qm;
  const FastDiv fd_pq{a.pq_mul, a.pq_shift}, fd_q{a.q_mul, a.q_shift};
  // EPI 1: forward statistics | 2: fused BN-backward reduce, one branch | 3: two branches (Conv32Args::bnb)
  constexpr int KS = EPI == 3 ? 3 : 2;  // accumulated quantities per channel
  float sacc[FN][4][KS];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int k = 0; k < KS; ++k) sacc[i][r][k] = 0.f;
#pragma unroll
  for (int j = 0; j < FM; ++j) {
    const int64_t m = m0 + wm * WM + j * 16 + fr;
    if (m >= a.M) continue;
    const int mm = (int)m;
    const int nimg = (int)fdiv((uint32_t)mm, fd_pq);
    const int rem = mm - nimg * PQ;
    const int i_ = (int)fdiv((uint32_t)rem, fd_q), j_ = rem - i_ * a.Qm;
    const int oh = i_ * a.ost_h + a.ooff_h, ow = j_ * a.ost_w + a.ooff_w;
    const int64_t ob = (((int64_t)nimg * a.OH + oh) * a.OW + ow) * a.Kout;
#pragma unroll
    for (int i = 0; i < FN; ++i) {
      const int n = n0 + wn * WN + i * 16 + 4 * fq;
      f32x4v v = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      if constexpr (RES) v += *(const f32x4v*)(a.res + ob + n);
      if constexpr (EPI >= 2) {  // fused BN-backward reduce of the consumer BN (see Conv32Args::bnb)
        f32x4v m, x1;
        if constexpr (EPI == 2) {
          const f32x4v y1 = *(const f32x4v*)(a.bn_y1 + ob + n);
          // ReLU mask: from the stored activation, or (no activation tensor: the producer's BN + ReLU fused into
          // its consumers) recomputed from the BN input exactly as the forward computed it
          m = a.bn_mref ? *(const f32x4v*)(a.bn_mref + ob + n)
                        : y1 * *(const f32x4v*)(a.bn_coef + n) + *(const f32x4v*)(a.bn_coef + a.Kout + n);
          x1 = (y1 - *(const f32x4v*)(a.bn_coef + 2 * a.Kout + n)) * *(const f32x4v*)(a.bn_coef + 3 * a.Kout + n);
        } else {  // (EPI 3, the block output: always a stored mask reference)
          m = *(const f32x4v*)(a.bn_mref + ob + n);
          x1 = (*(const f32x4v*)(a.bn_y1 + ob + n) - *(const f32x4v*)(a.bn_coef + 2 * a.Kout + n)) *
               *(const f32x4v*)(a.bn_coef + 3 * a.Kout + n);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[r] = m[r] > 0.f ? v[r] : 0.f;
          sacc[i][r][0] += v[r];
          sacc[i][r][1] += v[r] * x1[r];
        }
        if constexpr (EPI == 3) {
          const f32x4v x2 = (*(const f32x4v*)(a.bn_y2 + ob + n) - *(const f32x4v*)(a.bn_coef2 + 2 * a.Kout + n)) *
                            *(const f32x4v*)(a.bn_coef2 + 3 * a.Kout + n);
#pragma unroll
          for (int r = 0; r < 4; ++r) sacc[i][r][2] += v[r] * x2[r];
        }
      }
      *(f32x4v*)(a.y + ob + n) = v;
      if constexpr (EPI == 1) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          sacc[i][r][0] += v[r];
          sacc[i][r][1] += v[r] * v[r];
        }
      }
    }
  }
  if constexpr (EPI != 0) {
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int k = 0; k < KS; ++k) sacc[i][r][k] = row16_sum(sacc[i][r][k]);
    float* red = (float*)smem;  // [WAVES_M][BN][KS] (the LDS ring is free: every wave passed the last barrier)
    if (fr == 15) {
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int nl = wn * WN + i * 16 + 4 * fq + r;
#pragma unroll
          for (int k = 0; k < KS; ++k) red[(wm * BN + nl) * KS + k] = sacc[i][r][k];
        }
    }
    __syncthreads();
    // stored quantities per channel: KO = 2, or 4 for two branches (sum dz stored twice: the finalize's layout)
    constexpr int KO = EPI == 3 ? 4 : 2;
    for (int idx = tid; idx < BN * KO; idx += 64 * NW) {
      const int nl = idx / KO, ko = idx - nl * KO;
      const int k = EPI == 3 ? (ko == 2 ? 0 : (ko == 3 ? 2 : ko)) : ko;
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < WAVES_M; ++w) t += red[(w * BN + nl) * KS + k];
      const int64_t row = (a.nphase > 0 ? (int64_t)blockIdx.y * a.srows_pp : 0) + tile_m;
      a.srows[(row * a.Kout + n0 + nl) * KO + ko] = t;
    }
  }
}

// WAVES_M x WAVES_N waves, each owning a (BM / WAVES_M) x (BN / WAVES_N) accumulator block.  128 x 128 / 4 waves
// needs 32 FLOP per staged byte: at the fp32 MFMA rate that is ~5 TB/s of L2 traffic for the whole chip, which
// the 4-wave tile does not get (52 % of fp32 MFMA peak, profiles/r2_fp32_path.md).  256 x 256 / 8 waves (and
// 256 x 128 / 8 waves for 128-channel GEMMs) double / 1.3x that intensity; one 128 KB-LDS block per CU with two
// waves per SIMD, each wave running 256 MFMAs (8192 cycles) per K-step behind the next stage's DMA.
template <int BM, int BN, int WAVES_M, int WAVES_N, int EPI, bool RES>
__global__ __launch_bounds__(64 * WAVES_M * WAVES_N) void conv32_kernel(Conv32Args args) {
  Conv32Args a = args;
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
      zero_stat_row32<EPI, BN>(a);
      return;
    }
  }
  constexpr int NW = WAVES_M * WAVES_N;
  constexpr int WN = BN / WAVES_N, WM = BM / WAVES_M;
  constexpr int FN = WN / 16, FM = WM / 16;
  constexpr int ROWB = 128;               // 32 fp32 K-elements per LDS row
  constexpr int RPI = 1024 / ROWB;        // rows per LDS-DMA wave-instruction
  constexpr int A_INSTR = BN / RPI / NW;  // weight rows
  constexpr int B_INSTR = BM / RPI / NW;  // activation rows
  constexpr int A_BYTES = BN * ROWB;
  constexpr int STAGE = (BN + BM) * ROWB;
  static_assert(A_INSTR * RPI * NW == BN && B_INSTR * RPI * NW == BM, "conv32 tile/instr mismatch");
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
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
  const int ksteps = TU * (a.C / 32);

  const int cs = a.cs ? a.cs : a.C;  // element stride between input pixels (window mode: 4)
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(a.x, (uint32_t)((uint64_t)a.N * a.H * a.W * cs * 4u));
  const __amdgpu_buffer_rsrc_t rw = make_rsrc(a.w, (uint32_t)((uint64_t)a.Kout * TU * a.C * 4u));
  const int lrow = lane >> 3, pchunk = lane & 7;
  int brow_h[B_INSTR], brow_w[B_INSTR];
  uint32_t brow_off[B_INSTR];
#pragma unroll
  for (int j = 0; j < B_INSTR; ++j) {
    const int row = (wave * B_INSTR + j) * RPI + lrow;
    const int64_t m = m0 + row;
    const int bch = pchunk ^ ((row >> 1) & 7);
    if (m < a.M) {
      const int nimg = (int)fdiv((uint32_t)m, fd_pq);
      const int rem = (int)m - nimg * PQ;
      const int i = (int)fdiv((uint32_t)rem, fd_q), jj = rem - i * a.Qm;
      brow_h[j] = i * a.ist_h + a.ioff_h;
      brow_w[j] = jj * a.ist_w + a.ioff_w;
      brow_off[j] = (uint32_t)((((int64_t)(nimg * a.H + brow_h[j]) * a.W + brow_w[j]) * cs + bch * 4) * 4);
    } else {
      brow_h[j] = -(1 << 29);
      brow_w[j] = 0;
      brow_off[j] = 0;
    }
  }
  uint32_t arow_off[A_INSTR];
#pragma unroll
  for (int j = 0; j < A_INSTR; ++j) {
    const int row = (wave * A_INSTR + j) * RPI + lrow;
    arow_off[j] = (uint32_t)((((int64_t)(n0 + row) * TU * a.C) + (pchunk ^ ((row >> 1) & 7)) * 4) * 4);
  }
  int cur_t = 0, cur_u = 0, cur_c = 0;
  auto stage_load = [&](int buf) {
    const int t = cur_t, u = cur_u, c0 = cur_c;
    cur_c += 32;
    if (cur_c == a.C) {
      cur_c = 0;
      if (++cur_u == a.U) { cur_u = 0; ++cur_t; }
    }
    char* sbase = smem + buf * STAGE;
    const uint32_t a_delta = (uint32_t)((t * a.U + u) * a.C + c0) * 4u;
#pragma unroll
    for (int j = 0; j < A_INSTR; ++j) buf_lds16(rw, sbase + (wave * A_INSTR + j) * 1024, arow_off[j] + a_delta);
    const int dh = t * a.tstep_h, dw = u * a.tstep_w;
    const int b_delta = ((dh * a.W + dw) * cs + c0) * 4;
#pragma unroll
    for (int j = 0; j < B_INSTR; ++j) {
      const int h = brow_h[j] + dh, w = brow_w[j] + dw;
      const bool ok = (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W;
      buf_lds16(rx, sbase + A_BYTES + (wave * B_INSTR + j) * 1024, ok ? brow_off[j] + (uint32_t)b_delta : kOOB);
    }
  };

  f32x4_t acc[FN][FM];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fq = lane >> 4;
  int a_off[FN], b_off[FM];
#pragma unroll
  for (int i = 0; i < FN; ++i) a_off[i] = (wn * WN + i * 16 + fr) * ROWB;
#pragma unroll
  for (int j = 0; j < FM; ++j) b_off[j] = A_BYTES + (wm * WM + j * 16 + fr) * ROWB;
  const int sw = (fr >> 1) & 7;  // row swizzle: every fragment base is a multiple of 16 rows

  auto compute_stage = [&](const char* sb) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      f32x4v af[FN], bfr[FM];
#pragma unroll
      for (int i = 0; i < FN; ++i) af[i] = *(const f32x4v*)(sb + a_off[i] + (((kk * 4 + fq) ^ sw) << 4));
#pragma unroll
      for (int j = 0; j < FM; ++j) bfr[j] = *(const f32x4v*)(sb + b_off[j] + (((kk * 4 + fq) ^ sw) << 4));
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int i = 0; i < FN; ++i)
#pragma unroll
          for (int j = 0; j < FM; ++j) acc[i][j] = mfma4(af[i][e], bfr[j][e], acc[i][j]);
    }
  };

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

  conv32_epilogue<BM, BN, WAVES_M, WAVES_N, EPI, RES>(a, acc, m0, n0, tile_m, wn, wm, tid, lane, smem);
}

// ----------------------------------------------------------------------------------------- conv32 halo
// 3x3 / stride-1 convolutions whose output grid is the input grid (ResNet layer1, 64 -> 64 channels: forward and
// backward-data; per-tap input offsets dh, dw in {-1, 0, 1}).  conv32_kernel re-stages the activation tile for every
// one of the 9 taps (21 FLOP per staged byte at 128 x 64, the L2 -> LDS stream bounds it); here a block stages, per
// 32-channel chunk, the input rows its 256 output pixels span plus one halo row above and below -- each (W + 2) LDS
// rows of 128 B with a zero column on either side, source-swizzled like the GEMM tiles -- ONCE, and runs all 9 taps
// off it: a tap is a per-lane LDS row offset dh * (W + 2) + dw.  A pixel whose tap row leaves its own image (a
// block's rows may span two images) reads a zero LDS row instead.  Per K-step only the 8 KB weight tap tile is
// staged (2-deep ring): ~70 FLOP per staged byte.  8 waves (4 x 2 of 64 x 32), 74 KB LDS: two blocks per CU.
// K order: chunk-major (chunk, tap), so the fp32 sums differ from conv32_kernel's (tap, chunk) order in rounding.
constexpr int kHalo32Rows = 464;  // LDS rows of one halo chunk: ((W + 254) / W + 3) * (W + 2) <= 464 (W = 56: 8 x 58)

template <int EPI, bool RES>
__global__ __launch_bounds__(512) void conv32_halo_kernel(Conv32Args args) {
  Conv32Args a = args;
  if (args.nphase > 0) {  // single-phase (stride-1) backward-data launch: the phase's weights and tap offsets
    a.ioff_h = args.pioff_h[0]; a.ioff_w = args.pioff_w[0];
    a.w = args.w + args.pwoff[0];
  }
  constexpr int BM = 256, BN = 64, WAVES_M = 4, WAVES_N = 2, NW = WAVES_M * WAVES_N;
  constexpr int WN = BN / WAVES_N, WM = BM / WAVES_M, FN = WN / 16, FM = WM / 16;
  constexpr int ROWB = 128;                          // 32 fp32 channels per LDS row
  constexpr int A_BYTES = BN * ROWB;                 // one weight tap tile (8 KB), 1 DMA instruction per wave
  constexpr int OFF_H = 2 * A_BYTES;                 // the halo chunk
  constexpr int OFF_Z = OFF_H + kHalo32Rows * ROWB;  // one zero row
  constexpr int NHI = kHalo32Rows / 8;               // halo DMA instructions (8 rows each)
  constexpr int HI = (NHI + NW - 1) / NW;            // ... per wave
  static_assert(A_BYTES == NW * 1024, "one weight DMA instruction per wave");
  __shared__ __attribute__((aligned(1024))) char smem[OFF_Z + ROWB];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wave % WAVES_N, wm = wave / WAVES_N;
  const int nwg = a.m_tiles * a.n_tiles;
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int tile_m = bid / a.n_tiles, tile_n = bid % a.n_tiles;
  const int64_t m0 = (int64_t)tile_m * BM;
  const int n0 = tile_n * BN;
  const int Wd = a.W, W2 = a.W + 2, C = a.C;
  const FastDiv fd_pq{a.pq_mul, a.pq_shift}, fd_q{a.q_mul, a.q_shift};  // Pm * Qm == H * W, Qm == W
  const int mlast = (int)(m0 + BM < a.M ? m0 + BM : a.M) - 1;
  const int gA = (int)fdiv((uint32_t)m0, fd_q);  // first output row, rows of all images stacked
  const int gB = (int)fdiv((uint32_t)mlast, fd_q);
  const int hrows = (gB - gA + 3) * W2;           // LDS rows in use (host: <= kHalo32Rows)
  const int NG = a.N * a.H;
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(a.x, (uint32_t)((uint64_t)a.N * a.H * a.W * C * 4u));
  const __amdgpu_buffer_rsrc_t rw = make_rsrc(a.w, (uint32_t)((uint64_t)a.Kout * 9 * C * 4u));
  const int lrow = lane >> 3, pchunk = lane & 7;

  // halo DMA sources: LDS row hr = (halo row) * W2 + column + 1; rows outside the tensor, the zero columns and
  // the unused tail read zeros (kOOB)
  uint32_t hoff[HI];
#pragma unroll
  for (int k = 0; k < HI; ++k) {
    const int hr = (wave * HI + k) * 8 + lrow;
    const int hrow = hr / W2, col = hr - hrow * W2 - 1;
    const int g = gA - 1 + hrow;
    const bool ok = hr < hrows && g >= 0 && g < NG && col >= 0 && col < Wd;
    hoff[k] = ok ? (uint32_t)(((g * Wd + col) * C + (pchunk ^ ((hr >> 1) & 7)) * 4) * 4) : kOOB;
  }
  const int arow = wave * 8 + lrow;
  const uint32_t aoff = (uint32_t)(((n0 + arow) * 9 * C + (pchunk ^ ((arow >> 1) & 7)) * 4) * 4);
  auto stage_halo = [&](int kc) {
#pragma unroll
    for (int k = 0; k < HI; ++k) {
      const int ii = wave * HI + k;  // wave-uniform
      if (ii < NHI && ii * 8 < hrows)
        buf_lds16_asm(rx, smem + OFF_H + ii * 1024, hoff[k] == kOOB ? kOOB : hoff[k] + (uint32_t)kc * 128u);
    }
  };
  auto stage_w = [&](int kc, int tap, int buf) {
    buf_lds16_asm(rw, smem + buf * A_BYTES + wave * 1024, aoff + (uint32_t)((tap * C + kc * 32) * 4));
  };

  // per-lane output pixel geometry: halo base row and the pixel's row within its image
  const int fr = lane & 15, fq = lane >> 4;
  int hb[FM], hin[FM];
#pragma unroll
  for (int j = 0; j < FM; ++j) {
    const int64_t m = m0 + wm * WM + j * 16 + fr;
    if (m < a.M) {
      const int g = (int)fdiv((uint32_t)m, fd_q);
      const int nimg = (int)fdiv((uint32_t)m, fd_pq);
      hb[j] = (g - gA + 1) * W2 + ((int)m - g * Wd) + 1;
      hin[j] = g - nimg * a.H;
    } else {  // past the end: any in-range LDS row (the result is not stored)
      hb[j] = W2 + 1;
      hin[j] = 0;
    }
  }
  int a_off[FN];
#pragma unroll
  for (int i = 0; i < FN; ++i) a_off[i] = (wn * WN + i * 16 + fr) * ROWB;
  const int sw = (fr >> 1) & 7;

  f32x4_t acc[FN][FM];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int buf, int tap) {
    const int t = tap / 3, u = tap - 3 * t;
    const int dh = a.ioff_h + t * a.tstep_h, dw = a.ioff_w + u * a.tstep_w;
    const int delta = dh * W2 + dw;
    int bo[FM], bsw[FM];
#pragma unroll
    for (int j = 0; j < FM; ++j) {
      const int hr = hb[j] + delta;
      const bool ok = (unsigned)(hin[j] + dh) < (unsigned)a.H;
      bo[j] = ok ? OFF_H + hr * ROWB : OFF_Z;
      bsw[j] = ok ? (hr >> 1) & 7 : 0;
    }
    const char* sa = smem + buf * A_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      f32x4v af[FN], bfr[FM];
#pragma unroll
      for (int i = 0; i < FN; ++i) af[i] = *(const f32x4v*)(sa + a_off[i] + (((kk * 4 + fq) ^ sw) << 4));
#pragma unroll
      for (int j = 0; j < FM; ++j) bfr[j] = *(const f32x4v*)(smem + bo[j] + (((kk * 4 + fq) ^ bsw[j]) << 4));
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int i = 0; i < FN; ++i)
#pragma unroll
          for (int j = 0; j < FM; ++j) acc[i][j] = mfma4(af[i][e], bfr[j][e], acc[i][j]);
    }
  };

  const int nchunks = C / 32;
  if (tid < 8) *(f32x4v*)(smem + OFF_Z + tid * 16) = f32x4v{0.f, 0.f, 0.f, 0.f};
  stage_halo(0);
  stage_w(0, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int kc = 0, tap = 0;
  for (int ks = 0; ks < 9 * nchunks; ++ks) {
    const int nkc = tap == 8 ? kc + 1 : kc, ntap = tap == 8 ? 0 : tap + 1;
    const bool more = nkc < nchunks;
    if (more) stage_w(nkc, ntap, (ks + 1) & 1);  // the other ring slot: its last reader passed the last barrier
    compute(ks & 1, tap);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (more && nkc != kc) {  // next chunk: restage the halo once every wave is past its last read of it
      stage_halo(nkc);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
    kc = nkc;
    tap = ntap;
  }
  conv32_epilogue<BM, BN, WAVES_M, WAVES_N, EPI, RES>(a, acc, m0, n0, tile_m, wn, wm, tid, lane, smem);
}

// conv32_halo_kernel's geometry contract (see above); conv32_set_halo(0): the tap-restaging conv32_kernel (tests)
static bool g_conv32_halo = true;
int conv32_set_halo(int on) {
  const int prev = g_conv32_halo ? 1 : 0;
  g_conv32_halo = on != 0;
  return prev;
}

static bool conv32_halo_ok(const Conv32Args& a, int bn) {
  if (!g_conv32_halo || bn != 64 || a.nphase > 1 || a.Kout % 64 != 0 || a.C % 32 != 0) return false;
  if (a.cs != 0 && a.cs != a.C) return false;
  const bool ph = a.nphase == 1;
  const int T = ph ? a.pT[0] : a.T, U = ph ? a.pU[0] : a.U;
  const int ioh = ph ? a.pioff_h[0] : a.ioff_h, iow = ph ? a.pioff_w[0] : a.ioff_w;
  const int Pm = ph ? a.pPm[0] : a.Pm, Qm = ph ? a.pQm[0] : a.Qm;
  if (T != 3 || U != 3 || a.ist_h != 1 || a.ist_w != 1 || Pm != a.H || Qm != a.W) return false;
  if (a.ost_h != 1 || a.ost_w != 1 || a.OH != a.H || a.OW != a.W) return false;
  if (ph ? (a.pooff_h[0] != 0 || a.pooff_w[0] != 0) : (a.ooff_h != 0 || a.ooff_w != 0)) return false;
  for (int t = 0; t < 3; ++t) {
    const int dh = ioh + t * a.tstep_h, dw = iow + t * a.tstep_w;
    if (dh < -1 || dh > 1 || dw < -1 || dw > 1) return false;
  }
  if (a.W < 1 || ((a.W + 254) / a.W + 3) * (a.W + 2) > kHalo32Rows) return false;
  return (int64_t)a.N * a.H * a.W * a.C < (int64_t(1) << 29);
}

void conv32_launch(Conv32Args a, int bm, int bn, hipStream_t s) {
  const bool halo = conv32_halo_ok(a, bn);
  if (halo) bm = 256;
  a.m_tiles = (int)((a.M + bm - 1) / bm);
  a.n_tiles = a.Kout / bn;
  {
    const FastDiv f1 = make_fastdiv((uint32_t)(a.Pm * a.Qm)), f2 = make_fastdiv((uint32_t)a.Qm);
    a.pq_mul = f1.mul; a.pq_shift = f1.shift; a.q_mul = f2.mul; a.q_shift = f2.shift;
  }
  int srows = 0, gx = a.m_tiles * a.n_tiles;
  if (a.nphase > 0) {
    int maxmt = 0;
    for (int p = 0; p < a.nphase; ++p) {
      a.pmt[p] = (int)(((int64_t)a.N * a.pPm[p] * a.pQm[p] + bm - 1) / bm);
      maxmt = maxmt > a.pmt[p] ? maxmt : a.pmt[p];
      if (a.pPm[p] > 0 && a.pQm[p] > 0) {
        const FastDiv f1 = make_fastdiv((uint32_t)(a.pPm[p] * a.pQm[p])), f2 = make_fastdiv((uint32_t)a.pQm[p]);
        a.ppq_mul[p] = f1.mul; a.ppq_shift[p] = f1.shift; a.pq1_mul[p] = f2.mul; a.pq1_shift[p] = f2.shift;
      }
    }
    a.srows_pp = maxmt;
    srows = a.nphase * maxmt;
    gx = maxmt * a.n_tiles;
  } else {
    a.srows_pp = a.m_tiles;
    srows = a.m_tiles;
  }
  if (gx == 0 || a.n_tiles == 0) return;
  PDT_COUNT(a.nphase > 0 ? "conv32_dgrad" : "conv32_fwd");
  const int KO = a.bnb && a.bn_y2 ? 4 : 2;
  Scratch part(a.stats ? (size_t)srows * a.Kout * KO * sizeof(float) : 0, s);
  a.srows = part.as<float>();
  const bool st = a.stats != nullptr, rs = a.res != nullptr;
  if (a.bnb && (!st || a.nphase == 0))
    pdt_hip_fail("conv32: the fused BN-backward epilogue needs a backward-data launch with stats", hipErrorInvalidValue,
                 __FILE__, __LINE__);
  if (a.bnb) PDT_COUNT("conv32_dgrad_bn_reduce_epilogue");
  const int two = a.bn_y2 != nullptr;
  if (halo) {
    PDT_COUNT("conv32_halo");
    dim3 grid(gx, 1), block(512);
    if (a.bnb && two && rs) hipLaunchKernelGGL((conv32_halo_kernel<3, true>), grid, block, 0, s, a);
    else if (a.bnb && two) hipLaunchKernelGGL((conv32_halo_kernel<3, false>), grid, block, 0, s, a);
    else if (a.bnb && rs) hipLaunchKernelGGL((conv32_halo_kernel<2, true>), grid, block, 0, s, a);
    else if (a.bnb) hipLaunchKernelGGL((conv32_halo_kernel<2, false>), grid, block, 0, s, a);
    else if (st && rs) hipLaunchKernelGGL((conv32_halo_kernel<1, true>), grid, block, 0, s, a);
    else if (st) hipLaunchKernelGGL((conv32_halo_kernel<1, false>), grid, block, 0, s, a);
    else if (rs) hipLaunchKernelGGL((conv32_halo_kernel<0, true>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((conv32_halo_kernel<0, false>), grid, block, 0, s, a);
    if (st) stat_rows_reduce_launch(a.srows, srows, a.Kout * KO, a.stats, s);
    return;
  }
#define PDT_C32(BM_, BN_, WM_, WN_)                                                                        \
  if (bm == BM_ && bn == BN_) {                                                                          \
    dim3 grid(gx, a.nphase > 0 ? a.nphase : 1), block(64 * WM_ * WN_);                                   \
    if (a.bnb && two && rs) hipLaunchKernelGGL((conv32_kernel<BM_, BN_, WM_, WN_, 3, true>), grid, block, 0, s, a); \
    else if (a.bnb && two) hipLaunchKernelGGL((conv32_kernel<BM_, BN_, WM_, WN_, 3, false>), grid, block, 0, s, a); \
    else if (a.bnb && rs) hipLaunchKernelGGL((conv32_kernel<BM_, BN_, WM_, WN_, 2, true>), grid, block, 0, s, a);   \
    else if (a.bnb) hipLaunchKernelGGL((conv32_kernel<BM_, BN_, WM_, WN_, 2, false>), grid, block, 0, s, a);  \
    else if (st && rs) hipLaunchKernelGGL((conv32_kernel<BM_, BN_, WM_, WN_, 1, true>), grid, block, 0, s, a); \
    else if (st) hipLaunchKernelGGL((conv32_kernel<BM_, BN_, WM_, WN_, 1, false>), grid, block, 0, s, a); \
    else if (rs) hipLaunchKernelGGL((conv32_kernel<BM_, BN_, WM_, WN_, 0, true>), grid, block, 0, s, a);  \
    else hipLaunchKernelGGL((conv32_kernel<BM_, BN_, WM_, WN_, 0, false>), grid, block, 0, s, a);         \
    if (st) stat_rows_reduce_launch(a.srows, srows, a.Kout * KO, a.stats, s);                              \
    return;                                                                                              \
  }
  PDT_C32(128, 128, 2, 2)
  PDT_C32(128, 64, 2, 2)
  PDT_C32(256, 256, 2, 4)
  PDT_C32(256, 128, 4, 2)
  PDT_C32(256, 64, 4, 1)
  PDT_C32(512, 64, 8, 1)
#undef PDT_C32
  pdt_hip_fail("conv32: unsupported tile (128x128, 128x64, 256x256, 256x128, 256x64 or 512x64)", hipErrorInvalidValue,
               __FILE__, __LINE__);
}

// ----------------------------------------------------------------------------------------------- wgrad32
// Block: 64 output channels x 64 input channels of ONE tap over a pixel range; 4 waves in 2 x 2 (32 x 32 each).
__global__ __launch_bounds__(256) void wgrad32_kernel(Wgrad32Args a) {
  constexpr int PIX = 64;              // pixels per staged chunk
  constexpr int TILE = PIX * 64 * 4;   // 16 KiB per operand tile ([pixel][64 channels] fp32, 256 B rows)
  __shared__ __attribute__((aligned(1024))) char smem[2 * 2 * TILE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wk = wave >> 1, wc = wave & 1;
  const int split = blockIdx.x, k0 = blockIdx.y * 64;
  const int cblocks = a.C / 64;
  const int tap = blockIdx.z / cblocks, c0 = (blockIdx.z - tap * cblocks) * 64;
  const int t = tap / a.U, u = tap - t * a.U;
  const int64_t p_begin = (int64_t)split * a.pix_per_split;
  const int64_t p_end = p_begin + a.pix_per_split < a.P ? p_begin + a.pix_per_split : a.P;
  const int cs = a.cs ? a.cs : a.C;  // elements per input pixel (window-pair mode: 4)
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(a.x, (uint32_t)((uint64_t)a.N * a.H * a.W * cs * 4u));
  const __amdgpu_buffer_rsrc_t rd = make_rsrc(a.dy, (uint32_t)((uint64_t)a.P * a.Kout * 4u));
  // DMA lane geometry: one wave-instruction = 4 rows x 16 chunks of 16 B; source chunk = LDS chunk ^ (row & 3) << 2
  const int lrow = lane >> 4, pc = lane & 15;
  const int sc = pc ^ (lrow << 2);
  const int pskip = sc >= 8 ? a.pair_skip : 0;
  const int PQ = a.Pm * a.Qm;
  auto stage = [&](int64_t p0, int buf) {
    char* dyb = smem + buf * 2 * TILE;
    char* xb = dyb + TILE;
#pragma unroll
    for (int q = 0; q < 4; ++q) {  // 16 instructions per tile, 4 per wave
      const int ins = wave * 4 + q;
      const int row = ins * 4 + lrow;
      const int64_t p = p0 + row;
      uint32_t od = kOOB, ox = kOOB;
      if (p < p_end) {
        od = (uint32_t)((p * a.Kout + k0 + sc * 4) * 4);
        const int n = (int)(p / PQ);
        const int rem = (int)(p - (int64_t)n * PQ);
        const int i = rem / a.Qm, j = rem - (rem / a.Qm) * a.Qm;
        const int ih = i * a.stride - a.pad + t * a.tstep, iw = j * a.stride - a.pad + u;
        if ((unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W)
          ox = (uint32_t)(((((int64_t)n * a.H + ih) * a.W + iw) * cs + c0 + sc * 4 + pskip) * 4);
      }
      buf_lds16(rd, dyb + ins * 1024, od);
      buf_lds16(rx, xb + ins * 1024, ox);
    }
  };
  f32x4_t acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fq = lane >> 4;
  // element (row, col) of a tile lives at row*256 + (((col >> 2) ^ ((row & 3) << 2)) << 4) + (col & 3)*4;
  // the rows read together are 4s + fq, so (row & 3) == fq
  int aoff[2], boff[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int col = wk * 32 + i * 16 + fr;
    aoff[i] = fq * 256 + ((((col >> 2) ^ (fq << 2))) << 4) + (col & 3) * 4;
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = wc * 32 + j * 16 + fr;
    boff[j] = TILE + fq * 256 + ((((col >> 2) ^ (fq << 2))) << 4) + (col & 3) * 4;
  }
  const int nchunks = p_end > p_begin ? (int)((p_end - p_begin + PIX - 1) / PIX) : 0;
  if (nchunks > 0) {
    stage(p_begin, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int ch = 0; ch < nchunks; ++ch) {
      const int cur = ch & 1;
      if (ch + 1 < nchunks) stage(p_begin + (int64_t)(ch + 1) * PIX, cur ^ 1);
      const char* base = smem + cur * 2 * TILE;
#pragma unroll 4
      for (int s4 = 0; s4 < PIX / 4; ++s4) {
        const char* sb = base + s4 * 4 * 256;
        float av[2], bv[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) av[i] = *(const float*)(sb + aoff[i]);
#pragma unroll
        for (int j = 0; j < 2; ++j) bv[j] = *(const float*)(sb + boff[j]);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = mfma4(av[i], bv[j], acc[i][j]);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  }
  // lane holds dW[k = k0 + wk*32 + i*16 + 4*fq + r][c = c0 + wc*32 + j*16 + fr]
  float* out = a.ws + (int64_t)split * a.Kout * a.ldw;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int k = k0 + wk * 32 + i * 16 + 4 * fq + r;
        const int c = c0 + wc * 32 + j * 16 + fr;
        out[(int64_t)k * a.ldw + tap * a.C + c] = acc[i][j][r];
      }
}

// dY of the fp32 stem backward for 4 channels of one conv-output pixel, in two halves so the loads can be issued
// ahead of the MFMAs that hide them: stem_dy32_load gathers the conv output and the (up to 4) pooling windows that
// can select the pixel; stem_dy32_finish applies the max-pool backward, the ReLU mask and dy = A*dz + B*y + C --
// the float operations and their order are stem_pool_dz32's + stem_pool_bwd_apply32's (windows in (oh, ow)
// ascending order, invalid ones skipped), so the result is the separate apply pass's.
struct StemDy32In {
  f32x4v yy, gv[4];
  uint32_t ib[4];
  int pos[4];  // kernel tap (kh * 3 + kw) of the pixel in window wi, -1: no such window
};
PDT_DEVICE void stem_dy32_load(const Wgrad32Args& a, int64_t p, int c0, StemDy32In& in) {
  const int PQ = a.Pm * a.Qm;
  const int n = (int)(p / PQ);
  const int rem = (int)(p - (int64_t)n * PQ);
  const int h = rem / a.Qm, w = rem - (rem / a.Qm) * a.Qm;
  in.yy = *(const f32x4v*)(a.f_y + p * 64 + c0);
  const int oh0 = h >> 1, oh1 = (h + 1) >> 1, ow0 = w >> 1, ow1 = (w + 1) >> 1;
#pragma unroll
  for (int wi = 0; wi < 4; ++wi) {
    const int oh = wi >> 1 ? oh1 : oh0, ow = wi & 1 ? ow1 : ow0;
    const int kh = h - (oh * 2 - 1), kw = w - (ow * 2 - 1);
    const bool ok = (!(wi >> 1) || oh1 != oh0) && (!(wi & 1) || ow1 != ow0) && oh < a.f_OH && ow < a.f_OW &&
                    kh >= 0 && kh <= 2 && kw >= 0 && kw <= 2;
    in.pos[wi] = ok ? kh * 3 + kw : -1;
    const int64_t o = (((int64_t)n * a.f_OH + (ok ? oh : oh0)) * a.f_OW + (ok ? ow : ow0)) * 64 + c0;
    in.ib[wi] = *(const uint32_t*)(a.f_idx + o);
    in.gv[wi] = *(const f32x4v*)(a.f_dp + o);
  }
}
PDT_DEVICE f32x4v stem_dy32_finish(const Wgrad32Args& a, const StemDy32In& in, int c0) {
  f32x4v acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int wi = 0; wi < 4; ++wi) {
    if (in.pos[wi] < 0) continue;
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if ((int)((in.ib[wi] >> (8 * e)) & 0xffu) == in.pos[wi]) acc[e] += in.gv[wi][e];
  }
  const f32x4v yy = in.yy;
#pragma unroll
  for (int e = 0; e < 4; ++e)
    if (!(yy[e] * a.f_coef[c0 + e] + a.f_coef[64 + c0 + e] > 0.f)) acc[e] = 0.f;
  const float* b = a.f_bcoef;
  return *(const f32x4v*)(b + c0) * acc + *(const f32x4v*)(b + 64 + c0) * yy + *(const f32x4v*)(b + 128 + c0);
}

// Window-pair stem weight gradient with ALL kernel-row pairs per block (the fp32 twin of the 16-bit
// wgrad_stem_kernel): wgrad32_kernel runs one block per (pair, split) and so stages every dY tile once per pair
// (4x) at 16 FLOP per staged byte.  Here a block stages one 32-pixel dY tile plus the 4 pair-windows of X (8 KB
// each, 40 KB per stage, 2-deep ring: 80 KB, two blocks per CU) and 8 waves own (pair = wave / 2) x (32 window
// columns) x all 64 output channels: 26 FLOP per staged byte.  Same LDS element layout and window addressing as
// wgrad32_kernel (Wgrad32Args window-pair fields).
// FUSE (Wgrad32Args::f_y): the dY tile of every chunk is computed in the kernel (stem_dy32_*) instead of DMA'd --
// the separate apply pass and its 3.85 GB fp32 dY write + re-read (ResNet-18, B = 1200) disappear.  A thread owns 4
// channels of one pixel row; the next chunk's gathers are issued before this chunk's MFMAs and finished after them.
template <bool FUSE>
__global__ __launch_bounds__(512) void wgrad32_stem4_kernel(Wgrad32Args a) {
  constexpr int PIX = 32;             // pixels per staged chunk
  constexpr int TILE = PIX * 64 * 4;  // 8 KiB per operand tile ([pixel][64] fp32, 256 B rows)
  constexpr int NT = 5;               // dY + 4 pair windows
  constexpr int STAGE = NT * TILE;
  constexpr int INS = NT * TILE / 1024 / 8;  // DMA wave-instructions per wave per stage (5)
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wt = wave >> 1, wc = wave & 1;  // pair, 32-column half
  const int split = blockIdx.x, k0 = blockIdx.y * 64;
  const int64_t p_begin = (int64_t)split * a.pix_per_split;
  const int64_t p_end = p_begin + a.pix_per_split < a.P ? p_begin + a.pix_per_split : a.P;
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(a.x, (uint32_t)((uint64_t)a.N * a.H * a.W * 4u * 4u));
  const __amdgpu_buffer_rsrc_t rd = make_rsrc(a.dy, (uint32_t)((uint64_t)a.P * a.Kout * 4u));
  const int lrow = lane >> 4, pc = lane & 15;
  const int sc = pc ^ (lrow << 2);
  const int pskip = sc >= 8 ? a.pair_skip : 0;
  const int PQ = a.Pm * a.Qm;
  auto stage = [&](int64_t p0, int buf) {
    char* sb = smem + buf * STAGE;
#pragma unroll
    for (int q = 0; q < INS; ++q) {
      const int ins = wave * INS + q;  // 0..39: tile ins / 8, rows (ins % 8) * 4 + lrow
      const int tile = ins >> 3;
      if (FUSE && tile == 0) continue;  // dY computed by dy_store
      const int row = (ins & 7) * 4 + lrow;
      const int64_t p = p0 + row;
      uint32_t off = kOOB;
      if (p < p_end) {
        if (tile == 0) {
          off = (uint32_t)((p * a.Kout + k0 + sc * 4) * 4);
        } else {
          const int n = (int)(p / PQ);
          const int rem = (int)(p - (int64_t)n * PQ);
          const int i = rem / a.Qm, j = rem - (rem / a.Qm) * a.Qm;
          const int ih = i * a.stride + (tile - 1) * a.tstep, iw = j * a.stride;
          if ((unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W)
            off = (uint32_t)(((((int64_t)n * a.H + ih) * a.W + iw) * 4 + sc * 4 + pskip) * 4);
        }
      }
      buf_lds16_asm(tile == 0 ? rd : rx, sb + ins * 1024, off);
    }
  };
  f32x4_t acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fq = lane >> 4;
  // element (row, col) of a tile: row*256 + (((col >> 2) ^ ((row & 3) << 2)) << 4) + (col & 3)*4; the rows read
  // together are 4s + fq, so (row & 3) == fq
  int aoff[4], boff[2];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int col = i * 16 + fr;
    aoff[i] = fq * 256 + ((((col >> 2) ^ (fq << 2))) << 4) + (col & 3) * 4;
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = wc * 32 + j * 16 + fr;
    boff[j] = (1 + wt) * TILE + fq * 256 + ((((col >> 2) ^ (fq << 2))) << 4) + (col & 3) * 4;
  }
  // FUSE: this thread's dY element group -- pixel row dr of the chunk, channels dc .. dc+3 (of the block's k0 slab)
  const int dr = tid >> 4, dc = k0 + (tid & 15) * 4;
  StemDy32In din;
  auto dy_load = [&](int64_t p0) {
    const int64_t p = p0 + dr;
    stem_dy32_load(a, p < p_end ? p : p_begin, dc, din);
  };
  auto dy_store = [&](int64_t p0, int buf) {
    const f32x4v v = p0 + dr < p_end ? stem_dy32_finish(a, din, dc) : f32x4v{0.f, 0.f, 0.f, 0.f};
    const int chunk = tid & 15;
    *(f32x4v*)(smem + buf * STAGE + dr * 256 + ((chunk ^ ((dr & 3) << 2)) << 4)) = v;
  };
  const int nchunks = p_end > p_begin ? (int)((p_end - p_begin + PIX - 1) / PIX) : 0;
  if (nchunks > 0) {
    stage(p_begin, 0);
    if constexpr (FUSE) {
      dy_load(p_begin);
      dy_store(p_begin, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int ch = 0; ch < nchunks; ++ch) {
      const int cur = ch & 1;
      const int64_t pn = p_begin + (int64_t)(ch + 1) * PIX;
      if (ch + 1 < nchunks) {
        stage(pn, cur ^ 1);
        if constexpr (FUSE) dy_load(pn);
      }
      const char* base = smem + cur * STAGE;
#pragma unroll 4
      for (int s4 = 0; s4 < PIX / 4; ++s4) {
        const char* sb = base + s4 * 4 * 256;
        float av[4], bv[2];
#pragma unroll
        for (int i = 0; i < 4; ++i) av[i] = *(const float*)(sb + aoff[i]);
#pragma unroll
        for (int j = 0; j < 2; ++j) bv[j] = *(const float*)(sb + boff[j]);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = mfma4(av[i], bv[j], acc[i][j]);
      }
      if constexpr (FUSE) {
        if (ch + 1 < nchunks) dy_store(pn, cur ^ 1);  // slot cur ^ 1 was last read in chunk ch - 1
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  }
  // lane holds dW[k = k0 + i*16 + 4*fq + r][pair wt, c = wc*32 + j*16 + fr]
  float* out = a.ws + (int64_t)split * a.Kout * a.ldw;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int k = k0 + i * 16 + 4 * fq + r;
        const int c = wc * 32 + j * 16 + fr;
        out[(int64_t)k * a.ldw + wt * 64 + c] = acc[i][j][r];
      }
}

// Wide variant: 128 (Kout) x 128 (C) output tile of one tap, 8 waves as 2 (k) x 4 (c), each 64 x 32 (4 x 2 MFMA
// tiles), 32-pixel chunks (dY and X tiles 16 KB each, 512-byte rows, 2-deep LDS-DMA ring: 64 KB, two blocks per
// CU).  32 FLOP per staged byte against the 64 x 64 kernel's 16: the 64 x 64 tile needs ~10 TB/s of L2 traffic at
// the fp32 MFMA rate, this one half that.  Rows are 32 chunks of 16 B; source chunk = LDS chunk ^ ((row & 3) << 2),
// so the 4 pixel rows one MFMA reads (lane / 16) land on 4 disjoint 16-bank groups (ds_read_b32 conflict free).
__global__ __launch_bounds__(512) void wgrad32w_kernel(Wgrad32Args a) {
  constexpr int PIX = 32;
  constexpr int ROW = 512;              // 128 fp32 channels
  constexpr int TILE = PIX * ROW;       // 16 KiB per operand tile
  __shared__ __attribute__((aligned(1024))) char smem[2 * 2 * TILE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wk = wave >> 2, wc = wave & 3;
  const int split = blockIdx.x, k0 = blockIdx.y * 128;
  const int cblocks = a.C / 128;
  const int tap = blockIdx.z / cblocks, c0 = (blockIdx.z - tap * cblocks) * 128;
  const int t = tap / a.U, u = tap - t * a.U;
  const int64_t p_begin = (int64_t)split * a.pix_per_split;
  const int64_t p_end = p_begin + a.pix_per_split < a.P ? p_begin + a.pix_per_split : a.P;
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(a.x, (uint32_t)((uint64_t)a.N * a.H * a.W * a.C * 4u));
  const __amdgpu_buffer_rsrc_t rd = make_rsrc(a.dy, (uint32_t)((uint64_t)a.P * a.Kout * 4u));
  // DMA lane geometry: one wave-instruction = 2 rows x 32 chunks of 16 B; 16 instructions per tile, 2 per wave
  const int lrow = lane >> 5, pc = lane & 31;
  const int PQ = a.Pm * a.Qm;
  auto stage = [&](int64_t p0, int buf) {
    char* dyb = smem + buf * 2 * TILE;
    char* xb = dyb + TILE;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int ins = wave * 2 + q;
      const int row = ins * 2 + lrow;
      const int sc = pc ^ ((row & 3) << 2);
      const int64_t p = p0 + row;
      uint32_t od = kOOB, ox = kOOB;
      if (p < p_end) {
        od = (uint32_t)((p * a.Kout + k0 + sc * 4) * 4);
        const int n = (int)(p / PQ);
        const int rem = (int)(p - (int64_t)n * PQ);
        const int i = rem / a.Qm, j = rem - (rem / a.Qm) * a.Qm;
        const int ih = i * a.stride - a.pad + t, iw = j * a.stride - a.pad + u;
        if ((unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W)
          ox = (uint32_t)(((((int64_t)n * a.H + ih) * a.W + iw) * a.C + c0 + sc * 4) * 4);
      }
      buf_lds16(rd, dyb + ins * 1024, od);
      buf_lds16(rx, xb + ins * 1024, ox);
    }
  };
  f32x4_t acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fq = lane >> 4;
  // element (row, col) lives at row*512 + (((col >> 2) ^ ((row & 3) << 2)) << 4) + (col & 3)*4; rows read
  // together are 4*s4 + fq, so (row & 3) == fq
  int aoff[4], boff[2];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int col = wk * 64 + i * 16 + fr;
    aoff[i] = fq * ROW + ((((col >> 2) ^ (fq << 2))) << 4) + (col & 3) * 4;
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = wc * 32 + j * 16 + fr;
    boff[j] = TILE + fq * ROW + ((((col >> 2) ^ (fq << 2))) << 4) + (col & 3) * 4;
  }
  const int nchunks = p_end > p_begin ? (int)((p_end - p_begin + PIX - 1) / PIX) : 0;
  if (nchunks > 0) {
    stage(p_begin, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int ch = 0; ch < nchunks; ++ch) {
      const int cur = ch & 1;
      if (ch + 1 < nchunks) stage(p_begin + (int64_t)(ch + 1) * PIX, cur ^ 1);
      const char* base = smem + cur * 2 * TILE;
#pragma unroll
      for (int s4 = 0; s4 < PIX / 4; ++s4) {
        const char* sb = base + s4 * 4 * ROW;
        float av[4], bv[2];
#pragma unroll
        for (int i = 0; i < 4; ++i) av[i] = *(const float*)(sb + aoff[i]);
#pragma unroll
        for (int j = 0; j < 2; ++j) bv[j] = *(const float*)(sb + boff[j]);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = mfma4(av[i], bv[j], acc[i][j]);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  }
  // lane holds dW[k = k0 + wk*64 + i*16 + 4*fq + r][c = c0 + wc*32 + j*16 + fr]
  float* out = a.ws + (int64_t)split * a.Kout * a.ldw;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int k = k0 + wk * 64 + i * 16 + 4 * fq + r;
        const int c = c0 + wc * 32 + j * 16 + fr;
        out[(int64_t)k * a.ldw + tap * a.C + c] = acc[i][j][r];
      }
}

// Halo variant for 3x3 / stride 1 / pad 1 convs over 64-channel blocks (ResNet layer1): a block owns ONE kernel row
// r_tap and computes all three taps s of it -- a 64 (Kout) x 192 (s, C) tile -- over whole output rows.  Per output
// row it stages the dY row (Q pixels) and the input row h + r_tap - 1 with a one-pixel halo (Q + 2 pixels, the
// image padding as zeros), and tap s reads the input tile shifted by s rows: 48 FLOP per staged byte instead of the
// 64 x 64 kernel's 16.  4 waves, each 64 (k) x 48 (s, c) = 4 x 3 MFMA 16x16 tiles; 2-deep LDS-DMA ring of
// (Q + Q + 2 + 2) x 256 B.  Rows: the pixel-row swizzle of wgrad32 (chunk ^ (row & 3) << 2) keeps the four rows one
// MFMA reads (lane / 16, plus the tap shift) on distinct bank groups.
constexpr int kHaloMaxQ = 62;
__global__ __launch_bounds__(256) void wgrad32_halo_kernel(Wgrad32Args a) {
  constexpr int ROW = 256;                       // 64 fp32 channels
  constexpr int XR = kHaloMaxQ + 2;               // staged input rows (halo included), 64
  constexpr int DR = kHaloMaxQ + 2;               // staged dY rows (multiple of 4 for the DMA), 64
  constexpr int TILE_D = DR * ROW, TILE_X = XR * ROW;
  constexpr int STAGE = TILE_D + TILE_X;          // 32 KB
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int split = blockIdx.x, rt = blockIdx.y;
  const int cblocks = a.C / 64;
  const int k0 = (blockIdx.z / cblocks) * 64, c0 = (blockIdx.z - (blockIdx.z / cblocks) * cblocks) * 64;
  const int Q = a.Qm, nrows = a.N * a.Pm;
  const int r_begin = split * a.pix_per_split;  // pix_per_split counts OUTPUT ROWS in this kernel
  const int r_end = r_begin + a.pix_per_split < nrows ? r_begin + a.pix_per_split : nrows;
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(a.x, (uint32_t)((uint64_t)a.N * a.H * a.W * a.C * 4u));
  const __amdgpu_buffer_rsrc_t rd = make_rsrc(a.dy, (uint32_t)((uint64_t)a.P * a.Kout * 4u));
  const int lrow = lane >> 4, pc = lane & 15;
  const int sc = pc ^ (lrow << 2);  // (row & 3) == lrow for rows 4*ins + lrow
  auto stage = [&](int orow, int buf) {
    char* db = smem + buf * STAGE;
    char* xb = db + TILE_D;
    const int n = orow / a.Pm, h = orow - n * a.Pm;
    const int ih = h + rt - 1;
    const bool row_ok = (unsigned)ih < (unsigned)a.H;
    // 16 dY rows-of-4 + 16 X rows-of-4 = 32 instructions, 8 per wave
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int ins = wave * 8 + q;
      if (ins < 16) {
        const int row = ins * 4 + lrow;  // dY pixel w = row
        const uint32_t od = row < Q ? (uint32_t)((((int64_t)orow * Q + row) * a.Kout + k0 + sc * 4) * 4) : kOOB;
        buf_lds16(rd, db + ins * 1024, od);
      } else {
        const int xi = ins - 16;
        const int row = xi * 4 + lrow;  // input pixel iw = row - 1
        const int iw = row - 1;
        const uint32_t ox = (row_ok && (unsigned)iw < (unsigned)a.W && row < Q + 2)
                                ? (uint32_t)(((((int64_t)n * a.H + ih) * a.W + iw) * a.C + c0 + sc * 4) * 4) : kOOB;
        buf_lds16(rx, xb + xi * 1024, ox);
      }
    }
  };
  f32x4_t acc[4][3];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fq = lane >> 4;
  int aoff[4], bcol[3], bsh[3];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int col = i * 16 + fr;  // k within the 64-wide block
    aoff[i] = fq * ROW + ((((col >> 2) ^ (fq << 2))) << 4) + (col & 3) * 4;
  }
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int cc = wave * 48 + j * 16;  // (s, c) column of this fragment
    bsh[j] = cc / 64;                   // tap s: the input tile shifted by s rows
    bcol[j] = (cc & 63) + fr;
  }
  const int steps = (Q + 3) / 4;
  if (r_end > r_begin) {
    stage(r_begin, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int orow = r_begin; orow < r_end; ++orow) {
      const int cur = (orow - r_begin) & 1;
      if (orow + 1 < r_end) stage(orow + 1, cur ^ 1);
      const char* db = smem + cur * STAGE;
      const char* xb = db + TILE_D;
      for (int s4 = 0; s4 < steps; ++s4) {
        float av[4], bv[3];
#pragma unroll
        for (int i = 0; i < 4; ++i) av[i] = *(const float*)(db + s4 * 4 * ROW + aoff[i]);
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const int row = s4 * 4 + fq + bsh[j];
          bv[j] = *(const float*)(xb + row * ROW + ((((bcol[j] >> 2) ^ ((row & 3) << 2))) << 4) + (bcol[j] & 3) * 4);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 3; ++j) acc[i][j] = mfma4(av[i], bv[j], acc[i][j]);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  }
  // lane holds dW[k = k0 + i*16 + 4*fq + r][tap (rt, s), c = c0 + bcol - fr + fr]; ws column = (rt*3 + s)*C + c
  float* out = a.ws + (int64_t)split * a.Kout * a.ldw;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int k = k0 + i * 16 + 4 * fq + r;
        out[(int64_t)k * a.ldw + (rt * 3 + bsh[j]) * a.C + c0 + bcol[j]] = acc[i][j][r];
      }
}

bool wgrad32_halo_supported(const Wgrad32Args& a) {
  return a.T == 3 && a.U == 3 && a.stride == 1 && a.pad == 1 && a.C % 64 == 0 && a.Kout % 64 == 0 &&
         a.Pm == a.H && a.Qm == a.W && a.Qm <= kHaloMaxQ;
}

void wgrad32_launch(const Wgrad32Args& a, hipStream_t s) {
  if (a.tile == 3) {  // halo kernel (wgrad32_halo_supported): splits over output rows
    if (!wgrad32_halo_supported(a))
      pdt_hip_fail("wgrad32: halo kernel needs a 3x3/s1/p1 conv, 64-channel blocks and W <= 62", hipErrorInvalidValue,
                   __FILE__, __LINE__);
    PDT_COUNT("wgrad32_halo");
    dim3 grid(a.splits, 3, (a.Kout / 64) * (a.C / 64)), block(256);
    hipLaunchKernelGGL(wgrad32_halo_kernel, grid, block, 0, s, a);
    return;
  }
  if (a.tile == 4) {  // window-pair stem, all 4 pairs per block
    if (a.cs != 4 || a.T != 4 || a.U != 1 || a.C != 64 || a.Kout % 64 != 0 || a.ldw != 256 || a.pad != 0 ||
        a.pix_per_split % 32 != 0)
      pdt_hip_fail("wgrad32: the 4-pair stem kernel needs the window-pair geometry (cs 4, 4 pairs, C 64)",
                   hipErrorInvalidValue, __FILE__, __LINE__);
    dim3 grid(a.splits, a.Kout / 64), block(512);
    if (a.f_y != nullptr) {
      if (a.Kout != 64)
        pdt_hip_fail("wgrad32: the fused stem kernel needs Kout == 64", hipErrorInvalidValue, __FILE__, __LINE__);
      PDT_COUNT("wgrad32_stem4_fused");
      hipLaunchKernelGGL(wgrad32_stem4_kernel<true>, grid, block, 0, s, a);
    } else {
      PDT_COUNT("wgrad32_stem4");
      hipLaunchKernelGGL(wgrad32_stem4_kernel<false>, grid, block, 0, s, a);
    }
    return;
  }
  if (a.tile == 128) {
    PDT_COUNT("wgrad32_wide");
    dim3 grid(a.splits, a.Kout / 128, a.T * a.U * (a.C / 128)), block(512);
    hipLaunchKernelGGL(wgrad32w_kernel, grid, block, 0, s, a);
    return;
  }
  PDT_COUNT("wgrad32");
  dim3 grid(a.splits, a.Kout / 64, a.T * a.U * (a.C / 64)), block(256);
  hipLaunchKernelGGL(wgrad32_kernel, grid, block, 0, s, a);
}

// ----------------------------------------------------------------------------------------- elementwise
// out = act(y*scale + shift + R), R = 0 | res | res*rscale + rshift
template <int RESMODE, bool RELU>
__global__ __launch_bounds__(256) void bn_apply32_kernel(const float* __restrict__ y, const float* __restrict__ coef,
                                                         const float* __restrict__ res, const float* __restrict__ rcoef,
                                                         float* __restrict__ out, int64_t n4, int C) {
  // channel of float4 v, stepped with the grid stride (one 64-bit modulo per thread, not per element)
  const int64_t v0 = (int64_t)blockIdx.x * 256 + threadIdx.x, vs = (int64_t)gridDim.x * 256;
  const int cstep = (int)((vs * 4) % C);
  int c = (int)((v0 * 4) % C);
  for (int64_t v = v0; v < n4; v += vs, c = c + cstep >= C ? c + cstep - C : c + cstep) {
    f32x4v val = ((const f32x4v*)y)[v] * *(const f32x4v*)(coef + c) + *(const f32x4v*)(coef + C + c);
    if constexpr (RESMODE == 1) val += ((const f32x4v*)res)[v];
    if constexpr (RESMODE == 2)
      val += ((const f32x4v*)res)[v] * *(const f32x4v*)(rcoef + c) + *(const f32x4v*)(rcoef + C + c);
    if constexpr (RELU) {
#pragma unroll
      for (int e = 0; e < 4; ++e) val[e] = fmaxf(val[e], 0.f);
    }
    ((f32x4v*)out)[v] = val;
  }
}

void bn_apply32_launch(const float* y, const float* coef, const float* res, const float* rcoef, float* out, int64_t n,
                       int C, int resmode, bool relu, hipStream_t s) {
  const int64_t n4 = n / 4;
  dim3 g(ew_blocks(n4)), b(256);
#define PDT_A32(RM, RL)                                                                                          \
  if (resmode == RM && relu == RL) {                                                                             \
    hipLaunchKernelGGL((bn_apply32_kernel<RM, RL>), g, b, 0, s, y, coef, res, rcoef, out, n4, C);                 \
    return;                                                                                                      \
  }
  PDT_A32(0, true) PDT_A32(1, true) PDT_A32(2, true) PDT_A32(0, false) PDT_A32(1, false) PDT_A32(2, false)
#undef PDT_A32
}

// Backward reduce: dz = g * (mref > 0) (mref: the post-ReLU activation, optional); per branch b:
//   sum dz, sum dz * (y_b - mean_b) * invstd_b   -> this block's partial row [C][K] (K = 2 or 4)
// A thread owns NV float4 channel groups of a row (C <= 2048), rows strided over the grid.
template <bool MASK, int NBR, int NV>
__global__ __launch_bounds__(256) void bn_bwd_reduce32_kernel(const float* __restrict__ g, const float* __restrict__ mref,
                                                              const float* __restrict__ y1, const float* __restrict__ coef1,
                                                              const float* __restrict__ y2, const float* __restrict__ coef2,
                                                              float* __restrict__ srows, int64_t rows, int C) {
  const int vpr = C / 4;
  const int lanes_c = vpr / NV;              // threads per row
  const int rpi = 256 / lanes_c;             // rows per block iteration
  const int cl = threadIdx.x % lanes_c, rl = threadIdx.x / lanes_c;
  constexpr int K = NBR * 2;
  float s[NV][K][4];
#pragma unroll
  for (int q = 0; q < NV; ++q)
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
      for (int e = 0; e < 4; ++e) s[q][k][e] = 0.f;
  if (rl < rpi) {
    for (int64_t r = (int64_t)blockIdx.x * rpi + rl; r < rows; r += (int64_t)gridDim.x * rpi) {
#pragma unroll
      for (int q = 0; q < NV; ++q) {
        const int c0 = (cl + q * lanes_c) * 4;
        const int64_t off = r * C + c0;
        f32x4v dz = *(const f32x4v*)(g + off);
        if constexpr (MASK) {
          const f32x4v m = *(const f32x4v*)(mref + off);
#pragma unroll
          for (int e = 0; e < 4; ++e) dz[e] = m[e] > 0.f ? dz[e] : 0.f;
        }
        const f32x4v x1 = (*(const f32x4v*)(y1 + off) - *(const f32x4v*)(coef1 + 2 * C + c0)) *
                          *(const f32x4v*)(coef1 + 3 * C + c0);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          s[q][0][e] += dz[e];
          s[q][1][e] += dz[e] * x1[e];
        }
        if constexpr (NBR == 2) {
          const f32x4v x2 = (*(const f32x4v*)(y2 + off) - *(const f32x4v*)(coef2 + 2 * C + c0)) *
                            *(const f32x4v*)(coef2 + 3 * C + c0);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            s[q][2][e] += dz[e];
            s[q][3][e] += dz[e] * x2[e];
          }
        }
      }
    }
  }
  extern __shared__ float red[];  // [rpi][C][K]
  if (rl < rpi) {
#pragma unroll
    for (int q = 0; q < NV; ++q)
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int k = 0; k < K; ++k) red[((int64_t)rl * C + (cl + q * lanes_c) * 4 + e) * K + k] = s[q][k][e];
  }
  __syncthreads();
  float* dst = srows + (int64_t)blockIdx.x * C * K;
  for (int idx = threadIdx.x; idx < C * K; idx += 256) {
    float tt = 0.f;
    for (int q = 0; q < rpi; ++q) tt += red[(int64_t)q * C * K + idx];
    dst[idx] = tt;
  }
}

int bn_bwd_reduce32_blocks(int64_t rows, int C) {
  const int vpr = C / 4;
  const int rpi = vpr >= 256 ? 1 : 256 / vpr;
  int64_t b = (rows + rpi * 16 - 1) / (rpi * 16);
  if (b > 1024) b = 1024;
  return (int)(b < 1 ? 1 : b);
}

void bn_bwd_reduce32_launch(const float* g, const float* mref, const float* y1, const float* coef1, const float* y2,
                            const float* coef2, double* slots, int blocks, int64_t rows, int C, hipStream_t s) {
  const int vpr = C / 4;
  const int nv = vpr > 256 ? vpr / 256 : 1;
  if (nv > 2 || (vpr > 256 && vpr % 256 != 0))
    pdt_hip_fail("bn_bwd_reduce32: C must be <= 2048 (and a multiple of 1024 above 1024)", hipErrorInvalidValue,
                 __FILE__, __LINE__);
  const int rpi = 256 / (vpr / nv);
  const int nbr = y2 ? 2 : 1;
  Scratch part((size_t)blocks * C * nbr * 2 * sizeof(float), s);
  float* srows = part.as<float>();
  const size_t smem = (size_t)rpi * C * nbr * 2 * sizeof(float);
  const bool mask = mref != nullptr;
#define PDT_R32(M_, NB_, NV_)                                                                                \
  if (mask == M_ && nbr == NB_ && nv == NV_) {                                                               \
    hipLaunchKernelGGL((bn_bwd_reduce32_kernel<M_, NB_, NV_>), dim3(blocks), dim3(256), smem, s, g, mref, y1, \
                       coef1, y2, coef2, srows, rows, C);                                                     \
    stat_rows_reduce_launch(srows, blocks, C * nbr * 2, slots, s);                                           \
    return;                                                                                                  \
  }
  PDT_R32(true, 1, 1) PDT_R32(true, 2, 1) PDT_R32(false, 1, 1) PDT_R32(false, 2, 1)
  PDT_R32(true, 1, 2) PDT_R32(true, 2, 2) PDT_R32(false, 1, 2) PDT_R32(false, 2, 2)
#undef PDT_R32
}

// dy_b = A_b*dz + B_b*y_b + C_b, dz = g * (mref > 0); optionally writes dz (identity-branch gradient)
template <bool MASK, int NBR, bool WDZ>
__global__ __launch_bounds__(256) void bn_bwd_apply32_kernel(const float* __restrict__ g, const float* __restrict__ mref,
                                                             const float* __restrict__ y1, const float* __restrict__ b1,
                                                             float* __restrict__ dy1, const float* __restrict__ y2,
                                                             const float* __restrict__ b2, float* __restrict__ dy2,
                                                             float* __restrict__ dz_out, int64_t n4, int C) {
  const int64_t v0 = (int64_t)blockIdx.x * 256 + threadIdx.x, vs = (int64_t)gridDim.x * 256;
  const int cstep = (int)((vs * 4) % C);
  int c = (int)((v0 * 4) % C);
  for (int64_t v = v0; v < n4; v += vs, c = c + cstep >= C ? c + cstep - C : c + cstep) {
    f32x4v dz = ((const f32x4v*)g)[v];
    if constexpr (MASK) {
      const f32x4v m = ((const f32x4v*)mref)[v];
#pragma unroll
      for (int e = 0; e < 4; ++e) dz[e] = m[e] > 0.f ? dz[e] : 0.f;
    }
    ((f32x4v*)dy1)[v] = *(const f32x4v*)(b1 + c) * dz + *(const f32x4v*)(b1 + C + c) * ((const f32x4v*)y1)[v] +
                        *(const f32x4v*)(b1 + 2 * C + c);
    if constexpr (NBR == 2)
      ((f32x4v*)dy2)[v] = *(const f32x4v*)(b2 + c) * dz + *(const f32x4v*)(b2 + C + c) * ((const f32x4v*)y2)[v] +
                          *(const f32x4v*)(b2 + 2 * C + c);
    if constexpr (WDZ) ((f32x4v*)dz_out)[v] = dz;
  }
}

void bn_bwd_apply32_launch(const float* g, const float* mref, const float* y1, const float* b1, float* dy1,
                           const float* y2, const float* b2, float* dy2, float* dz, int64_t n, int C, hipStream_t s) {
  const int64_t n4 = n / 4;
  dim3 gr(ew_blocks(n4)), bl(256);
  const bool mask = mref != nullptr, wdz = dz != nullptr;
  const int nbr = y2 ? 2 : 1;
#define PDT_B32(M_, NB_, WZ_)                                                                                     \
  if (mask == M_ && nbr == NB_ && wdz == WZ_) {                                                                   \
    hipLaunchKernelGGL((bn_bwd_apply32_kernel<M_, NB_, WZ_>), gr, bl, 0, s, g, mref, y1, b1, dy1, y2, b2, dy2, dz, \
                       n4, C);                                                                                    \
    return;                                                                                                       \
  }
  PDT_B32(true, 1, false) PDT_B32(true, 1, true) PDT_B32(true, 2, false) PDT_B32(true, 2, true)
  PDT_B32(false, 1, false) PDT_B32(false, 1, true) PDT_B32(false, 2, false) PDT_B32(false, 2, true)
#undef PDT_B32
}

// stem BN + ReLU + MaxPool(3, 2, 1), argmax (0..8) as uint8 (the backward's routing)
__global__ __launch_bounds__(256) void bn_relu_maxpool32_kernel(const float* __restrict__ y, const float* __restrict__ coef,
                                                                float* __restrict__ out, uint8_t* __restrict__ idx, int N,
                                                                int H, int W, int C, int OH, int OW) {
  const int cv = C / 4;
  const int64_t total = (int64_t)N * OH * OW * cv;
  for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < total; v += (int64_t)gridDim.x * 256) {
    const int64_t pix = v / cv;
    const int c0 = (int)(v - pix * cv) * 4;
    const int ow = (int)(pix % OW);
    const int64_t tq = pix / OW;
    const int oh = (int)(tq % OH), n = (int)(tq / OH);
    const f32x4v sc = *(const f32x4v*)(coef + c0), sh = *(const f32x4v*)(coef + C + c0);
    f32x4v best = {-1.f, -1.f, -1.f, -1.f};
    uint8_t bi[4] = {0, 0, 0, 0};
    for (int kh = 0; kh < 3; ++kh) {
      const int h = oh * 2 - 1 + kh;
      if ((unsigned)h >= (unsigned)H) continue;
      for (int kw = 0; kw < 3; ++kw) {
        const int w = ow * 2 - 1 + kw;
        if ((unsigned)w >= (unsigned)W) continue;
        const f32x4v q = *(const f32x4v*)(y + (((int64_t)n * H + h) * W + w) * C + c0);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float val = fmaxf(q[e] * sc[e] + sh[e], 0.f);
          if (val > best[e]) { best[e] = val; bi[e] = (uint8_t)(kh * 3 + kw); }
        }
      }
    }
    *(f32x4v*)(out + pix * C + c0) = best;
    *(uint32_t*)(idx + pix * C + c0) = (uint32_t)bi[0] | ((uint32_t)bi[1] << 8) | ((uint32_t)bi[2] << 16) |
                                       ((uint32_t)bi[3] << 24);
  }
}

void bn_relu_maxpool32_launch(const float* y, const float* coef, float* out, uint8_t* idx, int N, int H, int W, int C,
                              hipStream_t s) {
  const int OH = (H + 2 - 3) / 2 + 1, OW = (W + 2 - 3) / 2 + 1;
  hipLaunchKernelGGL(bn_relu_maxpool32_kernel, dim3(ew_blocks((int64_t)N * OH * OW * (C / 4))), dim3(256), 0, s, y,
                     coef, out, idx, N, H, W, C, OH, OW);
}

// gather-form max-pool backward fused with the ReLU mask recomputed from the BN input y
__global__ __launch_bounds__(256) void maxpool_bwd_relu32_kernel(const float* __restrict__ dp, const uint8_t* __restrict__ idx,
                                                                 const float* __restrict__ y, const float* __restrict__ coef,
                                                                 float* __restrict__ dz, int N, int H, int W, int C, int OH,
                                                                 int OW) {
  const int cv = C / 4;
  const int64_t total = (int64_t)N * H * W * cv;
  for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < total; v += (int64_t)gridDim.x * 256) {
    const int c0 = (int)(v % cv) * 4;
    int64_t pix = v / cv;
    const int w = (int)(pix % W);
    pix /= W;
    const int h = (int)(pix % H), n = (int)(pix / H);
    f32x4v acc = {0.f, 0.f, 0.f, 0.f};
    for (int oh = h / 2; oh <= (h + 1) / 2; ++oh) {
      const int kh = h - (oh * 2 - 1);
      if (oh >= OH || kh < 0 || kh > 2) continue;
      for (int ow = w / 2; ow <= (w + 1) / 2; ++ow) {
        const int kw = w - (ow * 2 - 1);
        if (ow >= OW || kw < 0 || kw > 2) continue;
        const uint8_t pos = (uint8_t)(kh * 3 + kw);
        const int64_t o = (((int64_t)n * OH + oh) * OW + ow) * C + c0;
        const uint32_t ib = *(const uint32_t*)(idx + o);
        const f32x4v gv = *(const f32x4v*)(dp + o);
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if ((uint8_t)(ib >> (8 * e)) == pos) acc[e] += gv[e];
      }
    }
    const int64_t i = (((int64_t)n * H + h) * W + w) * C + c0;
    const f32x4v yy = *(const f32x4v*)(y + i);
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (!(yy[e] * coef[c0 + e] + coef[C + c0 + e] > 0.f)) acc[e] = 0.f;
    *(f32x4v*)(dz + i) = acc;
  }
}

void maxpool_bwd_relu32_launch(const float* dp, const uint8_t* idx, const float* y, const float* coef, float* dz, int N,
                               int H, int W, int C, hipStream_t s) {
  const int OH = (H + 2 - 3) / 2 + 1, OW = (W + 2 - 3) / 2 + 1;
  hipLaunchKernelGGL(maxpool_bwd_relu32_kernel, dim3(ew_blocks((int64_t)N * H * W * (C / 4))), dim3(256), 0, s, dp, idx,
                     y, coef, dz, N, H, W, C, OH, OW);
}

// The stem's backward tail without the dz tensor (N x H x W x C fp32, 3.85 GB at ResNet-18 bs1200): dz = max-pool
// backward (gather over the <= 4 pooling windows covering a pixel, argmax routing) x ReLU mask (BN output > 0) is
// recomputed from the pooled gradient, the argmax bytes and y0 by both the BN-backward reduce and the apply, instead
// of maxpool_bwd_relu32 writing it and bn_bwd_reduce32 / bn_bwd_apply32 reading it back: ~28 -> ~14 GB of traffic.
// The gather and the float operations are maxpool_bwd_relu32's, and the reduce's thread / row / block structure is
// bn_bwd_reduce32's (NV = 1): the results equal the three separate passes' up to the compiler's fma contraction.
PDT_DEVICE f32x4v stem_pool_dz32(const float* __restrict__ dp, const uint8_t* __restrict__ idx, const f32x4v yy,
                                 const float* __restrict__ coef, int n, int h, int w, int c0, int C, int OH, int OW) {
  f32x4v acc = {0.f, 0.f, 0.f, 0.f};
  for (int oh = h / 2; oh <= (h + 1) / 2; ++oh) {
    const int kh = h - (oh * 2 - 1);
    if (oh >= OH || kh < 0 || kh > 2) continue;
    for (int ow = w / 2; ow <= (w + 1) / 2; ++ow) {
      const int kw = w - (ow * 2 - 1);
      if (ow >= OW || kw < 0 || kw > 2) continue;
      const uint8_t pos = (uint8_t)(kh * 3 + kw);
      const int64_t o = (((int64_t)n * OH + oh) * OW + ow) * C + c0;
      const uint32_t ib = *(const uint32_t*)(idx + o);
      const f32x4v gv = *(const f32x4v*)(dp + o);
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if ((uint8_t)(ib >> (8 * e)) == pos) acc[e] += gv[e];
    }
  }
#pragma unroll
  for (int e = 0; e < 4; ++e)
    if (!(yy[e] * coef[c0 + e] + coef[C + c0 + e] > 0.f)) acc[e] = 0.f;
  return acc;
}

__global__ __launch_bounds__(256) void stem_pool_bwd_reduce32_kernel(const float* __restrict__ dp,
                                                                     const uint8_t* __restrict__ idx,
                                                                     const float* __restrict__ y,
                                                                     const float* __restrict__ coef,
                                                                     float* __restrict__ srows, int N, int H, int W,
                                                                     int C, int OH, int OW, FastDiv fw, FastDiv fh) {
  const int lanes_c = C / 4, rpi = 256 / lanes_c;
  const int cl = threadIdx.x % lanes_c, rl = threadIdx.x / lanes_c;
  const int64_t rows = (int64_t)N * H * W;
  const int c0 = cl * 4;
  float s0[4] = {0.f, 0.f, 0.f, 0.f}, s1[4] = {0.f, 0.f, 0.f, 0.f};
  if (rl < rpi) {
    const f32x4v mean = *(const f32x4v*)(coef + 2 * C + c0), istd = *(const f32x4v*)(coef + 3 * C + c0);
    for (int64_t r = (int64_t)blockIdx.x * rpi + rl; r < rows; r += (int64_t)gridDim.x * rpi) {
      const int pix = (int)r;
      const int nh = (int)fdiv((uint32_t)pix, fw), w = pix - nh * W;
      const int n = (int)fdiv((uint32_t)nh, fh), h = nh - n * H;
      const f32x4v yy = *(const f32x4v*)(y + r * C + c0);
      const f32x4v dz = stem_pool_dz32(dp, idx, yy, coef, n, h, w, c0, C, OH, OW);
      const f32x4v x1 = (yy - mean) * istd;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        s0[e] += dz[e];
        s1[e] += dz[e] * x1[e];
      }
    }
  }
  extern __shared__ float red[];  // [rpi][C][2]
  if (rl < rpi) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      red[((int64_t)rl * C + c0 + e) * 2 + 0] = s0[e];
      red[((int64_t)rl * C + c0 + e) * 2 + 1] = s1[e];
    }
  }
  __syncthreads();
  float* dst = srows + (int64_t)blockIdx.x * C * 2;
  for (int i = threadIdx.x; i < C * 2; i += 256) {
    float tt = 0.f;
    for (int q = 0; q < rpi; ++q) tt += red[(int64_t)q * C * 2 + i];
    dst[i] = tt;
  }
}

void stem_pool_bwd_reduce32_launch(const float* dp, const uint8_t* idx, const float* y, const float* coef, double* slots,
                                   int blocks, int N, int H, int W, int C, hipStream_t s) {
  if (C % 4 != 0 || C / 4 > 256 || 256 % (C / 4) != 0)
    pdt_hip_fail("stem_pool_bwd_reduce32: C / 4 must divide 256", hipErrorInvalidValue, __FILE__, __LINE__);
  const int OH = (H + 2 - 3) / 2 + 1, OW = (W + 2 - 3) / 2 + 1;
  PDT_COUNT("stem_pool_bwd_fused32");
  const int rpi = 256 / (C / 4);
  Scratch part((size_t)blocks * C * 2 * sizeof(float), s);
  float* srows = part.as<float>();
  hipLaunchKernelGGL(stem_pool_bwd_reduce32_kernel, dim3(blocks), dim3(256), (size_t)rpi * C * 2 * sizeof(float), s, dp,
                     idx, y, coef, srows, N, H, W, C, OH, OW, make_fastdiv((uint32_t)W), make_fastdiv((uint32_t)H));
  stat_rows_reduce_launch(srows, blocks, C * 2, slots, s);
}

// The stem's BN-backward sums without touching the 112x112 tensors: the pooled output IS relu(scale*y + shift) at the
// window's argmax, so the ReLU mask there is (out > 0) and the BatchNorm input is y = (out - shift) / scale; summed
// over pooled elements, sum dz = sum dp * [out > 0] and sum dz*xhat = sum dp * [out > 0] * xhat(y) -- every pixel's dz
// is the sum of the dp of the windows that selected it, all with the same xhat.  Reads the two pooled tensors (2 x
// 0.96 GB fp32 at ResNet-18 B = 1200) instead of gathering windows + the 3.85 GB conv output (the fp32 twin of
// stem_pool_bwd_reduce_out_kernel; scale == 0, i.e. gamma == 0, contributes xhat = 0).
__global__ __launch_bounds__(256) void stem_pool_bwd_reduce_out32_kernel(const float* __restrict__ dp,
                                                                         const float* __restrict__ out,
                                                                         const float* __restrict__ coef,
                                                                         float* __restrict__ srows, int64_t rows, int C) {
  const int lanes_c = C / 4, rpi = 256 / lanes_c;
  const int cl = threadIdx.x % lanes_c, rl = threadIdx.x / lanes_c;
  const int c0 = cl * 4;
  float s0[4] = {0.f, 0.f, 0.f, 0.f}, s1[4] = {0.f, 0.f, 0.f, 0.f};
  if (rl < rpi) {
    float rsc[4], sh[4], mu[4], is[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float sc = coef[c0 + e];
      rsc[e] = sc != 0.f ? 1.f / sc : 0.f;
      sh[e] = coef[C + c0 + e];
      mu[e] = coef[2 * C + c0 + e];
      is[e] = coef[3 * C + c0 + e];
    }
    for (int64_t r = (int64_t)blockIdx.x * rpi + rl; r < rows; r += (int64_t)gridDim.x * rpi) {
      const f32x4v g = *(const f32x4v*)(dp + r * C + c0);
      const f32x4v ov = *(const f32x4v*)(out + r * C + c0);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float dz = ov[e] > 0.f ? g[e] : 0.f;
        const float xhat = rsc[e] != 0.f ? ((ov[e] - sh[e]) * rsc[e] - mu[e]) * is[e] : 0.f;
        s0[e] += dz;
        s1[e] += dz * xhat;
      }
    }
  }
  extern __shared__ float red[];  // [rpi][C][2]
  if (rl < rpi) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
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

void stem_pool_bwd_reduce_out32_launch(const float* dp, const float* out, const float* coef, double* slots, int blocks,
                                       int64_t rows, int C, hipStream_t s) {
  if (C % 4 != 0 || C / 4 > 256 || 256 % (C / 4) != 0)
    pdt_hip_fail("stem_pool_bwd_reduce_out32: C / 4 must divide 256", hipErrorInvalidValue, __FILE__, __LINE__);
  PDT_COUNT("stem_pool_bwd_reduce_out32");
  const int rpi = 256 / (C / 4);
  Scratch part((size_t)blocks * C * 2 * sizeof(float), s);
  float* srows = part.as<float>();
  hipLaunchKernelGGL(stem_pool_bwd_reduce_out32_kernel, dim3(blocks), dim3(256), (size_t)rpi * C * 2 * sizeof(float), s,
                     dp, out, coef, srows, rows, C);
  stat_rows_reduce_launch(srows, blocks, C * 2, slots, s);
}

// dy = A*dz + B*y + C with dz recomputed (stem_pool_dz32): bn_bwd_apply32<false, 1, false> over maxpool_bwd_relu32's dz
__global__ __launch_bounds__(256) void stem_pool_bwd_apply32_kernel(const float* __restrict__ dp,
                                                                    const uint8_t* __restrict__ idx,
                                                                    const float* __restrict__ y,
                                                                    const float* __restrict__ coef,
                                                                    const float* __restrict__ b, float* __restrict__ dy,
                                                                    int N, int H, int W, int C, int OH, int OW, FastDiv fw,
                                                                    FastDiv fh) {
  const int cv = C / 4;  // a power of two (host-checked)
  const int cshift = __builtin_ctz(cv);
  const int64_t total = (int64_t)N * H * W * cv;
  for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < total; v += (int64_t)gridDim.x * 256) {
    const int pix = (int)(v >> cshift);
    const int c0 = (int)(v - ((int64_t)pix << cshift)) * 4;
    const int nh = (int)fdiv((uint32_t)pix, fw), w = pix - nh * W;
    const int n = (int)fdiv((uint32_t)nh, fh), h = nh - n * H;
    const f32x4v yy = ((const f32x4v*)y)[v];
    const f32x4v dz = stem_pool_dz32(dp, idx, yy, coef, n, h, w, c0, C, OH, OW);
    ((f32x4v*)dy)[v] = *(const f32x4v*)(b + c0) * dz + *(const f32x4v*)(b + C + c0) * yy + *(const f32x4v*)(b + 2 * C + c0);
  }
}

void stem_pool_bwd_apply32_launch(const float* dp, const uint8_t* idx, const float* y, const float* coef, const float* b,
                                  float* dy, int N, int H, int W, int C, hipStream_t s) {
  const int OH = (H + 2 - 3) / 2 + 1, OW = (W + 2 - 3) / 2 + 1;
  if (C % 4 != 0 || ((C / 4) & (C / 4 - 1)) != 0)
    pdt_hip_fail("stem_pool_bwd_apply32: C / 4 must be a power of two", hipErrorInvalidValue, __FILE__, __LINE__);
  hipLaunchKernelGGL(stem_pool_bwd_apply32_kernel, dim3(ew_blocks((int64_t)N * H * W * (C / 4))), dim3(256), 0, s, dp,
                     idx, y, coef, b, dy, N, H, W, C, OH, OW, make_fastdiv((uint32_t)W), make_fastdiv((uint32_t)H));
}

// global average pool [N][HW][C] -> feat [N][ldf] (columns >= C are left alone) and its backward
__global__ __launch_bounds__(256) void avgpool32_fwd_kernel(const float* __restrict__ x, float* __restrict__ feat, int N,
                                                            int HW, int C, int ldf) {
  const int64_t total = (int64_t)N * C;
  for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < total; v += (int64_t)gridDim.x * 256) {
    const int n = (int)(v / C), c = (int)(v - (int64_t)n * C);
    const float* p = x + (int64_t)n * HW * C + c;
    float s = 0.f;
    for (int i = 0; i < HW; ++i) s += p[(int64_t)i * C];
    feat[(int64_t)n * ldf + c] = s / (float)HW;
  }
}

__global__ __launch_bounds__(256) void avgpool32_bwd_kernel(const float* __restrict__ dfeat, float* __restrict__ g, int N,
                                                            int HW, int C, int ldf) {
  const int64_t total = (int64_t)N * HW * C;
  const float inv = 1.f / (float)HW;
  for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < total; v += (int64_t)gridDim.x * 256) {
    const int c = (int)(v % C);
    const int n = (int)(v / ((int64_t)HW * C));
    g[v] = dfeat[(int64_t)n * ldf + c] * inv;
  }
}

void avgpool32_fwd_launch(const float* x, float* feat, int N, int HW, int C, int ldf, hipStream_t s) {
  hipLaunchKernelGGL(avgpool32_fwd_kernel, dim3(ew_blocks((int64_t)N * C)), dim3(256), 0, s, x, feat, N, HW, C, ldf);
}

void avgpool32_bwd_launch(const float* dfeat, float* g, int N, int HW, int C, int ldf, hipStream_t s) {
  hipLaunchKernelGGL(avgpool32_bwd_kernel, dim3(ew_blocks((int64_t)N * HW * C)), dim3(256), 0, s, dfeat, g, N, HW, C,
                     ldf);
}

// softmax cross-entropy forward + backward + top-1 (first maximum) over fp32 logits, one wave per row
__global__ __launch_bounds__(256) void xent32_kernel(const float* __restrict__ logits, int ldl, const float* __restrict__ bias,
                                                     const int64_t* __restrict__ target, int B, int ncls,
                                                     float* __restrict__ out_logits, float* __restrict__ dlogits,
                                                     const float* __restrict__ loss_scale, float grad_div,
                                                     float* __restrict__ row_loss, float* __restrict__ row_correct) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= B) return;
  const float* lr = logits + (int64_t)row * ldl;
  const int tgt = (int)target[row];
  float mx = -INFINITY;
  int amax = 0x7fffffff;
  for (int c = lane; c < ncls; c += 64) {
    const float v = lr[c] + (bias ? bias[c] : 0.f);
    if (out_logits) out_logits[(int64_t)row * ncls + c] = v;
    if (v > mx) { mx = v; amax = c; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(mx, o, 64);
    const int oa = __shfl_xor(amax, o, 64);
    if (om > mx || (om == mx && oa < amax)) { mx = om; amax = oa; }
  }
  float se = 0.f;
  for (int c = lane; c < ncls; c += 64) se += __expf(lr[c] + (bias ? bias[c] : 0.f) - mx);
  se = wave_sum(se);
  const float lse = mx + __logf(se);
  const float xt = lr[tgt] + (bias ? bias[tgt] : 0.f);
  if (dlogits) {
    const float gsc = (loss_scale ? *loss_scale : 1.f) / grad_div;
    float* dr = dlogits + (int64_t)row * ldl;
    const float inv = 1.f / se;
    for (int c = lane; c < ldl; c += 64) {
      float d = 0.f;
      if (c < ncls) d = (__expf(lr[c] + (bias ? bias[c] : 0.f) - mx) * inv - (c == tgt ? 1.f : 0.f)) * gsc;
      dr[c] = d;
    }
  }
  if (lane == 0) {
    row_loss[row] = lse - xt;
    row_correct[row] = (amax == tgt) ? 1.f : 0.f;
  }
}

void xent32_launch(const float* logits, int ldl, const float* bias, const int64_t* target, int B, int ncls,
                   float* out_logits, float* dlogits, const float* loss_scale, float grad_div, float* row_loss,
                   float* row_correct, hipStream_t s) {
  hipLaunchKernelGGL(xent32_kernel, dim3((B + 3) / 4), dim3(256), 0, s, logits, ldl, bias, target, B, ncls, out_logits,
                     dlogits, loss_scale, grad_div, row_loss, row_correct);
}

// out[c] = scale * sum_b d[b][c]: 64 columns x 4 row lanes per block, fixed-order LDS reduction
__global__ __launch_bounds__(256) void colsum32_kernel(const float* __restrict__ d, int B, int ld, int ncols,
                                                       float* __restrict__ out, float scale) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63), rl = threadIdx.x >> 6;
  float s = 0.f;
  if (c < ncols)
    for (int b = rl; b < B; b += 4) s += d[(int64_t)b * ld + c];
  __shared__ float red[4][64];
  red[rl][threadIdx.x & 63] = s;
  __syncthreads();
  if (rl == 0 && c < ncols)
    out[c] = scale * (((red[0][threadIdx.x] + red[1][threadIdx.x]) + red[2][threadIdx.x]) + red[3][threadIdx.x]);
}

void colsum32_launch(const float* d, int B, int ld, int ncols, float* out, float scale, hipStream_t s) {
  hipLaunchKernelGGL(colsum32_kernel, dim3((ncols + 63) / 64), dim3(256), 0, s, d, B, ld, ncols, out, scale);
}

// fp32 NCHW images -> zero-padded NHWC4: one thread per padded pixel, one 16-byte store
__global__ __launch_bounds__(256) void stem_pack32_kernel(const float* __restrict__ x, float* __restrict__ out, int C,
                                                          int H, int W, int pad, int Hp, int Wp, int64_t total) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int wp = (int)(i % Wp);
  const int64_t t = i / Wp;
  const int hp = (int)(t % Hp);
  const int n = (int)(t / Hp);
  const int h = hp - pad, w = wp - pad;
  float v[4] = {0.f, 0.f, 0.f, 0.f};
  if ((unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W) {
#pragma unroll
    for (int c = 0; c < 3; ++c)
      if (c < C) v[c] = x[(((int64_t)n * C + c) * H + h) * W + w];
  }
  *(f32x4v*)(out + i * 4) = f32x4v{v[0], v[1], v[2], v[3]};
}

void stem_pack32_launch(const float* x, float* out, int N, int C, int H, int W, int pad, int Hp, int Wp, hipStream_t s) {
  const int64_t total = (int64_t)N * Hp * Wp;
  hipLaunchKernelGGL(stem_pack32_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, x, out, C, H, W, pad,
                     Hp, Wp, total);
}

// fp32 NCHW images -> im2col rows [N*OH*OW][ldk], column k = (r*S + s)*C + c (zero beyond R*S*C / outside)
// One thread per (output pixel, 4 consecutive columns): the KRSC column order k = (r*S + s)*C + c, zero past R*S*C,
// written as one 16-byte store (a wave writes 1 KB contiguous); the 4 gathered inputs come from NCHW rows that
// neighbouring pixels share (L2 hits).  32-bit index math with FastDiv (the old version did two 64-bit divisions
// and modulos per element and streamed at ~1.3 TB/s: 18.5 ms of a 155 ms fp32 ResNet-18 step).
template <int CT, int ST>
__global__ __launch_bounds__(256) void im2col32_kernel(const float* __restrict__ x, float* __restrict__ out, int C_,
                                                       int H, int W, int R, int S_, int stride, int pad, int OH, int OW,
                                                       int ldk, uint32_t nchunk, FastDiv fd_cpp, FastDiv fd_ow,
                                                       FastDiv fd_oh) {
  const int C = CT > 0 ? CT : C_, S = ST > 0 ? ST : S_;
  const int KK = R * S * C;
  const uint32_t cpp = (uint32_t)ldk / 4u;
  for (uint32_t v = blockIdx.x * 256u + threadIdx.x; v < nchunk; v += gridDim.x * 256u) {
    const uint32_t pix = fdiv(v, fd_cpp);
    const int j = (int)(v - pix * cpp);
    const uint32_t t1 = fdiv(pix, fd_ow);
    const int ow = (int)(pix - t1 * (uint32_t)OW);
    const uint32_t n = fdiv(t1, fd_oh);
    const int oh = (int)(t1 - n * (uint32_t)OH);
    const int h0 = oh * stride - pad, w0 = ow * stride - pad;
    const float* xn = x + (int64_t)n * C * H * W;
    float4 o;
    float* op = reinterpret_cast<float*>(&o);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = 4 * j + e;
      float val = 0.f;
      if (k < KK) {
        const int c = k % C, rs = k / C;
        const int r = rs / S, s_ = rs - r * S;
        const int h = h0 + r, w = w0 + s_;
        if ((unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W) val = xn[((int64_t)c * H + h) * W + w];
      }
      op[e] = val;
    }
    *reinterpret_cast<float4*>(out + (int64_t)v * 4) = o;
  }
}

void im2col32_launch(const float* x, float* out, int N, int C, int H, int W, int R, int S, int stride, int pad, int ldk,
                     hipStream_t s) {
  const int OH = (H + 2 * pad - R) / stride + 1, OW = (W + 2 * pad - S) / stride + 1;
  const int64_t nchunk = (int64_t)N * OH * OW * (ldk / 4);
  if (nchunk <= 0) return;
  if (ldk % 4 != 0 || nchunk >= (int64_t(1) << 31))
    pdt_hip_fail("im2col32: ldk % 4 != 0 or more than 2^31 output chunks", hipErrorInvalidValue, __FILE__, __LINE__);
  const FastDiv fc = make_fastdiv((uint32_t)(ldk / 4)), fw = make_fastdiv((uint32_t)OW), fh = make_fastdiv((uint32_t)OH);
  const int64_t blocks64 = (nchunk + 255) / 256;
  const unsigned blocks = (unsigned)(blocks64 < 65536 ? blocks64 : 65536);
  if (C == 3 && S == 7)  // the ResNet stem: constant divisors
    hipLaunchKernelGGL((im2col32_kernel<3, 7>), dim3(blocks), dim3(256), 0, s, x, out, C, H, W, R, S, stride, pad, OH,
                       OW, ldk, (uint32_t)nchunk, fc, fw, fh);
  else
    hipLaunchKernelGGL((im2col32_kernel<0, 0>), dim3(blocks), dim3(256), 0, s, x, out, C, H, W, R, S, stride, pad, OH,
                       OW, ldk, (uint32_t)nchunk, fc, fw, fh);
}

}  // namespace pdt
