// Convolution weight gradient on MFMA (gfx950), split-K over pixels.
//
//   dW[k][tap][c] = sum_{pixels p} dY[p][k] * X[in(p, tap)][c]
//
// GEMM view: rows = input channels c of one tap (MFMA A = gathered X), cols = output channels k
// (MFMA B = dY), reduction over pixels.  Both operands are pixel-major in NHWC memory, so tiles are
// DMA'd into LDS as [pixel][channel] rows (global_load_lds_dwordx4, 16 B/lane) and the MFMA fragments
// are read with the gfx950 transposing LDS read ds_read_b64_tr_b16.  The LDS image is XOR-swizzled
// through the DMA source address so those transposed reads are bank-conflict free.
//
// Block tile: 64 (c) x 64 (k) x 128 pixels per K-step, 4 waves each owning a 32-pixel slice of every
// K-step and a full 64x64 accumulator; the waves are summed through LDS at the end and each block
// writes one fp32 partial tile.  Partials over the split-K axis are summed by wgrad_reduce, which
// writes (and scales) straight into the fp32 gradient buffer (the DDP bucket view).
#include <cstdlib>
#include <type_traits>

#include "../common.h"
#include "conv_wgrad.h"

namespace pdt {

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void glb_void;
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4;

// chunk swizzle for a [pixel][64 ch] (128-B row) image read by ds_read_b64_tr_b16
PDT_DEVICE int tr_swz(int row) { return (((row >> 1) & 1) << 1) | (((row >> 3) & 1) << 2); }

// Byte offsets of one DMA lane's source rows for pixel p of the K-step: X gathered through the tap,
// dY linear.  32-bit arithmetic; padding reads kOOB (zeros) and pixels past the end of the tensors land
// beyond the buffers' num_records (zeros), so no per-lane "live" test is needed (splits are multiples
// of the K-step).
template <bool WIN>
PDT_DEVICE void wgrad_rows(const ConvWgradArgs& a, int p, int th, int tw, int xcol, int lch, int ycol,
                           uint32_t& xoff, uint32_t& yoff) {
  const FastDiv dpq{a.div_pq_mul, a.div_pq_shift}, dq{a.div_q_mul, a.div_q_shift};
  const int PQ = a.Pm * a.Qm;
  const int nimg = (int)fdiv((uint32_t)p, dpq);
  const int rem = p - nimg * PQ;
  const int i = (int)fdiv((uint32_t)rem, dq);
  const int jj = rem - i * a.Qm;
  const int h = i * a.stride_h + th, w = jj * a.stride_w + tw;
  if constexpr (WIN) {
    xoff = (uint32_t)((((nimg * a.H + h + (lch >> 2)) * a.W + w) * a.cs + (lch & 3) * 8) * 2);
  } else {
    const bool ok = (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W;
    const uint32_t off = (uint32_t)((((nimg * a.H + h) * a.W + w) * a.cs + xcol + lch * 8) * 2);
    xoff = ok ? off : kOOB;
  }
  yoff = (uint32_t)(p * (a.ldy ? a.ldy : a.Kout) + ycol + lch * 8) * 2u;
}

// WIN: the ResNet stem's "window" mode.  X is the zero-padded NHWC4 image and a 64-wide tile column
// block covers two kernel rows of 8 pixels x 4 channels: chunk ch (8 elements) reads image row
// (h + (ch >> 2)) at element offset (ch & 3) * 8 -- im2col is never materialised.
template <int DT, bool WIN>
__global__ __launch_bounds__(256) void conv_wgrad_kernel(ConvWgradArgs a) {
  int sl = 0;
  if (a.nslice > 1) {  // slice-batched grouped conv: this block's channel slice
    sl = blockIdx.z;
    a.x += (int64_t)sl * a.C;
    a.dy += (int64_t)sl * a.Kout;
  }
  using E = E16<DT>;
  typedef typename E::vec8 vec8;
  constexpr int BKP = 128;       // pixels per K-step
  constexpr int ROWB = 128;      // 64 channels * 2 B
  constexpr int XB = BKP * ROWB; // bytes of the X tile
  constexpr int STAGE = 2 * XB;
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

  // block -> (k tile, (tap, c) tile, split)
  const int c_tiles = a.C / 64;
  const int n_tiles = a.T * a.U * c_tiles;
  const int k_tiles = a.Kout / 64;
  const int nwg = k_tiles * n_tiles * a.splits;
  const int bid = xcd_remap(blockIdx.x, nwg);
  // consecutive blocks (one XCD after the remap) = different tiles of the SAME pixel range, so the
  // dY / X rows a split streams are fetched from HBM once and re-read from that XCD's L2
  const int tile = bid % (k_tiles * n_tiles);
  const int split = bid / (k_tiles * n_tiles);
  const int kt = tile % k_tiles;
  const int nt = tile / k_tiles;
  const int tap = nt / c_tiles;
  const int c0 = (nt - tap * c_tiles) * 64;
  const int k0 = kt * 64;
  const int t = tap / a.U, u = tap - (tap / a.U) * a.U;

  const int pix_begin = split * a.pix_per_split;
  const int pix_end = min(a.P, pix_begin + a.pix_per_split);
  const int nsteps = (pix_end - pix_begin + BKP - 1) / BKP;

  const int th = t * a.dil_h - a.pad_h, tw = u * a.dil_w - a.pad_w;
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(a.x, (uint32_t)a.N * a.H * a.W * a.cs * 2u);
  const __amdgpu_buffer_rsrc_t ry = make_rsrc(a.dy, (uint32_t)a.P * (a.ldy ? a.ldy : a.Kout) * 2u);

  // DMA lane geometry: 8 rows x 8 chunks per 1 KiB instruction
  const int lrow = lane >> 3, pch = lane & 7;

  auto stage_load = [&](int step, int buf) {
    const int pbase = pix_begin + step * BKP;
    char* sb = smem + buf * STAGE;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = (wave * 4 + j) * 8 + lrow;  // 0..127
      const int lch = pch ^ tr_swz(row);
      uint32_t xo, yo;
      wgrad_rows<WIN>(a, pbase + row, th, tw, c0, lch, k0, xo, yo);
      buf_lds16_asm(rx, sb + (wave * 4 + j) * 1024, xo);
      buf_lds16_asm(ry, sb + XB + (wave * 4 + j) * 1024, yo);
    }
  };

  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // transposed-read lane geometry: group g = lane>>4 holds k = 8g..8g+7 of the 32-pixel slice
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p4 = li & 3;

  if (nsteps > 0) {
    stage_load(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int s = 0; s < nsteps; ++s) {
      const int cur = s & 1;
      if (s + 1 < nsteps) stage_load(s + 1, cur ^ 1);
      const char* sb = smem + cur * STAGE;
      vec8 af[4], bfr[4];
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        s16x4_t lo, hi;
        {
          const int row0 = wave * 32 + 8 * g + q;
          const int col = f * 16 + 4 * p4;  // element within the 64-wide row
          const int ch = col >> 3, off = (col & 7) * 2;
          const int r0 = row0, r1 = row0 + 4;
          lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (lds_s16x4*)(sb + r0 * ROWB + ((ch ^ tr_swz(r0)) << 4) + off));
          hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (lds_s16x4*)(sb + r1 * ROWB + ((ch ^ tr_swz(r1)) << 4) + off));
        }
        af[f] = __builtin_bit_cast(vec8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
        {
          const int row0 = wave * 32 + 8 * g + q;
          const int col = f * 16 + 4 * p4;
          const int ch = col >> 3, off = (col & 7) * 2;
          const int r0 = row0, r1 = row0 + 4;
          lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (lds_s16x4*)(sb + XB + r0 * ROWB + ((ch ^ tr_swz(r0)) << 4) + off));
          hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (lds_s16x4*)(sb + XB + r1 * ROWB + ((ch ^ tr_swz(r1)) << 4) + off));
        }
        bfr[f] = __builtin_bit_cast(vec8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = E::mfma16x16x32(af[i], bfr[j], acc[i][j]);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  }

  // ---- sum the 4 waves' 64x64 tiles through LDS, write one fp32 partial tile ----
  // acc[i][j]: rows c = 16i + 4*(lane>>4) + r, col k = 16j + (lane&15)
  float* red = (float*)smem;  // [4 waves][64 k][64 c]
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = 16 * j + (lane & 15);
      const int c = 16 * i + 4 * (lane >> 4);
      *(f32x4_t*)(red + (wave * 64 + k) * 64 + c) = acc[i][j];
    }
  __syncthreads();
  const int nsl = a.nslice > 1 ? a.nslice : 1;
  float* dst = a.ws + (((int64_t)split * nsl + sl) * a.Kout + k0) * a.ldw + tap * a.C + c0;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int idx = (e * 256 + tid) * 4;  // 0..4095
    const int k = idx >> 6, c = idx & 63;
    f32x4_t v = *(f32x4_t*)(red + k * 64 + c);
#pragma unroll
    for (int w = 1; w < 4; ++w) v += *(f32x4_t*)(red + (w * 64 + k) * 64 + c);
    *(f32x4_t*)(dst + (int64_t)k * a.ldw + c) = v;
  }
}

// ------------------------------------------------------------------------------------------------
// Stem ("window" mode) weight gradient: ALL FOUR kernel-row pairs of the 7x7 stem in one block.
// The 64x64 kernel above runs one block per (pair, split) and so re-reads every dY tile 4 times; here a
// block stages the dY tile once plus the 4 pair-windows of X (64 pixels x 128 B each, 40 KB per stage,
// 2 stages -> 2 blocks per CU) and wave t owns pair t's 64 (window column) x 64 (cout) tile over the
// whole pixel range of its split.  The partial tile goes out through LDS as coalesced float4 rows.
// (The training path fuses the stem's backward tail into the weight gradient instead: wgrad_stem_rows_kernel /
// wgrad_stem_quad_kernel below; this one serves a materialised dY, PDT_STEM_FUSED=0.)
template <int DT>
__global__ __launch_bounds__(256) void wgrad_stem_kernel(ConvWgradArgs a) {
  using E = E16<DT>;
  typedef typename E::vec8 vec8;
  constexpr int BKP = 64;         // pixels per K-step
  constexpr int ROWB = 128;       // 64 elements * 2 B
  constexpr int TB = BKP * ROWB;  // 8 KB per tile
  constexpr int STAGE = 5 * TB;   // dY + 4 pair windows
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // = kernel-row pair
  const int split = blockIdx.x;
  const int pix_begin = split * a.pix_per_split;
  const int pix_end = min(a.P, pix_begin + a.pix_per_split);
  const int nsteps = (pix_end - pix_begin + BKP - 1) / BKP;
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(a.x, (uint32_t)a.N * a.H * a.W * a.cs * 2u);
  const __amdgpu_buffer_rsrc_t ry = make_rsrc(a.dy, (uint32_t)a.P * a.Kout * 2u);
  const int lrow = lane >> 3, pch = lane & 7;

  // 40 DMA instructions per stage (8 dY + 4 x 8 X), 10 per wave
  auto stage_load = [&](int step, int buf) {
    const int pbase = pix_begin + step * BKP;
    char* sb = smem + buf * STAGE;
#pragma unroll
    for (int m = 0; m < 10; ++m) {
      const int ii = wave + 4 * m;
      const int tile = ii >> 3;                 // 0 = dY, 1..4 = pair tile-1
      const int row = (ii & 7) * 8 + lrow;      // pixel within the step
      const int lch = pch ^ tr_swz(row);
      const int th = (tile - 1) * a.dil_h - a.pad_h;
      uint32_t xo, yo;
      wgrad_rows<true>(a, pbase + row, th, 0, 0, lch, 0, xo, yo);
      if (tile == 0)
        buf_lds16_asm(ry, sb + (ii & 7) * 1024, yo);
      else
        buf_lds16_asm(rx, sb + tile * TB + (ii & 7) * 1024, xo);
    }
  };

  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p4 = li & 3;

  if (nsteps > 0) {
    stage_load(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int st = 0; st < nsteps; ++st) {
      const int cur = st & 1;
      if (st + 1 < nsteps) stage_load(st + 1, cur ^ 1);
      const char* sy = smem + cur * STAGE;
      const char* sx = sy + (1 + wave) * TB;
#pragma unroll
      for (int kk = 0; kk < BKP / 32; ++kk) {
        const int r0 = kk * 32 + 8 * g + q, r1 = r0 + 4;
        const int sw0 = tr_swz(r0), sw1 = tr_swz(r1);
        vec8 af[4], bfr[4];
#pragma unroll
        for (int f = 0; f < 4; ++f) {
          const int col = f * 16 + 4 * p4;
          const int ch = col >> 3, off = (col & 7) * 2;
          s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (lds_s16x4*)(sx + r0 * ROWB + ((ch ^ sw0) << 4) + off));
          s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (lds_s16x4*)(sx + r1 * ROWB + ((ch ^ sw1) << 4) + off));
          af[f] = __builtin_bit_cast(vec8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
          lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(sy + r0 * ROWB + ((ch ^ sw0) << 4) + off));
          hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(sy + r1 * ROWB + ((ch ^ sw1) << 4) + off));
          bfr[f] = __builtin_bit_cast(vec8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = E::mfma16x16x32(af[i], bfr[j], acc[i][j]);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  }
  // acc[i][j]: rows (window column) c = 16i + 4*(lane>>4) + r, col k = 16j + (lane&15); transpose
  // through LDS ([4 pairs][64 k][64 c]) and write ws[split][k][pair*64 + c] as float4 rows
  float* red = (float*)smem;
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = 16 * j + (lane & 15);
      const int c = 16 * i + 4 * (lane >> 4);
      *(f32x4_t*)(red + (wave * 64 + k) * 64 + c) = acc[i][j];
    }
  __syncthreads();
  float* dst = a.ws + (int64_t)split * a.Kout * a.ldw;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int idx = (e * 256 + tid) * 4;  // 0..16383 over [k][pair][c]
    const int k = idx >> 8, pc = idx & 255, pr = pc >> 6, c = pc & 63;
    *(f32x4_t*)(dst + (int64_t)k * a.ldw + pc) = *(const f32x4_t*)(red + (pr * 64 + k) * 64 + c);
  }
}

// ------------------------------------------------------------------------------------------------
// The fused stem weight gradient over 2x2 pixel QUADS (round 5).  The GEMM's reduction runs over pixels in any
// order, so a K-step's 64 pixels are 16 quads (conv rows 2r, 2r+1 x columns 2s, 2s+1), in (image, r, s) order.
// A quad's four pixels draw their max-pool gradient from exactly the four pooling windows (r | r+1, s | s+1) --
// the same four windows a pixel-PAIR form (round 4) loaded for just two pixels -- and each window's
// argmax can select at most one pixel of the quad:
//     (2r, 2s)     <- (r, s) at tap 4
//     (2r, 2s+1)   <- (r, s) tap 5, (r, s+1) tap 3
//     (2r+1, 2s)   <- (r, s) tap 7, (r+1, s) tap 1
//     (2r+1, 2s+1) <- (r, s) tap 8, (r, s+1) tap 6, (r+1, s) tap 2, (r+1, s+1) tap 0
// so per element the max-pool backward is 9/4 compare-selects instead of 3, and the window loads and decodes are
// shared by four pixels instead of two (the kernel is VALU-issue bound: r4_after_pmc.md, 53 % active / 11 % wait).
// The sums add the windows in the same order as the separate apply pass (stem_pool_bwd_apply), so dY is
// bit-identical to it.  A thread owns one quad x 4 channels.  An odd
// conv-output height leaves the quads of the last row half dead (zero rows on both GEMM sides).  Pipeline, LDS
// images and MFMA part as wgrad_stem_kernel: 12 operand loads per thread per step.  Serves the shapes the
// raw-row kernel below does not (conv output not a multiple of 4 x 16 pixels).
PDT_DEVICE uint32_t gload4_asm(const void* p) {
  uint32_t v;
  asm volatile("global_load_dword %0, %1, off" : "=v"(v) : "v"(p));
  return v;
}

template <int DT>
__global__ __launch_bounds__(256) void wgrad_stem_quad_kernel(ConvWgradArgs a) {
  using E = E16<DT>;
  typedef typename E::vec8 vec8;
  constexpr int BKP = 64;         // pixels (16 quads) per K-step
  constexpr int ROWB = 128;       // 64 elements * 2 B
  constexpr int TB = BKP * ROWB;  // 8 KB per tile
  constexpr int STAGE = 5 * TB;   // dY + 4 pair windows
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // = kernel-row pair
  const int split = blockIdx.x;
  const int pix_begin = split * a.pix_per_split;
  const int pix_end = min(a.P, pix_begin + a.pix_per_split);  // a.P: quad-padded pixel count (launcher)
  const int nsteps = (pix_end - pix_begin + BKP - 1) / BKP;
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(a.x, (uint32_t)a.N * a.H * a.W * a.cs * 2u);
  const int lrow = lane >> 3, pch = lane & 7;
  const int QR = (a.Pm + 1) >> 1, QC = a.Qm >> 1;  // quad rows / columns per image
  const FastDiv dqimg{a.div_pq_mul, a.div_pq_shift}, dqc{a.div_q_mul, a.div_q_shift};  // by QR*QC, by QC

  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p4 = li & 3;

  // X DMA: rows ra = wave*8 + lrow and rb = ra + 32 of the step (pixel p = 4 * quad + sub), 4 pairs each
  const uint32_t pair_step = (uint32_t)a.dil_h * a.W * a.cs * 2u;
  auto x_off = [&](int p, int lch) -> uint32_t {
    const int qd = p >> 2, sub = p & 3;
    const int nimg = (int)fdiv((uint32_t)qd, dqimg);
    const int rem = qd - nimg * (QR * QC);
    const int r = (int)fdiv((uint32_t)rem, dqc), sc = rem - r * QC;
    const int h = 2 * r + (sub >> 1), w = 2 * sc + (sub & 1);
    // dead half-quad of an odd height: zero row (kOOB); pixels past the tensor land past num_records (zeros)
    if (h >= a.Pm) return kOOB;
    return (uint32_t)((((nimg * a.H + h * a.stride_h - a.pad_h + (lch >> 2)) * a.W + w * a.stride_w) * a.cs +
                       (lch & 3) * 8) * 2);
  };
  auto stage_load_x = [&](int step, int buf) {
    const int pbase = pix_begin + step * BKP;
    char* sb = smem + buf * STAGE;
    const int ra = wave * 8 + lrow, rb = ra + 32;
    const int lch = pch ^ tr_swz(ra);  // == pch ^ tr_swz(rb)
    const uint32_t xa = x_off(pbase + ra, lch), xb = x_off(pbase + rb, lch);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      buf_lds16_asm(rx, sb + (1 + t) * TB + wave * 1024, xa == kOOB ? kOOB : xa + t * pair_step);
      buf_lds16_asm(rx, sb + (1 + t) * TB + (wave + 4) * 1024, xb == kOOB ? kOOB : xb + t * pair_step);
    }
  };

  // ---- dY: quad qd of the step, channels 4*cg .. 4*cg + 3
  const int qd = tid >> 4, cg = tid & 15;
  // (the ReLU mask is in the argmax: bn_relu_maxpool marks windows whose maximum is 0 dead, so f_coef is not read)
  float fA[4], fB[4], fC[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int c = cg * 4 + e;
    fA[e] = a.f_bcoef[c]; fB[e] = a.f_bcoef[64 + c]; fC[e] = a.f_bcoef[128 + c];
  }
  u32x2v fy[4], fg[4];  // asm loads (common.h gload*_asm): waited for by QUAD_WAIT, which also carries them as
                        // operands so no use can be scheduled ahead of it
  uint32_t fi[4];
  int fvalid = 0;       // bit 0: quad live, bit 1: row 2r+1 live, bit 2: window row r+1, bit 3: window column s+1
  auto dy_load = [&](int step) {
    const int qg = (pix_begin + step * BKP) / 4 + qd;
    const bool live = qg * 4 < a.P;
    const int qq = live ? qg : 0;
    const int nimg = (int)fdiv((uint32_t)qq, dqimg);
    const int rem = qq - nimg * (QR * QC);
    const int r = (int)fdiv((uint32_t)rem, dqc), sc = rem - r * QC;
    const bool row1 = 2 * r + 1 < a.Pm;
    const bool okr = r + 1 < a.f_OH, oks = sc + 1 < a.f_OW;
#pragma unroll
    for (int sub = 0; sub < 4; ++sub) {
      const int h = min(2 * r + (sub >> 1), a.Pm - 1), w = 2 * sc + (sub & 1);
      fy[sub] = gload8_asm(a.f_y + ((uint32_t)(nimg * a.Pm + h) * a.Qm + w) * 64u + cg * 4);
    }
#pragma unroll
    for (int wi = 0; wi < 4; ++wi) {
      const int wr = (wi >> 1) && okr ? r + 1 : r, wc = (wi & 1) && oks ? sc + 1 : sc;
      const uint32_t o = (((uint32_t)nimg * a.f_OH + wr) * a.f_OW + wc) * 64u + cg * 4;
      fi[wi] = gload4_asm(a.f_idx + o);
      fg[wi] = gload8_asm(a.f_dp + o);
    }
    fvalid = (live ? 1 : 0) | (row1 ? 2 : 0) | (okr ? 4 : 0) | (oks ? 8 : 0);
  };
  auto dy_store = [&](int buf) {
    char* sy = smem + buf * STAGE;
    // missing windows select nothing (position 255); a dead quad or half-quad stores zero rows
    const uint32_t i0 = fi[0], i1 = fvalid & 8 ? fi[1] : 0xffffffffu, i2 = fvalid & 4 ? fi[2] : 0xffffffffu;
    const uint32_t i3 = (fvalid & 12) == 12 ? fi[3] : 0xffffffffu;
    const uint32_t keep0 = fvalid & 1 ? 0xffffffffu : 0u, keep1 = (fvalid & 3) == 3 ? 0xffffffffu : 0u;
    uint32_t ov[4][2];
    float dv[4][4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int sh = 16 * (e & 1);
      const uint32_t p0 = (i0 >> (8 * e)) & 0xffu, p1 = (i1 >> (8 * e)) & 0xffu;
      const uint32_t p2 = (i2 >> (8 * e)) & 0xffu, p3 = (i3 >> (8 * e)) & 0xffu;
      const float g0 = E::to_f((uint16_t)(fg[0][e >> 1] >> sh)), g1 = E::to_f((uint16_t)(fg[1][e >> 1] >> sh));
      const float g2 = E::to_f((uint16_t)(fg[2][e >> 1] >> sh)), g3 = E::to_f((uint16_t)(fg[3][e >> 1] >> sh));
      // branch-free (as conditional adds the compiler built a divergent switch on p0): selects of g or 0, summed
      // in window order (an unselected term adds an exact zero)
      float dz[4];
      dz[0] = p0 == 4 ? g0 : 0.f;
      dz[1] = (p0 == 5 ? g0 : 0.f) + (p1 == 3 ? g1 : 0.f);
      dz[2] = (p0 == 7 ? g0 : 0.f) + (p2 == 1 ? g2 : 0.f);
      dz[3] = (((p0 == 8 ? g0 : 0.f) + (p1 == 6 ? g1 : 0.f)) + (p2 == 2 ? g2 : 0.f)) + (p3 == 0 ? g3 : 0.f);
#pragma unroll
      for (int sub = 0; sub < 4; ++sub) {
        const float yv = E::to_f((uint16_t)(fy[sub][e >> 1] >> sh));
        dv[sub][e] = __builtin_fmaf(fA[e], dz[sub], __builtin_fmaf(fB[e], yv, fC[e]));
      }
    }
#pragma unroll
    for (int sub = 0; sub < 4; ++sub) {
      ov[sub][0] = E::pack2(dv[sub][0], dv[sub][1]);
      ov[sub][1] = E::pack2(dv[sub][2], dv[sub][3]);
    }
#pragma unroll
    for (int sub = 0; sub < 4; ++sub) {
      const int row = 4 * qd + sub;
      const uint32_t keep = sub < 2 ? keep0 : keep1;
      *(uint2*)(sy + row * ROWB + (((cg >> 1) ^ tr_swz(row)) << 4) + (cg & 1) * 8) =
          make_uint2(ov[sub][0] & keep, ov[sub][1] & keep);
    }
  };
  // step st+1's dY inputs are loaded at the end of step st-1 (after that step's dY tile was stored), so they have
  // all of step st to arrive: [loads(st+1): 12][DMA(st+1): 8] at the dY store (vmcnt(8): the DMA stays in flight
  // under the dY math), then [DMA(st+1): 8][loads(st+2): 12] before the barrier (vmcnt(12))
#define QUAD_WAIT(n)                                                                                     \
  asm volatile("s_waitcnt vmcnt(" #n ")"                                                                 \
               : "+v"(fy[0]), "+v"(fy[1]), "+v"(fy[2]), "+v"(fy[3]), "+v"(fi[0]), "+v"(fi[1]), "+v"(fi[2]), \
                 "+v"(fi[3]), "+v"(fg[0]), "+v"(fg[1]), "+v"(fg[2]), "+v"(fg[3])                         \
               :                                                                                         \
               : "memory")
  if (nsteps > 0) {
    dy_load(0);
    stage_load_x(0, 0);
    QUAD_WAIT(0);
    dy_store(0);
    if (nsteps > 1) dy_load(1);
    __syncthreads();
    for (int st = 0; st < nsteps; ++st) {
      const int cur = st & 1;
      if (st + 1 < nsteps) stage_load_x(st + 1, cur ^ 1);
      const char* sy = smem + cur * STAGE;
      const char* sx = sy + (1 + wave) * TB;
#pragma unroll
      for (int kk = 0; kk < BKP / 32; ++kk) {
        const int r0 = kk * 32 + 8 * g + q, r1 = r0 + 4;
        const int sw0 = tr_swz(r0), sw1 = tr_swz(r1);
        vec8 af[4], bfr[4];
#pragma unroll
        for (int f = 0; f < 4; ++f) {
          const int col = f * 16 + 4 * p4;
          const int ch = col >> 3, off = (col & 7) * 2;
          s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (lds_s16x4*)(sx + r0 * ROWB + ((ch ^ sw0) << 4) + off));
          s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (lds_s16x4*)(sx + r1 * ROWB + ((ch ^ sw1) << 4) + off));
          af[f] = __builtin_bit_cast(vec8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
          lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(sy + r0 * ROWB + ((ch ^ sw0) << 4) + off));
          hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(sy + r1 * ROWB + ((ch ^ sw1) << 4) + off));
          bfr[f] = __builtin_bit_cast(vec8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = E::mfma16x16x32(af[i], bfr[j], acc[i][j]);
      }
      __builtin_amdgcn_sched_barrier(0);  // the waits and the dY math stay behind the last MFMA
      if (st + 1 < nsteps) {
        QUAD_WAIT(8);
        __builtin_amdgcn_sched_barrier(0);
        dy_store(cur ^ 1);
        if (st + 2 < nsteps) {
          dy_load(st + 2);
          asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
        } else {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __syncthreads();
    }
  }
#undef QUAD_WAIT
  // acc[i][j]: rows (window column) c = 16i + 4*(lane>>4) + r, col k = 16j + (lane&15); transpose through LDS
  float* red = (float*)smem;
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = 16 * j + (lane & 15);
      const int c = 16 * i + 4 * (lane >> 4);
      *(f32x4_t*)(red + (wave * 64 + k) * 64 + c) = acc[i][j];
    }
  __syncthreads();
  float* dst = a.ws + (int64_t)split * a.Kout * a.ldw;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int idx = (e * 256 + tid) * 4;  // 0..16383 over [k][pair][c]
    const int k = idx >> 8, pc = idx & 255, pr = pc >> 6, c = pc & 63;
    *(f32x4_t*)(dst + (int64_t)k * a.ldw + pc) = *(const f32x4_t*)(red + (pr * 64 + k) * 64 + c);
  }
}

// ------------------------------------------------------------------------------------------------
// The fused stem weight gradient on RAW IMAGE ROWS (round 5).  PMC on the window-staged kernels above: the vector
// data-return path (TD) is ~80 % busy, and 60 % of what it returns is the window image: every pixel's 4 x 128 B
// of kernel-row-pair windows are DMA'd separately although neighbouring windows overlap 3/4 (stride 2, 8 pixels
// wide).  Here a K-step is a 4-row x 16-column block of conv-output pixels and stages just the padded image rows
// it touches -- 14 rows x 38 pixels x 4 channels, 4.2 KB instead of 32 KB -- and the MFMA A fragments are read
// straight out of them: the transposed LDS read only needs each lane's 8-byte address of 4 consecutive elements of
// its pixel's window row, and window column j of pixel (dh, wl) for kernel-row pair t is element 8 wl + (j & 31) of
// staged row 2 dh + 2 t + (j >> 5).  dY is computed per 2x2 quad as in wgrad_stem_quad_kernel (same arithmetic,
// same summation order) into the [pixel][64] tile.  Needs Pm % 4 == 0 and Qm % 16 == 0 (the ResNet stem at
// 224 px: 112 x 112); other shapes take the pixel-pair kernel.  12 operand loads + 2 DMA instructions per thread /
// wave per step; pixel p of a step = 16 dh + wl.
template <int DT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3, 3))) void wgrad_stem_rows_kernel(ConvWgradArgs a) {
  using E = E16<DT>;
  typedef typename E::vec8 vec8;
  constexpr int BKP = 64;             // pixels per K-step: 4 conv rows x 16 conv columns
  constexpr int ROWB = 128;           // dY tile: 64 channels * 2 B
  constexpr int TB = BKP * ROWB;      // 8 KB
  constexpr int XROWB = 38 * 4 * 2;   // one staged image row: 2 * 15 + 8 pixels x 4 channels (304 B)
  constexpr int XCH = XROWB / 16;     // 19 16-byte DMA chunks per row
  constexpr int XROWS = 14;           // image rows of a step: 2 * 3 + 2 * 3 + 1 + 1
  constexpr int XB = 512 * 16;        // 2 DMA instructions per wave x 4 waves x 64 lanes x 16 B (266 chunks live)
  constexpr int STAGE = TB + XB;      // 16 KB
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // = kernel-row pair
  const int split = blockIdx.x;
  const int steps_total = a.P / BKP;
  const int s_begin = split * (a.pix_per_split / BKP);
  const int s_end = min(steps_total, s_begin + a.pix_per_split / BKP);
  const int nsteps = max(0, s_end - s_begin);
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(a.x, (uint32_t)a.N * a.H * a.W * a.cs * 2u);
  const int SW = a.Qm / 16, SPI = (a.Pm / 4) * SW;  // steps per 4-row band, per image
  const FastDiv dspi{a.div_pq_mul, a.div_pq_shift}, dsw{a.div_q_mul, a.div_q_shift};
  const uint32_t img_row_b = (uint32_t)a.W * a.cs * 2u;

  // step -> (image, first conv row h0, first conv column w0), wave-uniform
  auto step_geom = [&](int st, int& n, int& h0, int& w0) {
    n = (int)fdiv((uint32_t)st, dspi);
    const int rem = st - n * SPI;
    const int hb = (int)fdiv((uint32_t)rem, dsw);
    h0 = 4 * hb;
    w0 = 16 * (rem - hb * SW);
  };
  // X DMA: lane slot L = j * 256 + wave * 64 + lane of the stage's 512 16-byte slots; slot L holds chunk L % 19 of
  // staged row L / 19 (slots past 14 rows read zeros)
  uint32_t xlane[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int L = j * 256 + wave * 64 + lane, k = L / XCH, c = L - k * XCH;
    xlane[j] = k < XROWS ? (uint32_t)k * img_row_b + (uint32_t)c * 16u : kOOB;
  }
  auto stage_load_x = [&](int st, int buf) {
    int n, h0, w0;
    step_geom(st, n, h0, w0);
    const uint32_t base = (((uint32_t)n * a.H + 2u * h0) * a.W + 2u * w0) * a.cs * 2u;
    char* sx = smem + buf * STAGE + TB;
#pragma unroll
    for (int j = 0; j < 2; ++j)
      buf_lds16_asm(rx, sx + (j * 256 + wave * 64) * 16, xlane[j] == kOOB ? kOOB : base + xlane[j]);
  };

  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p4 = li & 3;
  // A-fragment addresses (per kk, r0 | r1, column half): row 2 dh + 2 wave + half, element 8 wl + 4 p4 (+ 16 for
  // the odd fragment of a half)
  int xa[2][2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int p = kk * 32 + 8 * g + q + 4 * h, dh = p >> 4, wl = p & 15;
      xa[kk][h] = (2 * dh + 2 * wave) * XROWB + wl * 16 + p4 * 8;
    }

  // ---- dY: quad (qr, qc) = (qd >> 3, qd & 7) of the step, channels 4*cg .. 4*cg + 3
  const int qd = tid >> 4, cg = tid & 15, qr = qd >> 3, qc = qd & 7;
  // (the ReLU mask is in the argmax: bn_relu_maxpool marks windows whose maximum is 0 dead, so f_coef is not read)
  float fA[4], fB[4], fC[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int c = cg * 4 + e;
    fA[e] = a.f_bcoef[c]; fB[e] = a.f_bcoef[64 + c]; fC[e] = a.f_bcoef[128 + c];
  }
  u32x2v fy[4], fg[4];  // asm loads: waited for by ROWS_WAIT
  uint32_t fi[4];
  int fvalid = 0;       // bit 2: window row r+1 exists, bit 3: window column s+1 exists
  auto dy_load = [&](int st) {
    int n, h0, w0;
    step_geom(st, n, h0, w0);
    const int r = (h0 >> 1) + qr, sc = (w0 >> 1) + qc;
    const bool okr = r + 1 < a.f_OH, oks = sc + 1 < a.f_OW;
    const uint32_t pix = ((uint32_t)(n * a.Pm + 2 * r) * a.Qm + 2 * sc) * 64u + cg * 4;
    fy[0] = gload8_asm(a.f_y + pix);
    fy[1] = gload8_asm(a.f_y + pix + 64u);
    fy[2] = gload8_asm(a.f_y + pix + (uint32_t)a.Qm * 64u);
    fy[3] = gload8_asm(a.f_y + pix + (uint32_t)a.Qm * 64u + 64u);
    const uint32_t w00 = (((uint32_t)n * a.f_OH + r) * a.f_OW + sc) * 64u + cg * 4;
    const uint32_t dr = okr ? (uint32_t)a.f_OW * 64u : 0u, dc = oks ? 64u : 0u;
    fi[0] = gload4_asm(a.f_idx + w00);
    fg[0] = gload8_asm(a.f_dp + w00);
    fi[1] = gload4_asm(a.f_idx + w00 + dc);
    fg[1] = gload8_asm(a.f_dp + w00 + dc);
    fi[2] = gload4_asm(a.f_idx + w00 + dr);
    fg[2] = gload8_asm(a.f_dp + w00 + dr);
    fi[3] = gload4_asm(a.f_idx + w00 + dr + dc);
    fg[3] = gload8_asm(a.f_dp + w00 + dr + dc);
    fvalid = (okr ? 4 : 0) | (oks ? 8 : 0);
  };
  auto dy_store = [&](int buf) {
    char* sy = smem + buf * STAGE;
    const uint32_t i0 = fi[0], i1 = fvalid & 8 ? fi[1] : 0xffffffffu, i2 = fvalid & 4 ? fi[2] : 0xffffffffu;
    const uint32_t i3 = (fvalid & 12) == 12 ? fi[3] : 0xffffffffu;
    uint32_t ov[4][2];
    float dv[4][4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int sh = 16 * (e & 1);
      const uint32_t p0 = (i0 >> (8 * e)) & 0xffu, p1 = (i1 >> (8 * e)) & 0xffu;
      const uint32_t p2 = (i2 >> (8 * e)) & 0xffu, p3 = (i3 >> (8 * e)) & 0xffu;
      const float g0 = E::to_f((uint16_t)(fg[0][e >> 1] >> sh)), g1 = E::to_f((uint16_t)(fg[1][e >> 1] >> sh));
      const float g2 = E::to_f((uint16_t)(fg[2][e >> 1] >> sh)), g3 = E::to_f((uint16_t)(fg[3][e >> 1] >> sh));
      // branch-free (as conditional adds the compiler built a divergent switch on p0): selects of g or 0, summed
      // in window order (an unselected term adds an exact zero)
      float dz[4];
      dz[0] = p0 == 4 ? g0 : 0.f;
      dz[1] = (p0 == 5 ? g0 : 0.f) + (p1 == 3 ? g1 : 0.f);
      dz[2] = (p0 == 7 ? g0 : 0.f) + (p2 == 1 ? g2 : 0.f);
      dz[3] = (((p0 == 8 ? g0 : 0.f) + (p1 == 6 ? g1 : 0.f)) + (p2 == 2 ? g2 : 0.f)) + (p3 == 0 ? g3 : 0.f);
#pragma unroll
      for (int sub = 0; sub < 4; ++sub) {
        const float yv = E::to_f((uint16_t)(fy[sub][e >> 1] >> sh));
        dv[sub][e] = __builtin_fmaf(fA[e], dz[sub], __builtin_fmaf(fB[e], yv, fC[e]));
      }
    }
#pragma unroll
    for (int sub = 0; sub < 4; ++sub) {
      ov[sub][0] = E::pack2(dv[sub][0], dv[sub][1]);
      ov[sub][1] = E::pack2(dv[sub][2], dv[sub][3]);
    }
#pragma unroll
    for (int sub = 0; sub < 4; ++sub) {
      const int row = (2 * qr + (sub >> 1)) * 16 + 2 * qc + (sub & 1);
      *(uint2*)(sy + row * ROWB + (((cg >> 1) ^ tr_swz(row)) << 4) + (cg & 1) * 8) = make_uint2(ov[sub][0], ov[sub][1]);
    }
  };
  // per step the queue is [loads(st+1): 12][DMA(st+1): 2] at the dY store (vmcnt(2): the DMA stays in flight
  // under the dY math), then [DMA(st+1): 2][loads(st+2): 12] before the barrier (vmcnt(12))
#define ROWS_WAIT(n)                                                                                     \
  asm volatile("s_waitcnt vmcnt(" #n ")"                                                                 \
               : "+v"(fy[0]), "+v"(fy[1]), "+v"(fy[2]), "+v"(fy[3]), "+v"(fi[0]), "+v"(fi[1]), "+v"(fi[2]), \
                 "+v"(fi[3]), "+v"(fg[0]), "+v"(fg[1]), "+v"(fg[2]), "+v"(fg[3])                         \
               :                                                                                         \
               : "memory")
  if (nsteps > 0) {
    dy_load(s_begin);
    stage_load_x(s_begin, 0);
    ROWS_WAIT(0);
    dy_store(0);
    if (nsteps > 1) dy_load(s_begin + 1);
    __syncthreads();
    for (int st = 0; st < nsteps; ++st) {
      const int cur = st & 1;
      if (st + 1 < nsteps) stage_load_x(s_begin + st + 1, cur ^ 1);
      const char* sy = smem + cur * STAGE;
      const char* sx = sy + TB;
#pragma unroll
      for (int kk = 0; kk < BKP / 32; ++kk) {
        const int r0 = kk * 32 + 8 * g + q, r1 = r0 + 4;
        const int sw0 = tr_swz(r0), sw1 = tr_swz(r1);
        vec8 af[4], bfr[4];
#pragma unroll
        for (int f = 0; f < 4; ++f) {
          const int xo = (f >> 1) * XROWB + (f & 1) * 32;  // column half -> next staged row; odd fragment +16 el
          s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(sx + xa[kk][0] + xo));
          s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(sx + xa[kk][1] + xo));
          af[f] = __builtin_bit_cast(vec8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
          const int col = f * 16 + 4 * p4;
          const int ch = col >> 3, off = (col & 7) * 2;
          lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(sy + r0 * ROWB + ((ch ^ sw0) << 4) + off));
          hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(sy + r1 * ROWB + ((ch ^ sw1) << 4) + off));
          bfr[f] = __builtin_bit_cast(vec8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = E::mfma16x16x32(af[i], bfr[j], acc[i][j]);
      }
      __builtin_amdgcn_sched_barrier(0);  // the waits and the dY math stay behind the last MFMA
      if (st + 1 < nsteps) {
        ROWS_WAIT(2);
        __builtin_amdgcn_sched_barrier(0);
        dy_store(cur ^ 1);
        if (st + 2 < nsteps) {
          dy_load(s_begin + st + 2);
          asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
        } else {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __syncthreads();
    }
  }
#undef ROWS_WAIT
  // acc[i][j]: rows (window column) c = 16i + 4*(lane>>4) + r, col k = 16j + (lane&15); transposed through the
  // 32 KB of LDS two pairs at a time ([2 pairs][64 k][64 c] fp32), written as ws[split][k][pair*64 + c] rows
  float* red = (float*)smem;
  float* dst = a.ws + (int64_t)split * a.Kout * a.ldw;
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    __syncthreads();
    if ((wave >> 1) == half) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int k = 16 * j + (lane & 15);
          const int c = 16 * i + 4 * (lane >> 4);
          *(f32x4_t*)(red + ((wave & 1) * 64 + k) * 64 + c) = acc[i][j];
        }
    }
    __syncthreads();
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int idx = (e * 256 + tid) * 4;  // 0..8191 over [k][pair of the half][c]
      const int k = idx >> 7, pc = idx & 127, pr = pc >> 6, c = pc & 63;
      *(f32x4_t*)(dst + (int64_t)k * a.ldw + half * 128 + pc) = *(const f32x4_t*)(red + (pr * 64 + k) * 64 + c);
    }
  }
}

// ------------------------------------------------------------------------------------------------
// 128 (c) x 128 (k) tile variant for layers with C, Kout multiples of 128: 4 waves in a 2x2 grid over
// the output tile, each wave owning 64x64 for ALL 64 pixels of a K-step (32 MFMAs per K-step per wave,
// 4x the MFMA work per loaded pixel row of the 64x64 variant).  64 KiB of LDS -> 2 blocks per CU.
//
// PAIR (C == 64, Kout % 128 == 0: ResNet layer2's first 3x3/2 conv and its 1x1/2 downsample): the 128-wide
// c side of the tile is TWO TAPS of 64 channels -- X row chunk ch < 8 is gathered through tap 2*nt, chunk
// ch >= 8 through tap 2*nt + 1 -- so the 64-channel layers run at the 128x128 tile's MFMA work per staged
// byte instead of the 64x64 kernel's.  With C == 64 the two taps' columns tap*64 + c are contiguous in
// dW, so the epilogue is unchanged; an odd tap count leaves the last tile's second half dead (zero-filled
// DMA, its two waves skip the MFMAs and the store).
PDT_DEVICE int tr_swz16(int row) { return ((row & 3) << 1) | (((row >> 3) & 1) << 3); }

int wgrad_ctiles(const ConvWgradArgs& a) {
  if (a.tile == kWgradWide) return (a.T * a.U * (a.C / 128) + 1) / 2;
  if (a.tile == 128 && a.C == 64) return (a.T * a.U + 1) / 2;
  return a.T * a.U * (a.C / a.tile);
}

int wgrad_ktile(const ConvWgradArgs& a) { return a.tile == kWgradWide ? 128 : a.tile; }

// PRE (PAIR, 1x1 / stride 1 / no padding only): x is the RAW output of the producer conv and its BatchNorm + ReLU
// (a.pre_coef) is applied to each x fragment after the LDS read, bit-identical to bn_apply.  A fragment's 8
// values are 8 pixels of ONE channel (MFMA A row = lane & 15), so a lane needs one scale / shift per fragment.
// Rows past the split end are zero-filled and transform to relu(shift), but their dY rows are zero too.
template <int DT, bool PAIR, bool PRE = false>
__global__ __launch_bounds__(256) void conv_wgrad128_kernel(ConvWgradArgs a) {
  using E = E16<DT>;
  typedef typename E::vec8 vec8;
  constexpr int BKP = 64;          // pixels per K-step
  constexpr int ROWB = 256;        // 128 channels * 2 B
  constexpr int XB = BKP * ROWB;   // 16 KiB
  constexpr int STAGE = 2 * XB;
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wave & 1, wk = wave >> 1;

  const int taps = a.T * a.U;
  const int c_tiles = PAIR ? 1 : a.C / 128;
  const int n_tiles = PAIR ? (taps + 1) / 2 : taps * c_tiles;
  const int k_tiles = a.Kout / 128;
  const int nwg = k_tiles * n_tiles * a.splits;
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int tile = bid % (k_tiles * n_tiles);
  const int split = bid / (k_tiles * n_tiles);
  const int kt = tile % k_tiles;
  const int nt = tile / k_tiles;
  const int tap = PAIR ? 2 * nt : nt / c_tiles;  // PAIR: the first of the two taps
  const int c0 = PAIR ? 0 : (nt - tap * c_tiles) * 128;
  const int k0 = kt * 128;

  const int pix_begin = split * a.pix_per_split;
  const int pix_end = min(a.P, pix_begin + a.pix_per_split);
  const int nsteps = (pix_end - pix_begin + BKP - 1) / BKP;

  // tap offsets of the two column halves (equal unless PAIR)
  int th2[2], tw2[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int tp = PAIR ? min(tap + h, taps - 1) : tap;
    const int t = tp / a.U, u = tp - (tp / a.U) * a.U;
    th2[h] = t * a.dil_h - a.pad_h;
    tw2[h] = u * a.dil_w - a.pad_w;
  }
  const bool half1_live = !PAIR || tap + 1 < taps;
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(a.x, (uint32_t)a.N * a.H * a.W * a.cs * 2u);
  const __amdgpu_buffer_rsrc_t ry = make_rsrc(a.dy, (uint32_t)a.P * a.Kout * 2u);

  // ---- DMA (incremental source offsets, as the wide kernel): this wave stages pixel rows 16 wave + 4 j + lrow (j < 4)
  // of the K-step, lane chunk lch_j = pch ^ tr_swz16(row) (PAIR: column half h_j = lch_j >> 3 -> tap)
  const int lrow = lane >> 4, pch = lane & 15;
  const int sh = a.stride_h, sw = a.stride_w, Qm = a.Qm, Pm = a.Pm, W = a.W, H = a.H, cs = a.cs;
  const int adv_i = BKP / Qm, adv_j = BKP - adv_i * Qm;
  const int toff0 = (th2[0] * W + tw2[0]) * cs, toff1 = (th2[1] * W + tw2[1]) * cs;
  int xi, xj, ih, iw, xo;  // grid position of pixel p0 = pix_begin + step * BKP + 16 wave + lrow, tap-less input
  {
    const FastDiv dpq{a.div_pq_mul, a.div_pq_shift}, dq{a.div_q_mul, a.div_q_shift};
    const int p0 = pix_begin + 16 * wave + lrow;
    const int n = (int)fdiv((uint32_t)p0, dpq);
    const int rem = p0 - n * Pm * Qm;
    xi = (int)fdiv((uint32_t)rem, dq);
    xj = rem - xi * Qm;
    ih = xi * sh;
    iw = xj * sw;
    xo = ((n * H + ih) * W + iw) * cs;
  }
  const int row_step = (sh * W - Qm * sw) * cs, img_step = (H - Pm * sh) * W * cs;
  int ycur = ((pix_begin + 16 * wave + lrow) * a.Kout + k0) * 2;
  // +4 pixels with at most one row wrap (Qm >= 4, the launcher's condition) and one image wrap, branch-free
  auto step4 = [&](int& i, int& jq, int& hh, int& ww, int& o) {
    jq += 4; ww += 4 * sw; o += 4 * sw * cs;
    const bool wr = jq >= Qm;
    jq -= wr ? Qm : 0; ww -= wr ? Qm * sw : 0; hh += wr ? sh : 0; o += wr ? row_step : 0; i += wr ? 1 : 0;
    const bool wi = i >= Pm;
    i -= wi ? Pm : 0; hh -= wi ? Pm * sh : 0; o += wi ? img_step : 0;
  };
  auto stage_load = [&](int buf) {  // the next K-step in sequence (advances the lane state)
    char* sb = smem + buf * STAGE;
    int i = xi, jq = xj, hh = ih, ww = iw, o = xo;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (j > 0) step4(i, jq, hh, ww, o);
      const int lch = pch ^ ((lrow << 1) | (((j >> 1) & 1) << 3));
      const int h = PAIR ? lch >> 3 : 0;
      const int th = h ? th2[1] : th2[0], tw = h ? tw2[1] : tw2[0];
      // (bitwise &: a short-circuit && compiles to divergent branches around each DMA's offset)
      const bool ok = ((unsigned)(hh + th) < (unsigned)H) & ((unsigned)(ww + tw) < (unsigned)W) &
                      (!PAIR || !h || half1_live);
      const int col = (PAIR ? -h * 64 : c0) + lch * 8;
      const uint32_t xoff = ok ? (uint32_t)((o + (h ? toff1 : toff0) + col) * 2) : kOOB;
      buf_lds16_asm(rx, sb + (wave * 4 + j) * 1024, xoff);
      buf_lds16_asm(ry, sb + XB + (wave * 4 + j) * 1024, (uint32_t)(ycur + (j * 4 * a.Kout + lch * 8) * 2));
    }
    ycur += BKP * a.Kout * 2;
    xj += adv_j; iw += adv_j * sw; xo += adv_j * sw * cs;
    xi += adv_i; ih += adv_i * sh; xo += adv_i * sh * W * cs;
    if (xj >= Qm) { xj -= Qm; iw -= Qm * sw; ih += sh; xo += row_step; ++xi; }
    while (xi >= Pm) { xi -= Pm; ih -= Pm * sh; xo += img_step; }
  };

  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int g = lane >> 4, li = lane & 15, q = li >> 2, p4 = li & 3;
  // fragment byte addresses (stage 0, kk 0; tr_swz16 of rows kk * 32 + 8 g + q (+4) does not depend on kk): a stage /
  // kk shift is an immediate
  int xa[4][2], ya[4][2];
#pragma unroll
  for (int f = 0; f < 4; ++f) {
    const int cc = wc * 64 + f * 16 + 4 * p4, kc = wk * 64 + f * 16 + 4 * p4;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int rr = 8 * g + q + 4 * r, sz = tr_swz16(rr);
      xa[f][r] = rr * ROWB + (((cc >> 3) ^ sz) << 4) + (cc & 7) * 2;
      ya[f][r] = XB + rr * ROWB + (((kc >> 3) ^ sz) << 4) + (kc & 7) * 2;
    }
  }

  float psc[4], psh[4];
  if constexpr (PRE) {
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      const int ch = (wc * 64 + f * 16 + (lane & 15)) & 63;
      psc[f] = a.pre_coef[ch];
      psh[f] = a.pre_coef[64 + ch];
    }
  }

  auto kstep = [&](auto stc, int s) {
    constexpr int ST = decltype(stc)::value;  // ring buffer of K-step s (s & 1)
    if (s + 1 < nsteps) stage_load(ST ^ 1);
#pragma unroll
    for (int kk = 0; kk < BKP / 32; ++kk) {
      const int so = ST * STAGE + kk * 32 * ROWB;
      vec8 af[4], bfr[4];
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(smem + xa[f][0] + so));
        s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(smem + xa[f][1] + so));
        af[f] = __builtin_bit_cast(vec8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
        if constexpr (PRE) {
          float sc8[8], sh8[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) { sc8[e] = psc[f]; sh8[e] = psh[f]; }
          af[f] = __builtin_bit_cast(vec8, pre_act8<DT>(__builtin_bit_cast(uint4, af[f]), sc8, sh8));
        }
        lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(smem + ya[f][0] + so));
        hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(smem + ya[f][1] + so));
        bfr[f] = __builtin_bit_cast(vec8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
      if (wc == 0 || half1_live) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = E::mfma16x16x32(af[i], bfr[j], acc[i][j]);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  };

  if (nsteps > 0) {
    stage_load(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // unrolled over the 2 ring buffers: every buffer offset is a compile-time immediate
    for (int s = 0; s < nsteps; s += 2) {
      kstep(std::integral_constant<int, 0>{}, s);
      if (s + 1 < nsteps) kstep(std::integral_constant<int, 1>{}, s + 1);
    }
  }
  if (wc == 1 && !half1_live) return;
  // acc[i][j]: rows c = wc*64 + 16i + 4*(lane>>4) + r, col k = wk*64 + 16j + (lane&15)
  float* dst = a.ws + ((int64_t)split * a.Kout + k0) * a.ldw + tap * a.C + c0;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = wk * 64 + 16 * j + (lane & 15);
      const int c = wc * 64 + 16 * i + 4 * (lane >> 4);
      *(f32x4_t*)(dst + (int64_t)k * a.ldw + c) = acc[i][j];
    }
}

// s_waitcnt vmcnt(N) only (expcnt / lgkmcnt left at their maxima)
template <int N>
PDT_DEVICE void wg_vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}

// ------------------------------------------------------------------------------------------------
// "Wide" 256 (c) x 128 (k) tile for C % 128 == 0, Kout % 128 == 0 layers below the ping-pong kernel's 256 x 256
// (ResNet-18 layer2's 3x3 128->128 convs, layer3.0's 128->256 ones; ResNet-50 stage 2).  The dW column axis
// (tap * C + c) is cut into 128-wide column blocks -- one tap's channel range each, contiguous in dW -- and a tile
// is TWO consecutive column blocks (two taps when C == 128; an odd count leaves the last tile's second half dead).
// 8 waves as 4 (c) x 2 (k), each owning 64 x 64 over all 64 pixels of a K-step: 85 FLOP per staged byte against
// the 128 x 128 tile's 64.  One workgroup per CU with a 3-deep ring of 48 KB stages: the DMA of K-step s+2 is
// issued while K-step s computes, and each K-step waits only for its own stage (counted vmcnt(kWideDma): the 6
// DMA instructions per wave of the stage behind it stay in flight) -- the 128 x 128 kernel drains its single
// prefetch (vmcnt(0)) every K-step and is latency-bound at ~30 % MFMA busy.
// (A BKP = 32 form with 24 KB stages and two workgroups per CU measured slower and was removed in round 5.)
// DMA instructions per wave per stage: X 2 sub-tiles x BKP/4 rows-of-4 over 8 waves, dY BKP/4 over 8 waves.
template <int BKP>
constexpr int wide_dma() { return 2 * (BKP / 4) / 8 + (BKP / 4) / 8; }

template <int DT, int BKP>
__global__ __launch_bounds__(512) void conv_wgrad_wide_kernel(ConvWgradArgs a) {
  using E = E16<DT>;
  typedef typename E::vec8 vec8;
  constexpr int kWideDma = wide_dma<BKP>();
  static_assert(BKP == 64 && kWideDma == 6, "the DMA row mapping below is written for 64-pixel K-steps");
  constexpr int ROWB = 256;        // 128 channels * 2 B
  constexpr int SUB = BKP * ROWB;  // one column block's X image, or the dY image
  constexpr int STAGE = 3 * SUB;   // X block 0 | X block 1 | dY
  constexpr int NST = 3;
  __shared__ __attribute__((aligned(1024))) char smem[NST * STAGE];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wave & 3, wk = wave >> 2;

  const int taps = a.T * a.U;
  const int cblocks = taps * (a.C / 128);  // 128-wide column blocks of dW
  const int n_tiles = (cblocks + 1) / 2;
  const int k_tiles = a.Kout / 128;
  const int nwg = k_tiles * n_tiles * a.splits;
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int tile = bid % (k_tiles * n_tiles);
  const int split = bid / (k_tiles * n_tiles);
  const int kt = tile % k_tiles;
  const int nt = tile / k_tiles;
  const int k0 = kt * 128;

  const int pix_begin = split * a.pix_per_split;
  const int pix_end = min(a.P, pix_begin + a.pix_per_split);
  const int nsteps = (pix_end - pix_begin + BKP - 1) / BKP;

  // the two column blocks: tap offsets and channel base
  int th2[2], tw2[2], cb0[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int cb = min(2 * nt + h, cblocks - 1);
    const int tp = cb * 128 / a.C;
    const int t = tp / a.U, u = tp - (tp / a.U) * a.U;
    th2[h] = t * a.dil_h - a.pad_h;
    tw2[h] = u * a.dil_w - a.pad_w;
    cb0[h] = cb * 128 - tp * a.C;
  }
  const bool half1_live = 2 * nt + 1 < cblocks;
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(a.x, (uint32_t)a.N * a.H * a.W * a.cs * 2u);
  const __amdgpu_buffer_rsrc_t ry = make_rsrc(a.dy, (uint32_t)a.P * a.Kout * 2u);

  // ---- DMA: every source offset is updated incrementally (adds and compares, no per-pixel division or multiply:
  // the round-5 form spent ~90 quarter-rate VALU per K-step and wave on them, more issue time than its MFMAs).
  // X: this wave stages column block hx = wave / 4, pixel rows 16 (wave & 3) + 4 j + lrow (j < 4) of the K-step;
  // dY: rows 8 wave + 4 j + lrow (j < 2).  LDS: X block h of ring stage st at (3 h + st) SUB, dY at (6 + st) SUB, so
  // every fragment read below is a lane register plus an immediate below 64 KB.
  const int lrow = lane >> 4, pch = lane & 15;
  const int hx = wave >> 2;
  const int sh = a.stride_h, sw = a.stride_w, Qm = a.Qm, Pm = a.Pm, W = a.W, H = a.H, cs = a.cs;
  const int adv_i = BKP / Qm, adv_j = BKP - adv_i * Qm;  // one K-step = adv_i rows + adv_j columns of the grid
  // lane state of pixel p0 = pix_begin + step * BKP + 16 (wave & 3) + lrow: grid row xi, column xj, input row /
  // column xh / xw (tap offset included) and element offset xo of the input pixel (column excluded)
  int xi, xj, xh, xw, xo;
  {
    const FastDiv dpq{a.div_pq_mul, a.div_pq_shift}, dq{a.div_q_mul, a.div_q_shift};
    const int p0 = pix_begin + 16 * (wave & 3) + lrow;
    const int n = (int)fdiv((uint32_t)p0, dpq);
    const int rem = p0 - n * Pm * Qm;
    xi = (int)fdiv((uint32_t)rem, dq);
    xj = rem - xi * Qm;
    xh = xi * sh + th2[hx];
    xw = xj * sw + tw2[hx];
    xo = ((n * H + xh) * W + xw) * cs;
  }
  const int row_step = (sh * W - Qm * sw) * cs, img_step = (H - Pm * sh) * W * cs;
  // one grid-column step of d pixels with at most one row wrap (d < Qm) and one image wrap, branch-free
  auto step_px = [&](int& i, int& j, int& h, int& w, int& o, int d) {
    j += d; w += d * sw; o += d * sw * cs;
    const bool wr = j >= Qm;
    j -= wr ? Qm : 0; w -= wr ? Qm * sw : 0; h += wr ? sh : 0; o += wr ? row_step : 0; i += wr ? 1 : 0;
    const bool wi = i >= Pm;
    i -= wi ? Pm : 0; h -= wi ? Pm * sh : 0; o += wi ? img_step : 0;
  };
  int ycur;  // dY byte offset of this lane's j = 0 row for the next K-step to stage
  const int ystr = a.ldy ? a.ldy : a.Kout;
  const int lchy = pch ^ ((lrow << 1) | ((wave & 1) << 3));
  ycur = ((pix_begin + 8 * wave + lrow) * ystr + k0 + lchy * 8) * 2;
  const bool x_live = hx == 0 || half1_live;
  const int xcolb = cb0[hx];

  auto stage_load = [&](int buf) {  // the next K-step in sequence (advances the lane state)
    int i = xi, j = xj, h = xh, w = xw, o = xo;
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      if (jj > 0) step_px(i, j, h, w, o, 4);
      const int lch = pch ^ ((lrow << 1) | (((jj >> 1) & 1) << 3));
      const bool ok = x_live & ((unsigned)h < (unsigned)H) & ((unsigned)w < (unsigned)W);  // (no short-circuit branch)
      const uint32_t off = ok ? (uint32_t)((o + xcolb + lch * 8) * 2) : kOOB;
      buf_lds16_asm(rx, smem + (3 * hx + buf) * SUB + (4 * (wave & 3) + jj) * 1024, off);
    }
#pragma unroll
    for (int jj = 0; jj < 2; ++jj)
      buf_lds16_asm(ry, smem + (6 + buf) * SUB + (2 * wave + jj) * 1024, (uint32_t)(ycur + jj * 4 * ystr * 2));
    // advance to the next K-step
    ycur += BKP * ystr * 2;
    xj += adv_j; xw += adv_j * sw; xo += adv_j * sw * cs;
    xi += adv_i; xh += adv_i * sh; xo += adv_i * sh * W * cs;
    if (xj >= Qm) { xj -= Qm; xw -= Qm * sw; xh += sh; xo += row_step; ++xi; }
    while (xi >= Pm) { xi -= Pm; xh -= Pm * sh; xo += img_step; }
  };

  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int g = lane >> 4, li = lane & 15, q = li >> 2, p4 = li & 3;
  const int xsub = wc >> 1;  // this wave's X sub-tile (column block)
  const bool live = xsub == 0 || half1_live;
  // fragment byte addresses (stage 0, kk 0): the transposed-read swizzle tr_swz16 of rows kk * 32 + 8 g + q (+4)
  // does not depend on kk, so a stage / kk shift is an immediate
  int xa[4][2], ya[4][2];
#pragma unroll
  for (int f = 0; f < 4; ++f) {
    const int cc = (wc & 1) * 64 + f * 16 + 4 * p4, kc = wk * 64 + f * 16 + 4 * p4;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int rr = 8 * g + q + 4 * r, sz = tr_swz16(rr);
      xa[f][r] = 3 * xsub * SUB + rr * ROWB + (((cc >> 3) ^ sz) << 4) + (cc & 7) * 2;
      ya[f][r] = 6 * SUB + rr * ROWB + (((kc >> 3) ^ sz) << 4) + (kc & 7) * 2;
    }
  }

  auto kstep = [&](auto stc, int s) {
    constexpr int ST = decltype(stc)::value;  // ring stage of K-step s (s % 3)
    // stage s landed: the younger stage s+1 (kWideDma per wave) may stay in flight
    if (s + 1 < nsteps)
      wg_vm_wait<kWideDma>();
    else
      wg_vm_wait<0>();
    // every wave's DMA of stage s landed; every wave's MFMAs (hence its fragment reads) of stage s-1 done, so
    // the ring slot of stage s-1 may be refilled.  A plain s_barrier: __syncthreads' release fence would also
    // drain the stage still in flight (vmcnt(0)).
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (s + 2 < nsteps) stage_load((ST + 2) % NST);
    if (live) {
#pragma unroll
      for (int kk = 0; kk < BKP / 32; ++kk) {
        const int so = ST * SUB + kk * 32 * ROWB;
        vec8 af[4], bfr[4];
#pragma unroll
        for (int f = 0; f < 4; ++f) {
          s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(smem + xa[f][0] + so));
          s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(smem + xa[f][1] + so));
          af[f] = __builtin_bit_cast(vec8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
          lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(smem + ya[f][0] + so));
          hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(smem + ya[f][1] + so));
          bfr[f] = __builtin_bit_cast(vec8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
        }
        // raised priority while this wave's 16 MFMAs issue: the SIMD's other wave then slots its fragment reads
        // in between instead of both waves reading at once
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = E::mfma16x16x32(af[i], bfr[j], acc[i][j]);
        __builtin_amdgcn_s_setprio(0);
      }
    }
  };

  if (nsteps > 0) {
    stage_load(0);
    if (nsteps > 1) stage_load(1);
    // unrolled over the 3 ring stages: every stage offset is a compile-time immediate
    for (int s = 0; s < nsteps; s += NST) {
      kstep(std::integral_constant<int, 0>{}, s);
      if (s + 1 < nsteps) kstep(std::integral_constant<int, 1>{}, s + 1);
      if (s + 2 < nsteps) kstep(std::integral_constant<int, 2>{}, s + 2);
    }
  }
  if (!live) return;
  // acc[i][j]: rows c = (wc & 1)*64 + 16i + 4*(lane>>4) + r of column block 2nt + xsub, col k = wk*64 + 16j + (lane&15)
  float* dst = a.ws + ((int64_t)split * a.Kout + k0) * a.ldw + (2 * nt + xsub) * 128;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = wk * 64 + 16 * j + (lane & 15);
      const int c = (wc & 1) * 64 + 16 * i + 4 * (lane >> 4);
      *(f32x4_t*)(dst + (int64_t)k * a.ldw + c) = acc[i][j];
    }
}

// ------------------------------------------------------------------------------------------------
// 256 (c) x 256 (k) ping-pong weight-gradient kernel for layers with C, Kout multiples of 256 (ResNet
// layer3/4, ResNet-50 stages 2-4): the schedule of conv_pp_kernel (conv_fwd.hip) on the wgrad GEMM.
// 8 waves as 2 (c) x 4 (k), each owning 128 c x 64 k (128 fp32 accumulators), one workgroup per CU,
// 64-pixel K-steps in 4 phases of 16 MFMAs; waves 4-7 run one barrier behind waves 0-3 so that on
// every SIMD one wave computes while its partner reads fragments / issues DMA.
// The X and dY images of a K-step are split in halves by channel (X half h: c = g*128 + h*64 .. +64
// for g = 0, 1; dY half h: k = g*64 + h*32 .. +32 for g = 0..3), each [64 px][128 ch] (256-B rows,
// tr_swz16-swizzled for conflict-free ds_read_b64_tr_b16).  Phase p reads (X half, dY half):
//   p1: X0 + Y0, compute X0 x Y0;  p2: Y1, X0 x Y1;  p3: X1, X1 x Y1;  p4: -, X1 x Y0
// and issues the next K-step's X0, Y0, Y1, X1 DMA with the counted-vmcnt discipline of conv_pp_kernel.
// The DMA goes through buf_lds16_asm (common.h): with the builtin form the compiler drains the whole
// DMA pipeline (vmcnt(0)) before every transposed read.

template <int DT>
__global__ __launch_bounds__(512) void conv_wgrad_pp_kernel(ConvWgradArgs a) {
  using E = E16<DT>;
  typedef typename E::vec8 vec8;
  constexpr int BKP = 64, ROWB = 256;
  constexpr int HALF = BKP * ROWB;          // 16 KiB per half image
  constexpr int BUF = 4 * HALF;             // X0 X1 Y0 Y1
  constexpr int OX0 = 0, OX1 = HALF, OY0 = 2 * HALF, OY1 = 3 * HALF;
  __shared__ __attribute__((aligned(1024))) char smem[2 * BUF];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave >> 2;              // waves w and w+4 share a SIMD
  const int wx = wave & 1, wy = wave >> 1;  // 2 (c) x 4 (k)

  const int c_tiles = a.C / 256, k_tiles = a.Kout / 256;
  const int n_tiles = a.T * a.U * c_tiles;
  const int nwg = k_tiles * n_tiles * a.splits;
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int tile = bid % (k_tiles * n_tiles);
  const int split = bid / (k_tiles * n_tiles);
  const int kt = tile % k_tiles, nt = tile / k_tiles;
  const int tap = nt / c_tiles;
  const int c0 = (nt - tap * c_tiles) * 256, k0 = kt * 256;
  const int t = tap / a.U, u = tap - (tap / a.U) * a.U;
  const int pix_begin = split * a.pix_per_split;
  const int pix_end = min(a.P, pix_begin + a.pix_per_split);
  const int nsteps = (pix_end - pix_begin + BKP - 1) / BKP;
  const int th = t * a.dil_h - a.pad_h, tw = u * a.dil_w - a.pad_w;
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(a.x, (uint32_t)a.N * a.H * a.W * a.cs * 2u);
  const __amdgpu_buffer_rsrc_t ry = make_rsrc(a.dy, (uint32_t)a.P * (a.ldy ? a.ldy : a.Kout) * 2u);

  // DMA lane geometry: 4 pixel rows x 16 chunks per 1 KiB instruction, 2 instructions per wave per half
  const int lrow = lane >> 4, pch = lane & 15;
  int drow[2], lch[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    drow[j] = (wave * 2 + j) * 4 + lrow;
    lch[j] = pch ^ tr_swz16(drow[j]);
  }
  // image column (8-channel chunk) -> channel within the tile, half 0 (half 1 adds 64 / 32)
  int xcol[2], ycol[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = lch[j] * 8;
    xcol[j] = c0 + (col >> 6) * 128 + (col & 63);
    ycol[j] = k0 + (col >> 5) * 64 + (col & 31);
  }
  uint32_t xo[2], yo[2];
  auto offsets = [&](int step) {  // source offsets of this lane's two rows for K-step `step`
    const int pbase = pix_begin + step * BKP;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      uint32_t x_, y_;
      wgrad_rows<false>(a, pbase + drow[j], th, tw, xcol[j] - lch[j] * 8, lch[j], ycol[j] - lch[j] * 8, x_, y_);
      xo[j] = x_;
      yo[j] = y_;
    }
  };
  auto dma_x = [&](char* buf, int h) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
      buf_lds16_asm(rx, buf + (h ? OX1 : OX0) + (wave * 2 + j) * 1024, xo[j] == kOOB ? kOOB : xo[j] + h * 128u);
  };
  auto dma_y = [&](char* buf, int h) {
#pragma unroll
    for (int j = 0; j < 2; ++j) buf_lds16_asm(ry, buf + (h ? OY1 : OY0) + (wave * 2 + j) * 1024, yo[j] + h * 64u);
  };

  f32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // transposed-read lane geometry (see conv_wgrad128_kernel): rows r0 / r0+4 of each 32-pixel group
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p4 = li & 3;
  vec8 xs[4][2], y0r[2][2], y1r[2][2];
  auto frag = [&](const char* base, int cc, int kk) {
    const int r0 = kk * 32 + 8 * g + q, r1 = r0 + 4;
    s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_s16x4*)(base + r0 * ROWB + (((cc >> 3) ^ tr_swz16(r0)) << 4) + (cc & 7) * 2));
    s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_s16x4*)(base + r1 * ROWB + (((cc >> 3) ^ tr_swz16(r1)) << 4) + (cc & 7) * 2));
    return __builtin_bit_cast(vec8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
  };
  auto read_x = [&](const char* base) {
#pragma unroll
    for (int f = 0; f < 4; ++f)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) xs[f][kk] = frag(base, wx * 64 + f * 16 + 4 * p4, kk);
  };
  auto read_y = [&](vec8 (&yr)[2][2], const char* base) {
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) yr[f][kk] = frag(base, wy * 32 + f * 16 + 4 * p4, kk);
  };
  auto compute = [&](const vec8 (&yr)[2][2], int xh, int yh) {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int f2 = 0; f2 < 2; ++f2)
#pragma unroll
        for (int f = 0; f < 4; ++f)
          acc[xh * 4 + f][yh * 2 + f2] = E::mfma16x16x32(xs[f][kk], yr[f2][kk], acc[xh * 4 + f][yh * 2 + f2]);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  if (nsteps > 0) {
    offsets(0);
    dma_x(smem, 0);
    dma_y(smem, 0);
    dma_y(smem, 1);
    dma_x(smem, 1);
    wg_vm_wait<4>();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    if (grp == 1) __builtin_amdgcn_s_barrier();
    for (int ks = 0; ks < nsteps; ++ks) {
      const char* cb = smem + (ks & 1) * BUF;
      char* nb = smem + ((ks + 1) & 1) * BUF;
      const bool more = ks + 1 < nsteps;
      if (more) offsets(ks + 1);
      if (more) { dma_x(nb, 0); wg_vm_wait<4>(); } else { wg_vm_wait<2>(); }
      read_x(cb + OX0);
      read_y(y0r, cb + OY0);
      compute(y0r, 0, 0);
      if (more) { dma_y(nb, 0); wg_vm_wait<4>(); } else { wg_vm_wait<0>(); }
      read_y(y1r, cb + OY1);
      compute(y1r, 0, 1);
      if (more) dma_y(nb, 1);
      read_x(cb + OX1);
      compute(y1r, 1, 1);
      if (more) { dma_x(nb, 1); wg_vm_wait<4>(); }
      compute(y0r, 1, 0);
    }
    if (grp == 0) __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  }
  // acc[i][j]: c = wx*128 + 16i + 4*(lane>>4) + r (i = xh*4 + f), k = wy*64 + 16j + (lane&15)
  float* dst = a.ws + ((int64_t)split * a.Kout + k0) * a.ldw + tap * a.C + c0;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = wy * 64 + 16 * j + (lane & 15);
      const int c = wx * 128 + 16 * i + 4 * (lane >> 4);
      *(f32x4_t*)(dst + (int64_t)k * a.ldw + c) = acc[i][j];
    }
}

// ------------------------------------------------------------------------------------------------
// 3x3 / stride 1 / pad 1 weight gradient for C = Kout = 64 and W = 56 (ResNet layer1, the most
// expensive weight gradients of ResNet-18/34), all 9 taps in one block.
//
// The 64x64-tile kernel above re-reads dY and X once per tap (32 FLOP per staged byte: L2/DMA bound).
// Here a block tile is 4 output rows x 56 columns of one image: dY rows [4][56][64] and the X halo
// [6][58][64] (rows h0-1 .. h0+4, columns -1 .. 56, zero padding through the buffer range check) are
// staged ONCE per tile (72 KB, 2-deep LDS-DMA ring), and the 9 taps read shifted windows of the halo
// (~230 FLOP per staged byte).  Waves split the 64 x 64 output quadrant-wise (32 k x 32 c x 9 taps,
// 144 fp32 accumulators per lane).  A K-step = 32 pixels = column block j (8 px) of each of the 4
// output rows, so every 8-pixel MFMA k-group stays inside one row and tap shifts are plain row offsets.
// LDS rows are swizzled by (column bit 1, tile-row bit 0): conflict-free transposed reads for every
// tap shift (tools/ simulation).  Blocks are persistent (one per CU); each writes one fp32 partial
// [64][9*64] that wgrad_reduce sums.
namespace {
constexpr int kL1W = 56;                      // image width handled
constexpr int kL1XP = kL1W + 2;               // halo row pitch (pixels)
constexpr int kL1XRows = 6 * kL1XP;           // 348 halo pixels
constexpr int kL1XBytes = 44 * 1024;          // 352 rows of 128 B (rows >= 348 read zeros)
constexpr int kL1YBytes = 4 * kL1W * 128;     // 28 KB
constexpr int kL1Stage = kL1XBytes + kL1YBytes;
PDT_DEVICE int l1_swz(int row2d, int col) { return (((col >> 1) & 1) << 1) | ((row2d & 1) << 2); }
}  // namespace

// PRE: x is the raw output of the block's first conv; its BatchNorm + ReLU is applied to each staged X halo in
// LDS (conv_l1.hip, PRE) -- the activation is never materialised.
// NWV = 8: two waves per SIMD on the same staged tile, so a SIMD has a second wave to issue from while the other
// waits on its transposed LDS reads (one wave per SIMD: ~36 % MFMA busy, r4_after_pmc.md).  Waves w and w + 4 share
// one 32 k x 32 c quadrant and split either
//  - the column blocks (TSPL = false: even / odd blocks, separate partials, 2 per block; 144 accumulators per lane,
//    too many registers left for PRE's halo transform), or
//  - the taps (TSPL = true: taps 0-4 / 5-8 into one partial per block; 80 accumulators per lane).
template <int DT, bool PRE = false, int NWV = 4, bool TSPL = false>
__global__ __launch_bounds__(64 * NWV) void wgrad3x3_c64_kernel(ConvWgradArgs a) {
  static_assert(NWV == 4 ? !TSPL : (NWV == 8 && (TSPL || !PRE)), "unsupported wgrad3x3_c64 form");
  constexpr int NT = TSPL ? 5 : 9;  // taps per wave
  using E = E16<DT>;
  typedef typename E::vec8 vec8;
  __shared__ __attribute__((aligned(1024))) char smem[2 * kL1Stage];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kh = wave & 1, chh = (wave >> 1) & 1;  // this wave's k half and c half
  const int jp = wave >> 2;                          // NWV = 8: column-block parity / tap half

  const int TH = (a.H + 3) / 4;  // row tiles per image
  const int tiles = a.N * TH;
  const int G = gridDim.x;
  const int xcd = blockIdx.x & 7, lb = blockIdx.x >> 3, per_x = G >> 3;
  const int t_per = (tiles + 7) >> 3;
  const int t_begin = xcd * t_per, t_end = min(tiles, t_begin + t_per);

  // pixel strides (elements): 64, or a 64-channel slice of wider tensors (grouped convs: x stride a.cs, dY a.ldy)
  const int xcs = a.cs > 0 ? a.cs : 64, ycs = a.ldy > 0 ? a.ldy : 64;
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(a.x, (uint32_t)a.N * a.H * kL1W * (uint32_t)xcs * 2u);
  const __amdgpu_buffer_rsrc_t ry = make_rsrc(a.dy, (uint32_t)a.N * a.H * kL1W * (uint32_t)ycs * 2u);
  const int lrow = lane >> 3, pch = lane & 7;

  // 72 DMA instructions per stage (44 X + 28 dY), 72 / NWV per wave
  auto stage_tile = [&](int t, int buf) {
    const int n = t / TH, h0 = (t - n * TH) * 4;
    char* sb = smem + buf * kL1Stage;
#pragma unroll
    for (int m = 0; m < 72 / NWV; ++m) {
      const int ii = wave + NWV * m;
      if (ii < 44) {
        const int R = ii * 8 + lrow;
        const int hr = R / kL1XP, wc = R - (R / kL1XP) * kL1XP;
        const int h = h0 - 1 + hr, w = wc - 1;
        const bool ok = R < kL1XRows && (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)kL1W;
        const int ch = pch ^ l1_swz(hr, wc);
        const uint32_t off = ok ? (uint32_t)((((n * a.H + h) * kL1W + w) * xcs + ch * 8) * 2) : kOOB;
        buf_lds16_asm(rx, sb + ii * 1024, off);
      } else {
        const int R = (ii - 44) * 8 + lrow;
        const int r = R / kL1W, w = R - (R / kL1W) * kL1W;
        const int h = h0 + r;
        const int ch = pch ^ l1_swz(r, w);
        const uint32_t off = h < a.H ? (uint32_t)((((n * a.H + h) * kL1W + w) * ycs + ch * 8) * 2) : kOOB;
        buf_lds16_asm(ry, sb + ii * 1024, off);
      }
    }
  };

  f32x4_t acc[NT][2][2];
#pragma unroll
  for (int tp = 0; tp < NT; ++tp)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[tp][i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // transposed-read lane geometry: 16-lane group g <-> output row g of the K-step
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p4 = li & 3;
  // fragment read: 16 channels [f*16, f*16+16) x 8 pixels (LDS rows R0+0..3 and R0+4..7)
  auto frag = [&](const char* base, int row2d, int col, int f) -> vec8 {
    const int e = f * 16 + 4 * p4;
    const int ch = e >> 3, off = (e & 7) * 2;
    s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_s16x4*)(base + ((ch ^ l1_swz(row2d, col)) << 4) + off));
    s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_s16x4*)(base + 4 * 128 + ((ch ^ l1_swz(row2d, col + 4)) << 4) + off));
    return __builtin_bit_cast(vec8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
  };

  // PRE: thread tid transforms logical chunk tid % 8 (8 fixed channels) of halo rows R = tid/8 + 8*NWV*k; the
  // physical chunk follows the row's swizzle, so each 8-thread group covers one whole 128-B row
  float pre_sc[8], pre_sh[8];
  if constexpr (PRE) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      pre_sc[e] = a.pre_coef[(tid & 7) * 8 + e];
      pre_sh[e] = a.pre_coef[64 + (tid & 7) * 8 + e];
    }
  }

  int t = t_begin + lb;
  int buf = 0;
  if (t < t_end) stage_tile(t, 0);
  for (; t < t_end; t += per_x) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t + per_x < t_end) stage_tile(t + per_x, buf ^ 1);
    // PRE: transform this tile's X halo while the next tile's DMA (into the other buffer) is in flight
    if constexpr (PRE) {
      const int n = t / TH, h0 = (t - n * TH) * 4;
      char* sxw = smem + buf * kL1Stage;
      constexpr int KP = (kL1XRows + 8 * NWV - 1) / (8 * NWV);
      int off[KP];
      bool ok[KP];
#pragma unroll
      for (int k = 0; k < KP; ++k) {
        const int R = min((tid >> 3) + 8 * NWV * k, kL1XRows - 1);
        const int hr = R / kL1XP, wc = R - (R / kL1XP) * kL1XP;
        const int h = h0 - 1 + hr, w = wc - 1;
        ok[k] = (tid >> 3) + 8 * NWV * k < kL1XRows && (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)kL1W;
        off[k] = R * 128 + (((tid & 7) ^ l1_swz(hr, wc)) << 4);
      }
      pre_act_chunks<DT, KP>(sxw, off, ok, pre_sc, pre_sh);
      __syncthreads();
    }
    const char* sx = smem + buf * kL1Stage;
    const char* sy = sx + kL1XBytes;
#pragma unroll 1
    for (int j = TSPL ? 0 : jp; j < kL1W / 8; j += TSPL ? 1 : NWV / 4) {
      // A = dY^T (rows k): output row g, columns 8j + q (+4)
      const int ycol = 8 * j + q;
      const char* yb = sy + (g * kL1W + ycol) * 128;
      vec8 af[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = frag(yb, g, ycol, kh * 2 + i);
#pragma unroll
      for (int u = 0; u < NT; ++u) {
        const int tp = TSPL ? jp * 5 + u : u;  // TSPL: wave-uniform
        if (TSPL && tp >= 9) break;
        const int tr = tp / 3, tu = tp - tr * 3;
        // B = X (cols c): halo row g + tr, halo column 8j + tu + q (+4)
        const int xcol = 8 * j + tu + q;
        const char* xb = sx + ((g + tr) * kL1XP + xcol) * 128;
        vec8 bf[2];
#pragma unroll
        for (int c = 0; c < 2; ++c) bf[c] = frag(xb, g + tr, xcol, chh * 2 + c);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int c = 0; c < 2; ++c) acc[u][i][c] = E::mfma16x16x32(af[i], bf[c], acc[u][i][c]);
      }
    }
    buf ^= 1;
  }

  // partial dW[k][tap][c]: lane holds rows k = kb*16 + 4*(lane>>4) + r, column c = cb*16 + (lane&15); partials of a
  // grouped conv's slice are interleaved with the other slices' ([partial][nslice][64][ldw], a.ws at this slice)
  const int64_t part = TSPL ? (int64_t)blockIdx.x : (int64_t)blockIdx.x * (NWV / 4) + jp;
  float* dst = a.ws + part * (a.nslice > 1 ? a.nslice : 1) * 64 * a.ldw;
#pragma unroll
  for (int u = 0; u < NT; ++u) {
    const int tp = TSPL ? jp * 5 + u : u;
    if (TSPL && tp >= 9) break;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int k = (kh * 2 + i) * 16 + 4 * (lane >> 4);
        const int cc = (chh * 2 + c) * 16 + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) dst[(int64_t)(k + r) * a.ldw + tp * 64 + cc] = acc[u][i][c][r];
      }
  }
}

bool wgrad3x3_c64_supported(int C, int Kout, int T, int U, int W, int stride, int pad, int win) {
  return !win && C == 64 && Kout == 64 && T == 3 && U == 3 && W == kL1W && stride == 1 && pad == 1;
}

// PDT_WGRAD_L1_W8: 0 = 4 waves; 1 = 8 waves splitting the column blocks (two partials per block; calls with PRE
// stay on 4 waves); 2 = 8 waves splitting the taps (one partial per block, PRE included); 3 (default) = the column
// split without PRE, the tap split with PRE.
// Same box, ResNet-18 bf16 B = 1200: 20.166 / 20.111 / 20.064 (0) vs 20.017 / 20.050 / 20.038 ms (1).
// Kernel times, same box (tools/r5_w8_prof.sh): without PRE 268 us (1) vs 301 us (2); with PRE 442 us (4 waves)
// vs 390 us (2).
static int wgrad_l1_w8() {
  static const int mode = [] {
    const char* e = getenv("PDT_WGRAD_L1_W8");
    return e && e[0] >= '0' && e[0] <= '2' ? e[0] - '0' : 3;
  }();
  return mode;
}

// number of fp32 partials the kernel writes (blocks x partials per block)
int wgrad3x3_c64_blocks() {
  int dev = 0, cus = 256;
  PDT_HIP_CHECK(hipGetDevice(&dev));
  PDT_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const int mode = wgrad_l1_w8();
  return (cus + 7) / 8 * 8 * (mode == 1 || mode == 3 ? 2 : 1);
}

int wgrad3x3_c64_launch(const ConvWgradArgs& a, int partials, int dtype, hipStream_t s) {
  // the column-split form is built without PRE (its 144 accumulators + the halo transform exceed the 256 registers
  // of two waves per SIMD and spill inside the DMA window): PRE calls then run 4 waves, one partial per block
  const int mode = wgrad_l1_w8();
  const bool w8 = mode == 1 || mode == 3;  // column split for the calls without PRE
  const bool tspl = mode == 2 || (mode == 3 && a.pre_coef);
  const int blocks = w8 ? partials / 2 : partials;
  PDT_COUNT("wgrad3x3_c64");
  // (a software-pipelined tap loop for the 4-wave form ran slower -- 682 vs 758 TF/s isolated, 20.97 / 20.82 vs
  // 21.03 / 21.00 ms/step -- and was removed in round 6)
  if (a.pre_coef) PDT_COUNT("wgrad3x3_c64_fused_bn_relu");
#define PDT_W3(DT_, P_)                                                                         \
  do {                                                                                          \
    if (tspl)                                                                                   \
      hipLaunchKernelGGL((wgrad3x3_c64_kernel<DT_, P_, 8, true>), dim3(blocks), dim3(512), 0, s, a); \
    else if (w8 && !P_)                                                                         \
      hipLaunchKernelGGL((wgrad3x3_c64_kernel<DT_, false, 8>), dim3(blocks), dim3(512), 0, s, a); \
    else                                                                                        \
      hipLaunchKernelGGL((wgrad3x3_c64_kernel<DT_, P_>), dim3(blocks), dim3(256), 0, s, a); \
  } while (0)
  if (dtype == kBF16) {
    if (a.pre_coef) PDT_W3(kBF16, true); else PDT_W3(kBF16, false);
  } else {
    if (a.pre_coef) PDT_W3(kF16, true); else PDT_W3(kF16, false);
  }
#undef PDT_W3
  return w8 && !a.pre_coef ? partials : blocks;  // partials written (the tap split: one per block)
}

// out[r][c] = scale * sum_s ws[s][r][c]   (r < rows, c < cols; ws row stride ldw, out row stride ldo)
// Block = 64 float4 column groups x 4 split lanes; each split lane keeps 4 loads in flight.
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ ws, int splits, int rows,
                                                            int cols, int ldw, int64_t split_stride,
                                                            float* __restrict__ out, int ldo, float scale,
                                                            int accumulate) {
  const int cv = cols / 4;  // cols % 4 == 0 on this path
  const int64_t nvec = (int64_t)rows * cv;
  const int64_t v = (int64_t)blockIdx.x * 64 + (threadIdx.x & 63);
  const int sl = threadIdx.x >> 6;
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
  int r = 0, c = 0;
  if (v < nvec) {
    r = (int)(v / cv);
    c = (int)(v - (int64_t)r * cv) * 4;
    const float* p = ws + (int64_t)r * ldw + c;
    int s = sl;
    for (; s + 12 < splits; s += 16) {
      const f32x4_t a0 = *(const f32x4_t*)(p + (int64_t)s * split_stride);
      const f32x4_t a1 = *(const f32x4_t*)(p + (int64_t)(s + 4) * split_stride);
      const f32x4_t a2 = *(const f32x4_t*)(p + (int64_t)(s + 8) * split_stride);
      const f32x4_t a3 = *(const f32x4_t*)(p + (int64_t)(s + 12) * split_stride);
      acc += (a0 + a1) + (a2 + a3);
    }
    for (; s < splits; s += 4) acc += *(const f32x4_t*)(p + (int64_t)s * split_stride);
  }
  __shared__ f32x4_t red[4][64];
  red[sl][threadIdx.x & 63] = acc;
  __syncthreads();
  if (sl == 0 && v < nvec) {
    const int t = threadIdx.x;
    const f32x4_t sum = (red[0][t] + red[1][t]) + (red[2][t] + red[3][t]);
    float* o = out + (int64_t)r * ldo + c;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = accumulate ? (o[e] + scale * sum[e]) : scale * sum[e];
  }
}

// scalar fallback for column counts that are not a multiple of 4 (e.g. the 147-wide stem)
__global__ __launch_bounds__(256) void wgrad_reduce_scalar_kernel(const float* __restrict__ ws, int splits, int rows,
                                                                   int cols, int ldw, int64_t split_stride,
                                                                   float* __restrict__ out, int ldo, float scale,
                                                                   int accumulate) {
  const int64_t n = (int64_t)rows * cols;
  for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < n; idx += (int64_t)gridDim.x * 256) {
    const int r = (int)(idx / cols), c = (int)(idx - (int64_t)(idx / cols) * cols);
    const float* p = ws + (int64_t)r * ldw + c;
    float s0 = 0.f, s1 = 0.f;
    int k = 0;
    for (; k + 1 < splits; k += 2) { s0 += p[k * split_stride]; s1 += p[(k + 1) * split_stride]; }
    if (k < splits) s0 += p[k * split_stride];
    float* o = out + (int64_t)r * ldo + c;
    *o = accumulate ? (*o + scale * (s0 + s1)) : scale * (s0 + s1);
  }
}

int wgrad_tile(int C, int Kout, int win) {
  // PDT_WGRAD_PP=0 disables the 256x256 ping-pong kernel (A/B sweeps)
  static const bool pp_on = [] {
    const char* e = getenv("PDT_WGRAD_PP");
    return !(e && e[0] == '0');
  }();
  // PDT_WGRAD_PAIR=0 keeps C == 64 layers on the 64x64 kernel (A/B sweeps)
  static const bool pair_on = [] {
    const char* e = getenv("PDT_WGRAD_PAIR");
    return !(e && e[0] == '0');
  }();
  // PDT_WGRAD_WIDE=0 keeps C % 128 == 0 layers below 256 x 256 on the 128 x 128 kernel (A/B sweeps)
  static const bool wide_on = [] {
    const char* e = getenv("PDT_WGRAD_WIDE");
    return !(e && e[0] == '0');
  }();
  if (!win && pp_on && C % 256 == 0 && Kout % 256 == 0) return 256;
  if (!win && wide_on && C % 128 == 0 && Kout % 128 == 0) return kWgradWide;
  if (!win && pair_on && C == 64 && Kout % 128 == 0) return 128;  // two-tap pair tile
  return (!win && C % 128 == 0 && Kout % 128 == 0) ? 128 : 64;
}

void conv_wgrad_plan(ConvWgradArgs& a, int target_blocks) {
  a.tile = wgrad_tile(a.C, a.Kout, a.win);
  const int tiles = (a.Kout / wgrad_ktile(a)) * wgrad_ctiles(a);
  int splits = (target_blocks + tiles - 1) / tiles;
  if (a.tile == 256 || a.tile == kWgradWide) {
    // one 8-wave block per CU: aim at whole rounds of the CU count (a 2.1-round grid runs 3 rounds)
    static const int cus = [] {
      int dev = 0, n = 0;
      if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        n = 256;
      return n > 0 ? n : 256;
    }();
    // one full round: each block then streams ~130 K-steps (ResNet-18 layer3/4), amortising its prologue
    // and its 256 KB fp32 partial; measured faster than two rounds (tools/conv_bench.py wgrad_256 column)
    (void)target_blocks;
    splits = cus / tiles > 0 ? cus / tiles : 1;
  }
  if (a.win && a.T == 4 && a.U == 1 && a.C == 64 && a.Kout == 64) {
    // the ResNet stem (one block per split covers all 4 pairs): the raw-row kernel runs 3 workgroups per CU
    // (wgrad_stem_rows_kernel: 168 registers, 32 KB LDS) -- one full round of them
    static const int cus3 = [] {
      int dev = 0, n = 0;
      if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        n = 256;
      return 3 * (n > 0 ? n : 256);
    }();
    (void)target_blocks;
    splits = cus3;
  }
  const int max_splits = (a.P + 511) / 512;  // keep >= 4 K-steps per block
  splits = splits < 1 ? 1 : (splits > max_splits ? max_splits : splits);
  int pps = (a.P + splits - 1) / splits;
  pps = (pps + 127) / 128 * 128;
  splits = (a.P + pps - 1) / pps;
  a.splits = splits;
  a.pix_per_split = pps;
}

void conv_wgrad_launch(const ConvWgradArgs& args, int dtype, hipStream_t s) {
  ConvWgradArgs a = args;
  if (a.nslice > 1 && (a.tile != 64 || a.win))
    pdt_hip_fail("conv_wgrad: slice-batched (grouped) launches run on the 64x64 tile only", hipErrorInvalidValue,
                 __FILE__, __LINE__);
  if (a.ldy && a.ldy != a.Kout && (a.tile != 64 || a.win))
    pdt_hip_fail("conv_wgrad: a strided dY (channel slice) runs on the 64x64 tile only", hipErrorInvalidValue,
                 __FILE__, __LINE__);
  if (a.pre_coef && !(a.tile == 128 && a.C == 64 && !a.win))
    pdt_hip_fail("conv_wgrad: a fused producer BN (pre_coef) runs on the 128-pair tile only (C == 64)",
                 hipErrorInvalidValue, __FILE__, __LINE__);
  // the wide kernel's incremental DMA addressing steps 4 grid columns with one row wrap: narrower outputs run the
  // 128 x 128 tile (same split plan and partial layout)
  if (a.tile == kWgradWide && a.Qm < 4) a.tile = 128;
  if (a.tile == 128 && a.Qm < 4) {  // (the 128 x 128 kernel steps 4 grid columns the same way)
    if (a.pre_coef)
      pdt_hip_fail("conv_wgrad: a fused producer BN needs an output at least 4 pixels wide", hipErrorInvalidValue,
                   __FILE__, __LINE__);
    a.tile = 64;
  }
  const int nwg = (a.Kout / wgrad_ktile(a)) * wgrad_ctiles(a) * a.splits;
  if (nwg == 0) return;
  const FastDiv dpq = make_fastdiv((uint32_t)(a.Pm * a.Qm)), dq = make_fastdiv((uint32_t)a.Qm);
  a.div_pq_mul = dpq.mul; a.div_pq_shift = dpq.shift; a.div_q_mul = dq.mul; a.div_q_shift = dq.shift;
  if (a.tile == 256) {
    PDT_COUNT("conv_wgrad_pp");
    if (dtype == kBF16)
      hipLaunchKernelGGL((conv_wgrad_pp_kernel<kBF16>), dim3(nwg), dim3(512), 0, s, a);
    else
      hipLaunchKernelGGL((conv_wgrad_pp_kernel<kF16>), dim3(nwg), dim3(512), 0, s, a);
  } else if (a.tile == kWgradWide) {
    PDT_COUNT("conv_wgrad_wide");
    if (dtype == kBF16) {
      hipLaunchKernelGGL((conv_wgrad_wide_kernel<kBF16, 64>), dim3(nwg), dim3(512), 0, s, a);
    } else {
      hipLaunchKernelGGL((conv_wgrad_wide_kernel<kF16, 64>), dim3(nwg), dim3(512), 0, s, a);
    }
  } else if (a.tile == 128 && a.C == 64 && a.pre_coef) {
    if (a.T != 1 || a.U != 1 || a.stride_h != 1 || a.stride_w != 1 || a.pad_h != 0 || a.pad_w != 0)
      pdt_hip_fail("conv_wgrad: a fused producer BN on the 128-pair tile needs a 1x1 / stride-1 conv",
                   hipErrorInvalidValue, __FILE__, __LINE__);
    PDT_COUNT("conv_wgrad_128_pair_fused_bn_relu");
    if (dtype == kBF16)
      hipLaunchKernelGGL((conv_wgrad128_kernel<kBF16, true, true>), dim3(nwg), dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL((conv_wgrad128_kernel<kF16, true, true>), dim3(nwg), dim3(256), 0, s, a);
  } else if (a.tile == 128 && a.C == 64) {
    PDT_COUNT("conv_wgrad_128_pair");
    if (dtype == kBF16)
      hipLaunchKernelGGL((conv_wgrad128_kernel<kBF16, true>), dim3(nwg), dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL((conv_wgrad128_kernel<kF16, true>), dim3(nwg), dim3(256), 0, s, a);
  } else if (a.tile == 128) {
    PDT_COUNT("conv_wgrad_128");
    if (dtype == kBF16)
      hipLaunchKernelGGL((conv_wgrad128_kernel<kBF16, false>), dim3(nwg), dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL((conv_wgrad128_kernel<kF16, false>), dim3(nwg), dim3(256), 0, s, a);
  } else if (a.win && a.T == 4 && a.U == 1 && a.C == 64 && a.Kout == 64 && a.ldw >= 256) {
    // ResNet stem (4 kernel-row pairs): one block per split covers all pairs
    if (a.f_y != nullptr)
      PDT_COUNT("wgrad_stem_fused");
    else
      PDT_COUNT("wgrad_stem");
    if (a.f_y != nullptr && a.Pm % 4 == 0 && a.Qm % 16 == 0 && a.pix_per_split % 64 == 0 &&
               a.stride_h == 2 && a.dil_h == 2 && a.pad_h == 0 && a.cs == 4) {
      // raw-image-row staging (wgrad_stem_rows_kernel): steps are 4 x 16 pixel blocks, divisions by steps per
      // image and per 4-row band
      const int SW = a.Qm / 16, SPI = (a.Pm / 4) * SW;
      const FastDiv dspi = make_fastdiv((uint32_t)SPI), dsw = make_fastdiv((uint32_t)SW);
      a.div_pq_mul = dspi.mul; a.div_pq_shift = dspi.shift; a.div_q_mul = dsw.mul; a.div_q_shift = dsw.shift;
      PDT_COUNT("wgrad_stem_rows");
      if (dtype == kBF16)
        hipLaunchKernelGGL((wgrad_stem_rows_kernel<kBF16>), dim3(a.splits), dim3(256), 0, s, a);
      else
        hipLaunchKernelGGL((wgrad_stem_rows_kernel<kF16>), dim3(a.splits), dim3(256), 0, s, a);
    } else if (a.f_y != nullptr) {
      // quad order (wgrad_stem_quad_kernel): the divisions are by quads per image and quads per row, and the
      // pixel count is padded to whole quads (an odd height's last quad row is half dead)
      const int QR = (a.Pm + 1) / 2, QC = a.Qm / 2;
      const FastDiv dqi = make_fastdiv((uint32_t)(QR * QC)), dqc = make_fastdiv((uint32_t)QC);
      a.div_pq_mul = dqi.mul; a.div_pq_shift = dqi.shift; a.div_q_mul = dqc.mul; a.div_q_shift = dqc.shift;
      a.P = a.N * QR * QC * 4;
      if (a.Qm % 2 != 0 || (int64_t)a.splits * a.pix_per_split < a.P)
        pdt_hip_fail("wgrad_stem_quad: needs an even width and a split plan over the quad-padded pixels",
                     hipErrorInvalidValue, __FILE__, __LINE__);
      if (dtype == kBF16)
        hipLaunchKernelGGL((wgrad_stem_quad_kernel<kBF16>), dim3(a.splits), dim3(256), 0, s, a);
      else
        hipLaunchKernelGGL((wgrad_stem_quad_kernel<kF16>), dim3(a.splits), dim3(256), 0, s, a);
    } else if (dtype == kBF16) {
      hipLaunchKernelGGL((wgrad_stem_kernel<kBF16>), dim3(a.splits), dim3(256), 0, s, a);
    } else {
      hipLaunchKernelGGL((wgrad_stem_kernel<kF16>), dim3(a.splits), dim3(256), 0, s, a);
    }
  } else if (a.win) {
    PDT_COUNT("conv_wgrad_window");
    if (dtype == kBF16)
      hipLaunchKernelGGL((conv_wgrad_kernel<kBF16, true>), dim3(nwg), dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL((conv_wgrad_kernel<kF16, true>), dim3(nwg), dim3(256), 0, s, a);
  } else {
    PDT_COUNT("conv_wgrad_generic");
    const dim3 g(nwg, 1, a.nslice > 1 ? a.nslice : 1);
    if (dtype == kBF16)
      hipLaunchKernelGGL((conv_wgrad_kernel<kBF16, false>), g, dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL((conv_wgrad_kernel<kF16, false>), g, dim3(256), 0, s, a);
  }
  PDT_HIP_CHECK(hipGetLastError());  // a refused launch (e.g. LDS / register limits) must not leave ws stale
}

void wgrad_reduce_launch(const float* ws, int splits, int rows, int cols, int ldw, int64_t split_stride,
                         float* out, int ldo, float scale, bool accumulate, hipStream_t s) {
  if ((int64_t)rows * cols == 0) return;
  const bool vec = (cols % 4 == 0) && (ldw % 4 == 0) && (ldo % 4 == 0) && (split_stride % 4 == 0) &&
                   ((uintptr_t)ws % 16 == 0) && ((uintptr_t)out % 16 == 0);
  if (vec) {
    const int64_t nvec = (int64_t)rows * (cols / 4);
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)((nvec + 63) / 64)), dim3(256), 0, s, ws, splits, rows,
                       cols, ldw, split_stride, out, ldo, scale, (int)accumulate);
  } else {
    int64_t blocks = ((int64_t)rows * cols + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(wgrad_reduce_scalar_kernel, dim3((unsigned)blocks), dim3(256), 0, s, ws, splits, rows, cols,
                       ldw, split_stride, out, ldo, scale, (int)accumulate);
  }
}

}  // namespace pdt
