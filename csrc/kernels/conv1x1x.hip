// Expanding 1x1 / stride-1 GEMMs of ResNet-50 layers 2-4 (K = 128 / 256 / 512 reduction channels, N = 4K output
// channels) as persistent, store-overlapped kernels: the generalisation of conv1x1.hip (K = 64, N = 256) to
// reductions whose weights no longer fit in one block's registers.
//
// Two GEMMs have this shape: every bottleneck's conv3 forward (y[M][4C] = x[M][C] * W^T, + BN statistics) and the
// backward-data pass of its conv1 (dX[M][4C] = dY[M][C] * W, with the block-output BN-backward epilogue of
// conv_fwd.h EPI 3 / 4).  On the generic ping-pong kernel (one 512 x 128 tile per workgroup, 2-8 K-steps) they run
// at 2.1-2.8 TB/s of HBM traffic: each workgroup's life is load latency -> a few MFMAs -> an epilogue writing 4x the
// bytes it read, with nothing of the next tile in flight (profiles/r5_resnet50_bs1200_kernels.md).  Here:
//   * the N output channels are split into S slices of NS = 4 waves x 16*NF channels; a block owns one slice and
//     keeps that slice's weights (NS x K) resident in registers as MFMA A fragments, staged once through LDS in
//     64-channel K pieces;
//   * blocks are persistent (2 per CU) and walk BM-pixel tiles; a tile's input (BM x K) is DMA'd into a 2-deep LDS
//     ring one tile ahead, and the per-tile wait is COUNTED: the next tile's DMA is issued before this tile's
//     epilogue operand loads and stores, so waiting for it leaves them in flight;
//   * the S blocks of one tile sequence sit on the SAME XCD (block b runs on XCD b % 8 under the round-robin
//     dispatch): the input is fetched from HBM once and re-read by the other slices from that XCD's L2;
//   * statistics accumulate in registers over all of a block's tiles; one partial row per tile walker (the S slices
//     of a walker write disjoint channel ranges of the same row), reduced in fixed order (conv_fwd.h).
// Configurations (register budget: 2 waves per SIMD): K = 128: 64 channels per wave, BM = 64 (S = N / 256);
// K = 256: 64 (forward) / 32 (backward-data) channels per wave, BM = 64; K = 512: 32 channels per wave, BM = 32.
// The forward also takes stride-2 input (the downsample convs of layers 2-3: 256 -> 512, 512 -> 1024).
#include <cstdlib>
#include <type_traits>

#include "../common.h"
#include "conv1x1.h"
#include "conv_fwd.h"

namespace pdt {

namespace {
constexpr int kXRowB = 128;  // 64 16-bit channels per LDS row

template <int KH, int NF, int BM>
struct X1 {
  static constexpr int WCH = 16 * NF;              // output channels per wave
  static constexpr int NS = 4 * WCH;               // per block (slice)
  static constexpr int TILE = BM * KH * kXRowB;    // one tile's input, all 64-channel K pieces
  static constexpr int WPIECE = NS * kXRowB;       // one K piece of the slice's weights
  static constexpr int AREA = 2 * TILE > WPIECE ? 2 * TILE : WPIECE;
  static constexpr int XI = TILE / 1024 / 4;       // input DMA instructions per wave per tile
  static constexpr int WI = WPIECE / 1024 / 4;     // weight DMA instructions per wave per piece
  static_assert(XI * 4096 == TILE && WI * 4096 == WPIECE && BM % 32 == 0, "conv1x1x geometry");
  static_assert(NF == 2 || NF == 4, "fragment pairs");
};

// fragments 2p and 2p+1 give a lane 8 consecutive channels of its pixel (one 16-byte store per pixel and pair)
PDT_DEVICE int x1_wave_ch(int i, int row) { return (i >> 1) * 32 + (row >> 2) * 8 + (i & 1) * 4 + (row & 3); }

template <int N>
PDT_DEVICE void x1_vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}

// block -> (slice, tile walker): blocks b and b + 8 share an XCD; the S slices of walker l are consecutive there
struct X1Map {
  int slice, walker;
};
PDT_DEVICE X1Map x1_map(int b, int S) {
  const int xcd = b & 7, q = b >> 3;
  return X1Map{q % S, (q / S) * 8 + xcd};
}

// the slice's weights [n0, n0 + NS) x [0, 64 KH) into registers (af[i][kq]: fragment i, 32-channel K step kq),
// through the LDS area in 64-channel pieces
template <int DT, int KH, int NF, int BM>
PDT_DEVICE void x1_load_weights(typename E16<DT>::vec8 (&af)[NF][2 * KH], const __amdgpu_buffer_rsrc_t& rw,
                                char* wl, int n0, int wave, int lane) {
  using C = X1<KH, NF, BM>;
  typedef typename E16<DT>::vec8 vec8;
  const int fr = lane & 15, fq = lane >> 4, lrow = lane >> 3, pchunk = lane & 7;
#pragma unroll
  for (int hh = 0; hh < KH; ++hh) {
#pragma unroll
    for (int j = 0; j < C::WI; ++j) {
      const int ins = wave * C::WI + j;
      const int row = ins * 8 + lrow;
      buf_lds16_asm(rw, wl + ins * 1024,
                    (uint32_t)((n0 + row) * (KH * kXRowB) + hh * kXRowB + ((pchunk ^ ((row >> 1) & 7)) << 4)));
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NF; ++i) {
      const int wr = wave * C::WCH + x1_wave_ch(i, fr);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        af[i][2 * hh + kk] = *(const vec8*)(wl + wr * kXRowB + (((kk * 4 + fq) ^ ((wr >> 1) & 7)) << 4));
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();  // every wave holds this piece: the area is free again
  }
}

// strided input (a 1x1 / stride-st conv, st > 1: the downsample convs): output pixel m = (n, i, j) reads input pixel
// (n, st*i, st*j) of an H x W image; P*Q and Q as exact reciprocals
struct X1Geo {
  int st, H, W, PQ, Q;
  uint32_t pq_mul, pq_shift, q_mul, q_shift;
};

// one tile's input: XI DMA instructions per wave; rows past M read zeros (their results are not stored) -- CL: row
// M - 1 instead (every DMA piece a real access: counted waits that assume in-order retirement)
template <int KH, int NF, int BM, bool SD = false, bool CL = false>
PDT_DEVICE void x1_stage(const __amdgpu_buffer_rsrc_t& rx, char* xl, int64_t t, int buf, int64_t M, int wave,
                         int lane, const X1Geo& g = X1Geo{}) {
  using C = X1<KH, NF, BM>;
  const int lrow = lane >> 3, pchunk = lane & 7;
#pragma unroll
  for (int j = 0; j < C::XI; ++j) {
    const int ins = wave * C::XI + j;
    const int hh = ins / (BM / 8), row = (ins % (BM / 8)) * 8 + lrow;
    const int64_t m0 = t * BM + row;
    const int64_t m = CL && m0 >= M ? M - 1 : m0;
    int64_t src = m;
    if constexpr (SD) {
      const uint32_t mu = (uint32_t)m;
      const uint32_t n = fdiv(mu, FastDiv{g.pq_mul, g.pq_shift});
      const uint32_t rem = mu - n * (uint32_t)g.PQ;
      const uint32_t i = fdiv(rem, FastDiv{g.q_mul, g.q_shift}), jj = rem - i * (uint32_t)g.Q;
      src = ((int64_t)n * g.H + (int64_t)g.st * i) * g.W + (int64_t)g.st * jj;
    }
    const uint32_t off =
        m < M ? (uint32_t)(src * (KH * kXRowB) + hh * kXRowB + ((pchunk ^ ((row >> 1) & 7)) << 4)) : kOOB;
    buf_lds16_asm(rx, xl + buf * C::TILE + ins * 1024, off);
  }
}

// acc[i][j] (fragment i of the wave's channels, pixel fragment j of the PJ*16-pixel sub-tile s) over the whole
// reduction
template <int DT, int KH, int NF, int BM, int PJ>
PDT_DEVICE void x1_mma(f32x4_t (&acc)[NF][PJ], const typename E16<DT>::vec8 (&af)[NF][2 * KH], const char* xb, int s,
                       int lane) {
  typedef typename E16<DT>::vec8 vec8;
  const int fr = lane & 15, fq = lane >> 4, sw = (fr >> 1) & 7;
#pragma unroll
  for (int i = 0; i < NF; ++i)
#pragma unroll
    for (int j = 0; j < PJ; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kq = 0; kq < 2 * KH; ++kq) {
    vec8 bf[PJ];
#pragma unroll
    for (int j = 0; j < PJ; ++j)
      bf[j] = *(const vec8*)(xb + (kq >> 1) * BM * kXRowB + ((s * PJ + j) * 16 + fr) * kXRowB +
                             ((((kq & 1) * 4 + fq) ^ sw) << 4));
#pragma unroll
    for (int i = 0; i < NF; ++i)
#pragma unroll
      for (int j = 0; j < PJ; ++j) acc[i][j] = E16<DT>::mfma16x16x32(af[i][kq], bf[j], acc[i][j]);
  }
}

}  // namespace

// ------------------------------------------------------------------------------------------------ forward
// SD: strided input (X1Geo; x holds x_rows pixels)
template <int DT, bool STATS, int KH, int NF, int BM, bool SD>
__global__ __launch_bounds__(256, 2) void conv1x1x_kernel(const uint16_t* __restrict__ x,
                                                          const uint16_t* __restrict__ w, uint16_t* __restrict__ y,
                                                          float* __restrict__ srows, int64_t M, int N, int S,
                                                          int64_t x_rows, X1Geo geo) {
  using C = X1<KH, NF, BM>;
  using E = E16<DT>;
  typedef typename E::vec8 vec8;
  constexpr int OPS = (BM / 16) * (NF / 2);  // vector-memory ops per wave after the next tile's DMA (stores)
  __shared__ __attribute__((aligned(1024))) char smem[C::AREA];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const X1Map mp = x1_map(blockIdx.x, S);
  const int Gs = gridDim.x / S;
  const int n0 = mp.slice * C::NS;
  const int64_t tiles = (M + BM - 1) / BM;
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(x, (uint32_t)(x_rows * KH * kXRowB));
  const __amdgpu_buffer_rsrc_t rw = make_rsrc(w, (uint32_t)((int64_t)N * KH * kXRowB));

  vec8 af[NF][2 * KH];
  x1_load_weights<DT, KH, NF, BM>(af, rw, smem, n0, wave, lane);

  float ssum[NF][4], ssq[NF][4];
#pragma unroll
  for (int i = 0; i < NF; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) { ssum[i][r] = 0.f; ssq[i][r] = 0.f; }

  int64_t t = mp.walker;
  if (t < tiles) x1_stage<KH, NF, BM, SD>(rx, smem, t, 0, M, wave, lane, geo);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int buf = 0;
  bool first = true;
  for (; t < tiles; t += Gs) {
    if (!first) {
      // tile t's DMA was issued before the previous (full: only a walker's last tile can be the M tail) tile's OPS
      // stores; vector-memory ops retire in order, so waiting down to OPS outstanding retires the DMA only
      x1_vm_wait<OPS>();
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
    first = false;
    if (t + Gs < tiles) x1_stage<KH, NF, BM, SD>(rx, smem, t + Gs, buf ^ 1, M, wave, lane, geo);
    const char* xb = smem + buf * C::TILE;
#pragma unroll
    for (int s = 0; s < BM / 32; ++s) {
      f32x4_t acc[NF][2];
      x1_mma<DT, KH, NF, BM, 2>(acc, af, xb, s, lane);
      // pair p gives the lane channels n0 + wave*WCH + p*32 + 8*fq + [0, 8) of pixel t*BM + (2s + j)*16 + fr
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int64_t m = t * BM + (s * 2 + j) * 16 + fr;
        uint16_t* yp = y + m * N + n0 + wave * C::WCH + 8 * fq;
#pragma unroll
        for (int p = 0; p < NF / 2; ++p) {
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
#pragma unroll
    for (int i = 0; i < NF; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        ssum[i][r] = row16_sum(ssum[i][r]);
        ssq[i][r] = row16_sum(ssq[i][r]);
      }
    if (fr == 15) {
      float* dst = srows + (int64_t)mp.walker * N * 2;
#pragma unroll
      for (int i = 0; i < NF; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int c = n0 + wave * C::WCH + x1_wave_ch(i, 4 * fq + r);
          *(float2*)(dst + c * 2) = make_float2(ssum[i][r], ssq[i][r]);
        }
    }
  }
}

// ------------------------------------------------------------------------------------------------ backward data
// dX = dY * W with the block-output BN-backward epilogue (conv1x1.hip's conv1x1_c64_bnb_kernel, generalised):
// v = acc + res, dz = v where the block output's ReLU bit is set (else 0), stored rounded; per channel sum(dz) and
// sum(dz * (y1 - mean1) * invstd1) (BR = 2: + sum(dz * (y2 - mean2) * invstd2)) into the walker's statistics row.
//
// Every vector-memory operation of the loop is issued through inline asm and waited for with COUNTED vmcnt: with
// compiler-visible operand loads, the compiler's own waits (exact only for the operations it knows of) also retire
// the next tile's LDS-DMA issued ahead of them, and a partial-tile branch makes it fall back to vmcnt(0) at the loop
// top -- the DMA latency was exposed on every tile.  Here the epilogue operands (residual, BN inputs, the mask byte)
// of sub-tile s + 1 are loaded while sub-tile s computes (the next tile's first sub-tile during the last one), and a
// walker's last tile still issues the DMA and operand prefetch of the tile after it, so every wait count is a constant.
// Loads and DMA pieces of rows past M read row M - 1 (never an out-of-range access, whose early retirement would break
// the in-order count); stores keep the true row, and the range check drops those past M.  The counts cover LOADS only
// (per sub-tile NL operand loads): the wait for sub-tile s's operands leaves the younger DMA pieces / loads in flight,
// the loop-top wait for the tile's DMA the previous tile's SUB * NL loads; stores never relax a wait.
// (Round 5: with the stores counted and out-of-range operand rows, the C = 64 configuration read stale operands; the
// two changes were made together, so which one it needed is not isolated.)
// PJ: pixel fragments per sub-tile (two operand sets must fit the register budget).
namespace {
PDT_DEVICE u32x4v x1_ld16(const __amdgpu_buffer_rsrc_t& r, uint32_t off) {
  u32x4v v;
  asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(v) : "v"(off), "s"(r));
  return v;
}
PDT_DEVICE uint32_t x1_ld1(const __amdgpu_buffer_rsrc_t& r, uint32_t off) {
  uint32_t v;
  asm volatile("buffer_load_ubyte %0, %1, %2, 0 offen" : "=v"(v) : "v"(off), "s"(r));
  return v;
}
// (s_nop 1: a >8-byte store reads its data VGPRs after issue -- the next instructions hipcc places behind the opaque
// asm may overwrite them; it pads only the stores it emits itself)
PDT_DEVICE void x1_st16(const __amdgpu_buffer_rsrc_t& r, uint32_t off, u32x4v v) {
  asm volatile("buffer_store_dwordx4 %0, %1, %2, 0 offen\n\ts_nop 1" : : "v"(v), "v"(off), "s"(r) : "memory");
}
template <int SET, int PJ, int NP, int BR>
PDT_DEVICE void x1_pin(u32x4v (&rr)[2][PJ][NP], u32x4v (&yy)[2][PJ][NP], u32x4v (&yz)[2][BR == 2 ? PJ : 1][NP],
                       uint32_t (&mb)[2][PJ][NP]) {
#pragma unroll
  for (int j = 0; j < PJ; ++j)
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      asm volatile("" : "+v"(rr[SET][j][p]), "+v"(yy[SET][j][p]), "+v"(mb[SET][j][p]));
      if constexpr (BR == 2) asm volatile("" : "+v"(yz[SET][j][p]));
    }
}
template <int N>
PDT_DEVICE void x1_vm_wait_asm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
#ifdef PDT_X1_WAIT0
  asm volatile("s_waitcnt vmcnt(0)" : : : "memory");
#else
  asm volatile("s_waitcnt vmcnt(%0)" : : "n"(N) : "memory");
#endif
}
}  // namespace

template <int DT, int BR, int KH, int NF, int BM, int PJ>
__global__ __launch_bounds__(256, 2) void conv1x1x_bnb_kernel(
    const uint16_t* __restrict__ x, const uint16_t* __restrict__ w, uint16_t* __restrict__ y,
    const uint16_t* __restrict__ res, const uint16_t* __restrict__ y1, const float* __restrict__ coef1,
    const uint16_t* __restrict__ y2, const float* __restrict__ coef2, const uint8_t* __restrict__ mask,
    float* __restrict__ srows, int64_t M, int N, int S) {
  static_assert(BR == 1 || BR == 2, "one or two BatchNorm branches");
  using C = X1<KH, NF, BM>;
  using E = E16<DT>;
  typedef typename E::vec8 vec8;
  constexpr int NP = NF / 2;                          // channel pairs (8 consecutive channels each) per lane
  constexpr int SUB = BM / (16 * PJ);                 // sub-tiles per tile
  constexpr int NL = PJ * NP * (BR == 2 ? 4 : 3);     // operand loads per sub-tile (16-B res, y1 (, y2); mask byte)
  constexpr int NS = PJ * NP;                         // stores per sub-tile
  constexpr int TOP = SUB * NL;                       // loads in flight behind the next tile's DMA at the loop top
  static_assert(SUB % 2 == 0 && TOP < 64 && C::XI + NL < 64, "conv1x1x_bnb wait counts");
  __shared__ __attribute__((aligned(1024))) char smem[C::AREA + BR * 2 * C::NS * 4];
  float* const cf = (float*)(smem + C::AREA);  // cf[(branch * 2 + 0 | 1) * NS + c]: mean | invstd of the slice
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const X1Map mp = x1_map(blockIdx.x, S);
  const int Gs = gridDim.x / S;
  const int n0 = mp.slice * C::NS;
  const int64_t tiles = (M + BM - 1) / BM;
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(x, (uint32_t)(M * KH * kXRowB));
  const __amdgpu_buffer_rsrc_t rw = make_rsrc(w, (uint32_t)((int64_t)N * KH * kXRowB));
  const uint32_t obytes = (uint32_t)(M * N * 2);  // < 2^31 (host check): rows past M are out of range
  const __amdgpu_buffer_rsrc_t rres = make_rsrc(res, obytes), ry1 = make_rsrc(y1, obytes);
  const __amdgpu_buffer_rsrc_t ry2 = make_rsrc(BR == 2 ? y2 : y1, obytes), rdz = make_rsrc(y, obytes);
  const __amdgpu_buffer_rsrc_t rmask = make_rsrc(mask, (uint32_t)(M * N / 8));

  if (tid < C::NS) {
    cf[tid] = coef1[2 * N + n0 + tid];
    cf[C::NS + tid] = coef1[3 * N + n0 + tid];
    if constexpr (BR == 2) {
      cf[2 * C::NS + tid] = coef2[2 * N + n0 + tid];
      cf[3 * C::NS + tid] = coef2[3 * N + n0 + tid];
    }
  }
  vec8 af[NF][2 * KH];
  x1_load_weights<DT, KH, NF, BM>(af, rw, smem, n0, wave, lane);  // (its barriers also publish cf)

  float s0[NP][8], s1[NP][8], s2[BR == 2 ? NP : 1][8];
#pragma unroll
  for (int p = 0; p < NP; ++p)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      s0[p][e] = 0.f;
      s1[p][e] = 0.f;
      if constexpr (BR == 2) s2[p][e] = 0.f;
    }

  // operand sets: [set][pixel fragment j][pair p]
  u32x4v rr[2][PJ][NP], yy[2][PJ][NP], yz[2][BR == 2 ? PJ : 1][NP];
  uint32_t mb[2][PJ][NP];
  // element offset of (pixel fragment j of sub-tile s of tile t, pair p); CLAMP: operand loads read row M - 1 for
  // rows past M (every load a real access -- out-of-range ones could retire ahead of older loads), stores use the
  // true row and the range check drops them
  auto eoff = [&](int64_t t, int s, int j, int p, bool clamp) -> uint32_t {
    int64_t m = t * BM + (s * PJ + j) * 16 + fr;
    if (clamp) m = m < M ? m : M - 1;
    return (uint32_t)(m * N + n0 + wave * C::WCH + p * 32 + 8 * fq);
  };
  auto load_ops = [&](auto SETc, int64_t t, int s) {
    constexpr int SET = decltype(SETc)::value;
#pragma unroll
    for (int j = 0; j < PJ; ++j)
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        const uint32_t o = eoff(t, s, j, p, true);
        rr[SET][j][p] = x1_ld16(rres, o * 2u);
        yy[SET][j][p] = x1_ld16(ry1, o * 2u);
        if constexpr (BR == 2) yz[SET][j][p] = x1_ld16(ry2, o * 2u);
        mb[SET][j][p] = x1_ld1(rmask, o >> 3);
      }
  };
  auto pin_ops = [&](auto SETc) {  // after the covering wait: no use may be scheduled ahead of it
    x1_pin<decltype(SETc)::value, PJ, NP, BR>(rr, yy, yz, mb);
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;

  int64_t t = mp.walker;
  if (t < tiles) {
    x1_stage<KH, NF, BM, false, true>(rx, smem, t, 0, M, wave, lane);
    load_ops(I0{}, t, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  pin_ops(I0{});
  int buf = 0;
  bool first = true;
  for (; t < tiles; t += Gs) {
    if (!first) {
      x1_vm_wait_asm<TOP>();  // this tile's DMA; the previous tile's prefetch loads stay in flight
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
    first = false;
    // the next tile's DMA (past the walker's last tile: all rows out of range, zeros into the free ring slot)
    x1_stage<KH, NF, BM, false, true>(rx, smem, t + Gs, buf ^ 1, M, wave, lane);
    const char* xb = smem + buf * C::TILE;
    auto sub = [&](auto SETc, int s) {
      constexpr int SET = decltype(SETc)::value;
      // prefetch the next sub-tile's operands (the next tile's first one during the last sub-tile)
      if (s + 1 < SUB)
        load_ops(std::integral_constant<int, SET ^ 1>{}, t, s + 1);
      else
        load_ops(std::integral_constant<int, SET ^ 1>{}, t + Gs, 0);
      f32x4_t acc[NF][PJ];
      x1_mma<DT, KH, NF, BM, PJ>(acc, af, xb, s, lane);
      // wait for this sub-tile's operands: younger than them are the next tile's DMA (s == 0) or the previous
      // sub-tile's stores (s > 0), and the prefetch just issued
      if (s == 0)
        x1_vm_wait_asm<C::XI + NL>();
      else
        x1_vm_wait_asm<NL>();
      pin_ops(SETc);
#pragma unroll
      for (int j = 0; j < PJ; ++j) {
        const int64_t m = t * BM + (s * PJ + j) * 16 + fr;
#pragma unroll
        for (int p = 0; p < NP; ++p) {
          const u32x4v r4 = rr[SET][j][p], y4 = yy[SET][j][p];
          float vv[8], q1[8], q2[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            float v = acc[2 * p + (e >> 2)][j][e & 3] + E::to_f((uint16_t)(r4[e >> 1] >> (16 * (e & 1))));
            if (!((mb[SET][j][p] >> e) & 1u)) v = 0.f;
            vv[e] = v;
            q1[e] = E::to_f((uint16_t)(y4[e >> 1] >> (16 * (e & 1))));
          }
          if constexpr (BR == 2) {
            const u32x4v z4 = yz[SET][j][p];
#pragma unroll
            for (int e = 0; e < 8; ++e) q2[e] = E::to_f((uint16_t)(z4[e >> 1] >> (16 * (e & 1))));
          }
          uint4 pk;  // one v_cvt_pk_bf16_f32 per pair (E16::pack2)
          pk.x = E::pack2(vv[0], vv[1]);
          pk.y = E::pack2(vv[2], vv[3]);
          pk.z = E::pack2(vv[4], vv[5]);
          pk.w = E::pack2(vv[6], vv[7]);
          uint16_t o[8];
          unpack8(pk, o);
          x1_st16(rdz, eoff(t, s, j, p, false) * 2u, u32x4v{pk.x, pk.y, pk.z, pk.w});  // rows past M: dropped
          if (m < M) {
            const int cl = wave * C::WCH + p * 32 + 8 * fq;  // slice-local channel
            const float4 ma = *(const float4*)(cf + cl), mb4 = *(const float4*)(cf + cl + 4);
            const float4 ia = *(const float4*)(cf + C::NS + cl), ib = *(const float4*)(cf + C::NS + cl + 4);
            const float mu[8] = {ma.x, ma.y, ma.z, ma.w, mb4.x, mb4.y, mb4.z, mb4.w};
            const float is[8] = {ia.x, ia.y, ia.z, ia.w, ib.x, ib.y, ib.z, ib.w};
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float dz = E::to_f(o[e]);
              s0[p][e] += dz;
              s1[p][e] += dz * (q1[e] - mu[e]) * is[e];
            }
            if constexpr (BR == 2) {
              const float4 na = *(const float4*)(cf + 2 * C::NS + cl), nb = *(const float4*)(cf + 2 * C::NS + cl + 4);
              const float4 ja = *(const float4*)(cf + 3 * C::NS + cl), jb = *(const float4*)(cf + 3 * C::NS + cl + 4);
              const float mu2[8] = {na.x, na.y, na.z, na.w, nb.x, nb.y, nb.z, nb.w};
              const float is2[8] = {ja.x, ja.y, ja.z, ja.w, jb.x, jb.y, jb.z, jb.w};
#pragma unroll
              for (int e = 0; e < 8; ++e) s2[p][e] += E::to_f(o[e]) * (q2[e] - mu2[e]) * is2[e];
            }
          }
        }
      }
    };
#pragma unroll
    for (int s2i = 0; s2i < SUB; s2i += 2) {
      sub(I0{}, s2i);
      sub(I1{}, s2i + 1);
    }
    buf ^= 1;
  }
  // the last stores and the last (unused) operand prefetch -- set 0, pinned behind the wait: until then its registers
  // may not be handed to the statistics reduction below (a late load would overwrite it; found in round 5)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  pin_ops(I0{});

#pragma unroll
  for (int p = 0; p < NP; ++p)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      s0[p][e] = row16_sum(s0[p][e]);
      s1[p][e] = row16_sum(s1[p][e]);
      if constexpr (BR == 2) s2[p][e] = row16_sum(s2[p][e]);
    }
  if (fr == 15) {
    constexpr int KO = BR == 2 ? 4 : 2;
    float* dst = srows + (int64_t)mp.walker * N * KO;
#pragma unroll
    for (int p = 0; p < NP; ++p)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = n0 + wave * C::WCH + p * 32 + 8 * fq + e;
        if constexpr (BR == 2)
          *(float4*)(dst + c * 4) = make_float4(s0[p][e], s1[p][e], s0[p][e], s2[p][e]);
        else
          *(float2*)(dst + c * 2) = make_float2(s0[p][e], s1[p][e]);
      }
  }
}

// ------------------------------------------------------------------------------------------------ host
namespace {
int x1_cus() {
  static const int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      n = 256;
    return n > 0 ? n : 256;
  }();
  return cus;
}

// forward, C = 256: 64 channels per wave as for C = 128 (slices of 256: half the L2 re-reads of the input; ResNet-50
// 72.68 -> 72.27 ms/step, same box, against 32 channels per wave)
bool x1_wide() { return true; }
// NS of C's configuration (the backward-data kernel has no register room for the wide C = 256 variant)
int x1_slice(int C, bool fwd) { return C <= 128 || (C == 256 && fwd && x1_wide()) ? 256 : 128; }

// grid: 2 blocks per CU, a multiple of 8 * S (every XCD holds whole walkers), at least one walker per XCD
int x1_grid(int S, int64_t tiles) {
  const int unit = 8 * S;
  int g = (2 * x1_cus()) / unit * unit;
  if (g < unit) g = unit;
  const int64_t need = (tiles + 7) / 8 * 8 * S;  // no more walkers than tiles (rounded up to whole XCD rows)
  if ((int64_t)g > need) g = (int)((need + unit - 1) / unit * unit);
  return g;
}

void x1_check(int64_t M, int C, int N, const char* what) {
  if (!conv1x1x_supported(C, N))
    pdt_hip_fail(what, hipErrorInvalidValue, __FILE__, __LINE__);
  if (M * N >= (int64_t(1) << 30) || M * C >= (int64_t(1) << 30))
    pdt_hip_fail("conv1x1x: operands exceed 32-bit buffer offsets", hipErrorInvalidValue, __FILE__, __LINE__);
}
}  // namespace

int conv1x1x_mode(int set) {
  // PDT_CONV1X1X=0: the generic implicit-GEMM kernels for these shapes (A/B); set >= 0 switches at run time (tests)
  static int on = [] {
    const char* e = getenv("PDT_CONV1X1X");
    return e && e[0] == '0' ? 0 : 1;
  }();
  const int prev = on;
  if (set >= 0) on = set;
  return prev;
}

bool x1_n_ok(int C, int N);

bool conv1x1x_supported(int C, int N) {
  if (!conv1x1x_mode(-1) || !(C == 128 || C == 256 || C == 512) || N <= 0) return false;
  return x1_n_ok(C, N);
}

// the backward-data kernel also takes C = 64 (ResNet-50 layer1's conv1 backward-data; the binding prefers it over
// conv1x1_c64_bnb when conv1x1x_l1_mode(1) is set)
bool conv1x1x_bnb_supported(int C, int N) {
  if (!conv1x1x_mode(-1) || !(C == 64 || C == 128 || C == 256 || C == 512) || N <= 0) return false;
  return x1_n_ok(C, N);
}

bool x1_n_ok(int C, int N) {
  const int ns = x1_slice(C, false);  // (the narrower slice: N must suit both kernels)
  return N % ns == 0 && N / ns <= 32;
}

int conv1x1x_l1_mode(int set) {
  static int on = 0;  // (settable for tests / A/B through the binding)
  const int prev = on;
  if (set >= 0) on = set;
  return prev;
}
bool conv1x1x_prefer_l1() { return conv1x1x_l1_mode(-1) != 0; }

void conv1x1x_launch(const uint16_t* x, const uint16_t* w, uint16_t* y, double* stats, int64_t M, int C, int N,
                     int dtype, hipStream_t s, int st, int nimg, int H, int W) {
  if (M <= 0) return;
  x1_check(M, C, N, "conv1x1x: C must be 128 / 256 / 512 and N a multiple of the slice width");
  X1Geo geo{};
  int64_t x_rows = M;
  const bool sd = st > 1;
  if (sd) {
    const int P = (H - 1) / st + 1, Q = (W - 1) / st + 1;
    if ((int64_t)nimg * P * Q != M || (int64_t)nimg * H * W * C >= (int64_t(1) << 30))
      pdt_hip_fail("conv1x1x: strided geometry (M != N * P * Q, or input past 32-bit offsets)", hipErrorInvalidValue,
                   __FILE__, __LINE__);
    const FastDiv f1 = make_fastdiv((uint32_t)(P * Q)), f2 = make_fastdiv((uint32_t)Q);
    geo = X1Geo{st, H, W, P * Q, Q, f1.mul, f1.shift, f2.mul, f2.shift};
    x_rows = (int64_t)nimg * H * W;
  }
  const bool wide = C == 256 && N % 256 == 0 && x1_slice(C, true) == 256;
  const int S = N / (wide ? 256 : x1_slice(C, false));
  const int bm = C == 512 ? 32 : 64;
  const int G = x1_grid(S, (M + bm - 1) / bm);
  const int walkers = G / S;
  Scratch part(stats ? (size_t)walkers * N * 2 * sizeof(float) : 0, s);
  float* srows = part.as<float>();
  PDT_COUNT("conv1x1x");
  if (sd) PDT_COUNT("conv1x1x_strided");
#define PDT_X1(DT_, ST_, KH_, NF_, BM_, SD_)                                                                     \
  hipLaunchKernelGGL((conv1x1x_kernel<DT_, ST_, KH_, NF_, BM_, SD_>), dim3(G), dim3(256), 0, s, x, w, y, srows, M, \
                     N, S, x_rows, geo)
#define PDT_X1S(DT_, ST_, SD_)                                \
  if (C == 128) PDT_X1(DT_, ST_, 2, 4, 64, SD_);             \
  else if (wide) PDT_X1(DT_, ST_, 4, 4, 64, SD_);           \
  else if (C == 256) PDT_X1(DT_, ST_, 4, 2, 64, SD_);        \
  else PDT_X1(DT_, ST_, 8, 2, 32, SD_)
#define PDT_X1C(DT_, ST_) \
  if (sd) { PDT_X1S(DT_, ST_, true); } else { PDT_X1S(DT_, ST_, false); }
  if (dtype == kBF16) {
    if (stats) { PDT_X1C(kBF16, true); } else { PDT_X1C(kBF16, false); }
  } else {
    if (stats) { PDT_X1C(kF16, true); } else { PDT_X1C(kF16, false); }
  }
#undef PDT_X1C
#undef PDT_X1S
#undef PDT_X1
  if (stats) stat_rows_reduce_launch(srows, walkers, N * 2, stats, s);
}

void conv1x1x_bnb_launch(const uint16_t* x, const uint16_t* w, uint16_t* y, const uint16_t* res, const uint16_t* y1,
                         const float* coef1, const uint16_t* y2, const float* coef2, const uint8_t* mask,
                         double* slots, int64_t M, int C, int N, int dtype, hipStream_t s) {
  if (M <= 0) return;
  if (!conv1x1x_bnb_supported(C, N))
    pdt_hip_fail("conv1x1x_bnb: C must be 64 / 128 / 256 / 512 and N a multiple of the slice width",
                 hipErrorInvalidValue, __FILE__, __LINE__);
  if (M * N >= (int64_t(1) << 30) || M * C >= (int64_t(1) << 30))
    pdt_hip_fail("conv1x1x_bnb: operands exceed 32-bit buffer offsets", hipErrorInvalidValue, __FILE__, __LINE__);
  const int S = N / (C <= 128 && !y2 ? 256 : 128);  // the configuration's slice (PDT_XBC below)
  const int bm = C == 512 ? 32 : 64;
  const int G = x1_grid(S, (M + bm - 1) / bm);
  const int walkers = G / S;
  const int KO = y2 ? 4 : 2;
  Scratch part((size_t)walkers * N * KO * sizeof(float), s);
  float* srows = part.as<float>();
  PDT_COUNT("conv1x1x_bnb");
  if (y2) PDT_COUNT("conv1x1x_bnb_2br");
#define PDT_XB(DT_, BR_, KH_, NF_, BM_, PJ_)                                                                      \
  hipLaunchKernelGGL((conv1x1x_bnb_kernel<DT_, BR_, KH_, NF_, BM_, PJ_>), dim3(G), dim3(256), 0, s, x, w, y, res, \
                     y1, coef1, y2, coef2, mask, srows, M, N, S)
#define PDT_XBC(DT_, BR_)                                 \
  if (C == 64 && BR_ == 1) PDT_XB(DT_, BR_, 1, 4, 64, 1); \
  else if (C == 64) PDT_XB(DT_, BR_, 1, 2, 64, 2);       \
  else if (C == 128 && BR_ == 1) PDT_XB(DT_, BR_, 2, 4, 64, 1); \
  else if (C == 128) PDT_XB(DT_, BR_, 2, 2, 64, 2);      \
  else if (C == 256) PDT_XB(DT_, BR_, 4, 2, 64, 2);      \
  else PDT_XB(DT_, BR_, 8, 2, 32, 1)
  if (dtype == kBF16) {
    if (y2) { PDT_XBC(kBF16, 2); } else { PDT_XBC(kBF16, 1); }
  } else {
    if (y2) { PDT_XBC(kF16, 2); } else { PDT_XBC(kF16, 1); }
  }
#undef PDT_XBC
#undef PDT_XB
  stat_rows_reduce_launch(srows, walkers, N * KO, slots, s);
}

}  // namespace pdt
