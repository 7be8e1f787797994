// ResNet stem forward: 7x7 / stride 2 / pad 3 convolution, 3 -> 64 channels, as a persistent
// row-tile MFMA kernel (stem row; the stem is torchvision's conv1, instantiated by
// `dataparallel.py:112-117`).
//
// The stem's reduction is only 7 kernel rows x (8 pixels x 4 channels) = 224 long, so the generic
// implicit-GEMM kernel spends most of each block on pipeline fill and epilogue (~200 TF/s measured).
// This kernel is shaped around the stem's data reuse instead:
//   * block tile = 4 consecutive output rows of one image (wave w owns output row oh0 + w, all Q <= 112
//     columns as 7 groups of 16 pixels, all 64 output channels);
//   * the 13 padded-image rows those 4 output rows read are ONE contiguous 24 KB range of the
//     zero-padded NHWC4 image, so a tile's whole input is staged with 24 LDS-DMA instructions
//     (buffer_load ... lds) into a 2-deep LDS ring: tile i+1 streams in while tile i computes;
//   * an MFMA B fragment (8 consecutive K = 2 pixels x 4 channels of one kernel row) is one aligned
//     16-byte ds_read at column 2*ow + 2*fq of the staged row: each quarter-wave reads 256 contiguous
//     bytes (conflict-free), and the 4x overlap of neighbouring 7-wide windows costs no extra HBM/L2
//     traffic;
//   * the 64 x 224 weight matrix stays resident in LDS (rows padded to 480 B: conflict-free A reads);
//   * K = 224 exactly (no padding to a tile multiple); blocks are persistent and each XCD walks a
//     contiguous tile range;
//   * BatchNorm statistics of the rounded outputs are reduced per tile (16-lane shuffles), accumulated
//     in LDS across all of a block's tiles and reach the fp64 slot accumulators once per block.
// Weight layout ("window rows"): w[cout][r][j], j = s*4 + c (kernel column s < 7, channel c < 3; zeros
// elsewhere), i.e. [64][7][32].
#include "../common.h"
#include "conv_fwd.h"
#include "stem.h"

namespace pdt {

namespace {

constexpr int kCout = 64;
constexpr int kRows = 7;                   // kernel rows
constexpr int kWRow = kRows * 32 * 2;      // 448 B of weights per output channel
// Unpadded 448-byte weight rows; physical 16-byte chunk = logical chunk ^ ((row >> 4) & 2).  With the permuted A
// fragment rows below (fragment i, lane row fr -> weight row 16*(fr >> 2) + 4*i + (fr & 3)) the old 480-byte padded
// pitch put rows 16 apart on the same banks: every ds_read_b128 lane group was 2-way conflicted (PMC: 21.7 % of the
// kernel's LDS cycles were conflict cycles).  This layout gives every lane group 64 distinct banks (exhaustive
// check over fragments, kernel rows and the four ds_read_b128 lane groups) and 2 KB less LDS.
constexpr int kWPitch = kWRow;
PDT_DEVICE int wchunk_swz(int row) { return (row >> 4) & 2; }
constexpr int kOutRows = 4;                // output rows per tile (one per wave)
constexpr int kInRows = 2 * (kOutRows - 1) + kRows;  // 13 padded-image rows per tile
constexpr int kStage = 24 * 1024;          // LDS bytes per staged tile (>= kInRows * Wp * 8)
constexpr int kGroups = 7;                 // 16-pixel column groups per output row (Q <= 112)

}  // namespace

template <int DT, bool STATS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void stem_fwd_kernel(StemFwdArgs a) {
  using E = E16<DT>;
  typedef typename E::vec8 vec8;
  // ONE __shared__ object (a second one makes hipcc drain vmcnt(0) before every staged-tile read):
  // [2 staged tiles][resident weights][per-wave BN partials (no cross-wave LDS atomic contention)]
  __shared__ __attribute__((aligned(1024))) char smem[2 * kStage + kCout * kWPitch + 4 * kCout * 2 * 4];
  char* const wl = smem + 2 * kStage;
  float(*const red)[kCout * 2] = (float(*)[kCout * 2])(smem + 2 * kStage + kCout * kWPitch);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;

  // ---- resident weights: 1792 16-byte chunks ----
  {
    const uint4* wg = (const uint4*)a.w;
    for (int idx = tid; idx < kCout * (kWRow / 16); idx += 256) {
      const int r = idx / (kWRow / 16), c = idx - r * (kWRow / 16);
      *(uint4*)(wl + r * kWPitch + (c ^ wchunk_swz(r)) * 16) = wg[idx];
    }
    for (int i = tid; i < 4 * kCout * 2; i += 256) (&red[0][0])[i] = 0.f;
  }

  // ---- tile schedule: tile = (image n, output rows 4*k .. 4*k+3); XCD x owns a contiguous range ----
  const int G = gridDim.x;
  const int xcd = blockIdx.x & 7, lb = blockIdx.x >> 3;
  const int per_x = G >> 3;  // host launches a multiple of 8 blocks
  const int t_per = (a.tiles + 7) >> 3;
  const int t_begin = xcd * t_per;
  const int t_end = min(a.tiles, t_begin + t_per);
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(a.x, a.x_bytes);
  const FastDiv fd_tp{a.tp_mul, a.tp_shift};
  const uint32_t row_bytes = (uint32_t)a.Wp * 8u;

  auto tile_n_oh = [&](int t, int& n, int& oh0) {
    n = (int)fdiv((uint32_t)t, fd_tp);
    oh0 = (t - n * a.TP) * kOutRows;
  };
  // one tile's 13 input rows: contiguous bytes from row 2*oh0 of image n (6 wave-instructions/wave)
  auto stage_tile = [&](int t, int buf) {
    int n, oh0;
    tile_n_oh(t, n, oh0);
    const uint32_t base = (uint32_t)(n * a.Hp + 2 * oh0) * row_bytes;
#pragma unroll
    for (int i = 0; i < kStage / 4096; ++i) {
      const int chunk = (i * 4 + wave) * 1024;
      buf_lds16(rx, smem + buf * kStage + chunk, base + (uint32_t)chunk + (uint32_t)lane * 16u);
    }
  };

  int t = t_begin + lb;
  int buf = 0;
  bool stores_behind = false;  // the previous epilogue issued >= kStoresBehind stores after the DMA
  __syncthreads();             // resident weights visible to every wave
  if (t < t_end) stage_tile(t, 0);
  for (; t < t_end; t += per_x) {
    // This wave's DMA of tile t was issued before the previous epilogue's stores; vector-memory ops
    // retire in issue order, so a counted wait leaves those stores in flight.  Then a raw barrier
    // (no vmcnt(0) drain): every wave's DMA landed and every wave finished reading the other buffer.
    if (stores_behind)
      asm volatile("s_waitcnt vmcnt(14)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (t + per_x < t_end) stage_tile(t + per_x, buf ^ 1);

    f32x4_t acc[4][kGroups];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int g = 0; g < kGroups; ++g) acc[i][g] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    const char* sb = smem + buf * kStage + 2 * wave * row_bytes + (fr + fq) * 16;
    // kernel row r+1's fragments are read while row r's 28 MFMAs run (explicit register double buffer pinned by
    // scheduling barriers: read right before their MFMAs, each row's 11 LDS reads were exposed -- PMC: 63 % of the
    // wave cycles issue-stalled, 28 % MFMA busy)
    vec8 af[2][4], bf[2][kGroups];
    // A fragment i row fr = output channel (fr >> 2) * 16 + i * 4 + (fr & 3): a lane's 4 fragments x 4 rows are then
    // the 16 CONSECUTIVE channels 16 * fq .. +15 of its pixel -- two 16-byte stores per pixel instead of four 8-byte
    // ones (round 5, same box: ResNet-18 19.93/19.93/20.34 -> 19.86/19.80/20.24 ms, ResNet-50 72.67/72.64 ->
    // 72.56/72.51 ms)
    const int wswz = (fr >> 2) & 2;  // wchunk_swz of this lane's weight rows (r * 4 + fq < 28: only the low bits)
    auto load = [&](int r, int sl) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        af[sl][i] = *(const vec8*)(wl + ((fr >> 2) * 16 + i * 4 + (fr & 3)) * kWPitch + (r * 4 + (fq ^ wswz)) * 16);
#pragma unroll
      for (int g = 0; g < kGroups; ++g) bf[sl][g] = *(const vec8*)(sb + r * row_bytes + g * 256);
    };
    load(0, 0);
#pragma unroll
    for (int r = 0; r < kRows; ++r) {
      if (r + 1 < kRows) load(r + 1, (r + 1) & 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int g = 0; g < kGroups; ++g) acc[i][g] = E::mfma16x16x32(af[r & 1][i], bf[r & 1][g], acc[i][g]);
      __builtin_amdgcn_sched_barrier(0);
    }

    // ---- epilogue: lane holds couts 16*fq + 4*i + r of pixel (oh, g*16 + fr) ----
    int n, oh0;
    tile_n_oh(t, n, oh0);
    const int oh = oh0 + wave;
    stores_behind = oh < a.P && a.Q == kGroups * 16;  // then 14 stores follow the next DMA
    float csum[4][4], csq[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) { csum[i][r] = 0.f; csq[i][r] = 0.f; }
    if (oh < a.P) {
      uint16_t* yrow = a.y + ((int64_t)(n * a.P + oh) * a.Q) * kCout + 16 * fq;
#pragma unroll
      for (int g = 0; g < kGroups; ++g) {
        const int ow = g * 16 + fr;
        if (ow < a.Q) {
#pragma unroll
          for (int h = 0; h < 2; ++h) {  // channels 16*fq + 8h .. +7 = fragments 2h, 2h+1
            uint4 pk;  // one v_cvt_pk_bf16_f32 per pair (E16::pack2)
            pk.x = E::pack2(acc[2 * h][g][0], acc[2 * h][g][1]);
            pk.y = E::pack2(acc[2 * h][g][2], acc[2 * h][g][3]);
            pk.z = E::pack2(acc[2 * h + 1][g][0], acc[2 * h + 1][g][1]);
            pk.w = E::pack2(acc[2 * h + 1][g][2], acc[2 * h + 1][g][3]);
            uint16_t o[8];
            unpack8(pk, o);
            *(uint4*)(yrow + (int64_t)ow * kCout + 8 * h) = pk;
            if constexpr (STATS) {
#pragma unroll
              for (int e = 0; e < 8; ++e) {
                const float q = E::to_f(o[e]);
                csum[2 * h + (e >> 2)][e & 3] += q;
                csq[2 * h + (e >> 2)][e & 3] += q * q;
              }
            }
          }
        }
      }
    }
    if constexpr (STATS) {
      // per-tile channel partials: reduce over the 16 pixel lanes (DPP row scan, no LDS traffic),
      // accumulate in LDS (fp32) per wave
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          csum[i][r] = row16_sum(csum[i][r]);
          csq[i][r] = row16_sum(csq[i][r]);
        }
      if (fr == 15) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int c = 16 * fq + 4 * i + r;
            red[wave][c * 2 + 0] += csum[i][r];  // lanes fr == 15 of distinct fq own distinct c
            red[wave][c * 2 + 1] += csq[i][r];
          }
      }
    }
    buf ^= 1;
  }

  if constexpr (STATS) {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid < kCout * 2)  // this block's own partial row (deterministic statistics, conv_fwd.h)
      a.srows[(int64_t)blockIdx.x * kCout * 2 + tid] = red[0][tid] + red[1][tid] + red[2][tid] + red[3][tid];
  }
}

bool stem_fwd_supported(int Hp, int Wp, int P, int Q) {
  return Q <= kGroups * 16 && kInRows * Wp * 8 <= kStage && 2 * (Q - 1) + 8 <= Wp && 2 * (P - 1) + kRows <= Hp;
}

void stem_fwd_launch(StemFwdArgs a, int dtype, hipStream_t s) {
  PDT_COUNT("stem_fwd");
  a.TP = (a.P + kOutRows - 1) / kOutRows;
  a.tiles = a.N * a.TP;
  const FastDiv f = make_fastdiv((uint32_t)a.TP);
  a.tp_mul = f.mul; a.tp_shift = f.shift;
  if (a.tiles == 0) return;
  int dev = 0, cus = 256;
  PDT_HIP_CHECK(hipGetDevice(&dev));
  PDT_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  int G = cus * a.blocks_per_cu;
  const int cap = (a.tiles + 7) / 8 * 8;
  if (G > cap) G = cap;
  G = (G + 7) / 8 * 8;
  const bool st = a.stats != nullptr;
  Scratch part(st ? (size_t)G * kCout * 2 * sizeof(float) : 0, s);
  a.srows = part.as<float>();
#define PDT_STEM(DT_, ST_) hipLaunchKernelGGL((stem_fwd_kernel<DT_, ST_>), dim3(G), dim3(256), 0, s, a)
  if (dtype == kBF16) {
    if (st) PDT_STEM(kBF16, true); else PDT_STEM(kBF16, false);
  } else {
    if (st) PDT_STEM(kF16, true); else PDT_STEM(kF16, false);
  }
#undef PDT_STEM
  if (st) stat_rows_reduce_launch(a.srows, G, kCout * 2, a.stats, s);
}

}  // namespace pdt
