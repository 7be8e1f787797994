#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pdt {

// ResNet stem forward (7x7/2, 3 -> 64 channels) over the zero-padded NHWC4 image (see stem.hip).
struct StemFwdArgs {
  const uint16_t* x;  // [N][Hp][Wp][4] zero-padded image (pad already applied)
  uint32_t x_bytes;
  const uint16_t* w;  // [64][7][32] window-row weights
  uint16_t* y;        // [N][P][Q][64]
  double* stats;      // optional [kStatSlots][64][2] fp64 (sum, sumsq) of the rounded outputs
  float* srows;       // per-block partial rows [grid][64][2] behind ``stats`` (set by the launcher)
  int N, Hp, Wp, P, Q;
  int blocks_per_cu;  // persistent grid size = CUs x blocks_per_cu (rounded to a multiple of 8)
  // filled by the launcher
  int TP, tiles;      // 4-row tiles per image, total tiles
  uint32_t tp_mul, tp_shift;
};

// Geometry the kernel handles (Q <= 112 columns, 13 padded rows of Wp pixels fit a 24 KB stage).
bool stem_fwd_supported(int Hp, int Wp, int P, int Q);
void stem_fwd_launch(StemFwdArgs a, int dtype, hipStream_t s);

}  // namespace pdt
