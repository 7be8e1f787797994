#pragma once
#include <hip/hip_runtime.h>

#include "conv_fwd.h"

namespace pdt {

// Specialised 3x3/s1/p1, 64 -> 64 channel, 56-wide convolution (forward, or single-phase backward-data
// with flipped taps); see conv_l1.hip.  eligible() also reports whether the taps are flipped.
bool conv_l1_eligible(const ConvFwdArgs& a, int* flip);
void conv_l1_launch(const ConvFwdArgs& a, int flip, int dtype, hipStream_t s);
// 8-wave ping-pong kernel on (1) / off (0) / from PDT_CONV_L1_PP (-1, the default); returns the previous mode
int conv_l1_set_pp(int mode);

}  // namespace pdt
