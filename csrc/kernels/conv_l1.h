#pragma once
#include <hip/hip_runtime.h>

#include "conv_fwd.h"

namespace pdt {

// Specialised 3x3/s1/p1, 64 -> 64 channel, 56-wide convolution (forward, or single-phase backward-data
// with flipped taps); see conv_l1.hip.  eligible() also reports whether the taps are flipped.
bool conv_l1_eligible(const ConvFwdArgs& a, int* flip);
void conv_l1_launch(const ConvFwdArgs& a, int flip, int dtype, hipStream_t s);

}  // namespace pdt
