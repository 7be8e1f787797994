#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pdt {

// 1x1 / stride-1 convolution with 64 input and 256 output channels (ResNet-50 layer1's expanding conv3 and its
// downsample): y[m][k] = sum_c x[m][c] * w[k][c] over M pixels, optional BN statistics of the rounded outputs into
// fp64 slots (conv_fwd.h).  See conv1x1.hip.
bool conv1x1_c64_supported(int C, int Kout);
void conv1x1_c64_launch(const uint16_t* x, const uint16_t* w, uint16_t* y, double* stats, int64_t M, int dtype,
                        hipStream_t s);

}  // namespace pdt
