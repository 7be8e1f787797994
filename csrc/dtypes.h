#pragma once
namespace pdt {
// element type codes shared by the host bindings and the kernels
enum DType : int { kBF16 = 0, kF16 = 1, kF32 = 2 };
}  // namespace pdt
