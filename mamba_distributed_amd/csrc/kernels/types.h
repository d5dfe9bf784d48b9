// Host/device-neutral types shared by the kernels and the torch binding (no device code here).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mamba_amd {
typedef unsigned short bf16_t;  // raw bfloat16 bits
enum DType : int { kF32 = 0, kBF16 = 1, kF16 = 2 };
}  // namespace mamba_amd
