// ob_fp.h — fp32 operations that hipcc may not contract into an fma.
//
// HIP compiles with fp-contract "fast-honor-pragmas": a * b + c written as two operations may
// become one fma, and HIP's __fmul_rn / __fadd_rn are plain `*` / `+` unless OCML rounded ops
// are enabled, so they do not prevent it. Where a fused kernel must reproduce the rounding
// sequence of the unfused torch ops it replaces (mul, then add, each rounded), these
// helpers carry `contract(off)` into the IR.
#pragma once

#include <hip/hip_runtime.h>

namespace ob {

__device__ __forceinline__ float nc_mul(float a, float b) {
#pragma clang fp contract(off)
  return a * b;
}
__device__ __forceinline__ float nc_add(float a, float b) {
#pragma clang fp contract(off)
  return a + b;
}
__device__ __forceinline__ float nc_sub(float a, float b) {
#pragma clang fp contract(off)
  return a - b;
}

}  // namespace ob
