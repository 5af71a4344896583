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

// Fast-math helpers for the activation epilogues. HIP's __fdividef(x, y) is x / y and its
// __frcp_rn(x) is 1.0f / x: both compile to the full IEEE division sequence (v_div_scale x2,
// v_rcp, v_div_fmas, v_div_fixup and 4-5 fma) -- ~10 VALU ops per element, which made the
// swish epilogues VALU-bound. v_rcp_f32 (1 ulp) and v_exp_f32 (through __expf) instead:
//   fast_sigmoid(z) = 1 / (1 + 2^(-z log2 e)),  fast_silu(z) = z * fast_sigmoid(z).
__device__ __forceinline__ float fast_rcp(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ float fast_sigmoid(float z) { return fast_rcp(1.0f + __expf(-z)); }
__device__ __forceinline__ float fast_silu(float z) { return z * fast_sigmoid(z); }

}  // namespace ob
