// ob_quant.h — the reference quantizer's per-element semantics, shared by every kernel.
//
// One definition of the quantizer is used by the pack, dequant and backward kernels so
// that the forward codes and the backward STE mask / alpha term can never disagree.
// Each function cites the line of onebit_asr/quant.py it restates.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ob {

// quant.py:124 — QuantizedLinear passes |alpha| + 1e-8 into the quantizer.
// 1e-8f is the fp32 rounding of the Python float 1e-8 that torch applies.
// alpha_raw: 0 = alpha as given, 1 = |alpha| + 1e-8 (quant.py:124); >= 2 = the GEMM's B
// operand is the fp32 weight itself rounded to bf16 (quant-off, tgemm.hip): no alpha scale.
__device__ __forceinline__ float effective_alpha(const float* alpha, int alpha_raw) {
  if (alpha_raw >= 2) return 1.0f;
  const float a = *alpha;
  return alpha_raw ? (fabsf(a) + 1e-8f) : a;
}

// d|alpha|/dalpha as torch's abs backward computes it (sgn, with sgn(0) = 0).
__device__ __forceinline__ float alpha_chain(const float* alpha, int alpha_raw) {
  if (!alpha_raw) return 1.0f;
  const float a = *alpha;
  return a > 0.0f ? 1.0f : (a < 0.0f ? -1.0f : 0.0f);
}

// 2-bit code of one weight. quant.py:49 Wa = W / alpha (IEEE division: hipcc's default
// fp32 division is correctly rounded, which the 0.5 threshold needs);
// quant.py:50 clamp(-1,1) never changes the sign or the <0.5 test, so it folds away;
// quant.py:52-55 bits=1: sign(), zero -> +1;
// quant.py:56-60 bits=2: |clip| < 0.5 -> 0, else sign().
// Codes: 0 -> 0, 1 -> +1, 3 -> -1.
// NaN weights (outside the reference's working range; it propagates NaN) map to 0 / +1.
__device__ __forceinline__ uint32_t quant_code(float w, float a, int bits) {
  const float wa = w / a;
  if (bits == 2) {
    if (!(fabsf(wa) >= 0.5f)) return 0u;
    return wa > 0.0f ? 1u : 3u;
  }
  return wa < 0.0f ? 3u : 1u;
}

// Code -> fp32 value of Q (exact: 0, +1, -1).
__device__ __forceinline__ float code_value(uint32_t c) {
  return __uint_as_float(((c & 1u) * 0x3F800000u) | ((c & 2u) << 30));
}

// torch.sign on fp32 (sign(0) = 0; NaN not handled, see quant_code).
__device__ __forceinline__ float tsign(float x) {
  return x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : 0.0f);
}

// quant.py:80-82 — STE indicator 1[|Wa| <= 1] as fp32.
__device__ __forceinline__ float ste_indicator(float wa) {
  return fabsf(wa) <= 1.0f ? 1.0f : 0.0f;
}

// quant.py:86-90 — dW_hat/dalpha term:
//   |Wa| < 1 : -Wa + (bits==2 ? sign(Wa)*1[|Wa|>=0.5] : sign(Wa))
//   else     : sign(Wa)
__device__ __forceinline__ float alpha_term(float wa, int bits) {
  const float awa = fabsf(wa);
  const float s = tsign(wa);
  if (awa < 1.0f) {
    const float pq = (bits == 2) ? (awa >= 0.5f ? s : 0.0f) : s;
    return -wa + pq;
  }
  return s;
}

}  // namespace ob
