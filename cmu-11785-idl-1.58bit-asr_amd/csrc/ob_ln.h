// ob_ln.h — one LayerNorm row on 16 lanes, shared by the LayerNorm kernels (layernorm.hip)
// and the GEMM epilogues that normalise the rows they produce (tgemm.hip). Reference:
// onebit_asr/conformer.py:19-24 (nn.LayerNorm(d), eps 1e-5): biased variance, eps inside the
// square root, rstd = 1 / sqrt(var + eps); the same code on both sides, so a fused LN is
// bit-identical to the standalone kernel.
// Row mapping: 16 consecutive lanes per row; lane j holds the VW columns VW * (j + 16 i) + e of
// slot i (VW = 4: dwordx4 segments, 256 contiguous bytes per 16 lanes).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ob {
namespace lnrow {

constexpr int kLanesPerRow = 16;

// The sum over a row's 16 lanes on DPP (no LDS round trip; ds_bpermute was 4 dependent
// LDS-latency hops): quad_perm [1,0,3,2] and [2,3,0,1] pair lanes i ^ 1 and i ^ 2, then
// row_half_mirror (i <-> 7 - i) pairs each quad with the other quad of its half and
// row_mirror (i <-> 15 - i) each half with the other. Every lane of a quad / half holds the
// same partial (fp32 addition is commutative), so this is the xor tree's sum bit for bit.
template <int CTRL>
__device__ __forceinline__ float dpp_f32(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v),
                                                               CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float row_sum16(float v) {
  v += dpp_f32<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_f32<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_f32<0x141>(v);  // row_half_mirror
  v += dpp_f32<0x140>(v);  // row_mirror
  return v;
}

// VW consecutive columns of slot i of lane j: columns VW * (j + 16 i) + e, e < VW. VW = 4
// (d % 4 == 0, 16-byte aligned rows): dwordx4 loads and stores, 256 contiguous bytes per 16
// lanes; VW = 1: 64-byte segments.
template <int VW>
__device__ __forceinline__ void load_cols(const float* __restrict__ p, int c0, int d,
                                          float (&out)[VW]) {
  if constexpr (VW == 4) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    const f4 v = c0 < d ? *reinterpret_cast<const f4*>(p + c0) : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int e = 0; e < 4; ++e) out[e] = v[e];
  } else {
    out[0] = c0 < d ? p[c0] : 0.0f;
  }
}
template <int VW>
__device__ __forceinline__ void store_cols(float* __restrict__ p, int c0, const float (&v)[VW]) {
  if constexpr (VW == 4) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    *reinterpret_cast<f4*>(p + c0) = f4{v[0], v[1], v[2], v[3]};
  } else {
    p[c0] = v[0];
  }
}

template <int NPL, int VW = 1>
__device__ __forceinline__ float ln_row_v(const float (&v)[NPL][VW],
                                          const float* __restrict__ gamma,
                                          const float* __restrict__ beta, int64_t row, int d,
                                          float eps, float* __restrict__ y,
                                          float* __restrict__ mean_out,
                                          float* __restrict__ rstd_out,
                                          int8_t* __restrict__ yq = nullptr, float sx = 0.0f,
                                          float (*vout)[NPL][VW] = nullptr) {
  // no contraction: t = v - mean and var + eps stay separately rounded (as torch's LN), in
  // every kernel that includes this -- the fused LNs equal the standalone ones bit for bit
#pragma clang fp contract(off)
  const int j = threadIdx.x & (kLanesPerRow - 1);
  float s = 0.0f;
#pragma unroll
  for (int i = 0; i < NPL; ++i)
#pragma unroll
    for (int e = 0; e < VW; ++e) s += v[i][e];
  const float inv_d = 1.0f / (float)d;
  const float mean = row_sum16(s) * inv_d;
  float q = 0.0f;
#pragma unroll
  for (int i = 0; i < NPL; ++i)
#pragma unroll
    for (int e = 0; e < VW; ++e) {
      const int c = VW * (j + kLanesPerRow * i) + e;
      const float t = c < d ? v[i][e] - mean : 0.0f;
      q = fmaf(t, t, q);
    }
  const float var = row_sum16(q) * inv_d;
  const float rstd = 1.0f / sqrtf(var + eps);
  float amx = 0.0f;
#pragma unroll
  for (int i = 0; i < NPL; ++i) {
    const int c0 = VW * (j + kLanesPerRow * i);
    if (c0 < d) {
      float g[VW], b[VW], o[VW];
      if (gamma) load_cols<VW>(gamma, c0, d, g);
      if (beta) load_cols<VW>(beta, c0, d, b);
#pragma unroll
      for (int e = 0; e < VW; ++e) {
        o[e] = fmaf((v[i][e] - mean) * rstd, gamma ? g[e] : 1.0f, beta ? b[e] : 0.0f);
        amx = fmaxf(amx, fabsf(o[e]));
      }
      if (vout) {  // the normalised row for a following LN (the stored y values)
#pragma unroll
        for (int e = 0; e < VW; ++e) (*vout)[i][e] = o[e];
      }
      if (y) store_cols<VW>(y + row * d, c0, o);  // (nullptr: the absmax pass of the int8 LN)
      if (yq) {  // int8 consumer: xq = clamp(rint(y * sx), -127, 127) (tgemm_i8.hip's q4)
        uint32_t pk = 0;
#pragma unroll
        for (int e = 0; e < VW; ++e) {
          float q = rintf(o[e] * sx);
          q = fminf(fmaxf(q, -127.0f), 127.0f);
          pk |= ((uint32_t)(int)q & 0xFFu) << (8 * e);
        }
        if constexpr (VW == 4) *reinterpret_cast<uint32_t*>(yq + row * d + c0) = pk;
        else yq[row * d + c0] = (int8_t)pk;
      }
    }
  }
  if (j == 0) {
    if (mean_out) mean_out[row] = mean;
    if (rstd_out) rstd_out[row] = rstd;
  }
  return amx;
}

}  // namespace lnrow
}  // namespace ob
