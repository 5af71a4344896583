// tgemm_va.hip — the ternary BitLinear forward as a VALU sign-accumulate (north_star's first
// inner-product option), kept beside the bf16x3-MFMA kernel (tgemm.hip) for the A/B the
// north star asks for: "the inner product taken either as a wavefront sign-accumulate
// reduction or as int8 MFMA ... the winner evidenced by rocprof HBM GB/s and MFMA-busy".
//
//   Y[M][N] = a * sum_k X[m][k] * Q[n][k] + b[n]       (quant.py:126, F.linear of a*Q)
//
// Q in {-1, 0, +1}: x * q is exact in fp32, so every fma below is an exact signed add of x
// (or of 0) into the accumulator, rounded once -- the sign-accumulate, on packed fp32 FMA
// (v_pk_fma_f32: two columns per instruction) instead of a select + add pair. Summation runs
// in k order per output (one fp32 chain), so results differ from the MFMA kernel's by
// summation order only (tests/test_bitlinear_gpu.py: the same 1e-5 bar vs float64).
//
// Block = 256 threads, a 64 x 64 output tile, k in chunks of 32: the X chunk is staged
// transposed ([k][row]) and the code words decoded to fp32 Q ([k][col]) in LDS; thread
// (tr, tc) holds rows 4tr..4tr+3 x columns 4tc..4tc+3 (16 accumulators) and per k reads one
// dwordx4 of each (ds_read_b128) for 16 FMAs (8 packed). Not on the product path: the bf16x3
// MFMA kernel is faster (DESIGN.md "Inner product A/B").
#include "ob_launch.h"
#include "ob_quant.h"

namespace ob {

namespace {

typedef float f32x4v __attribute__((ext_vector_type(4)));
typedef float f32x2v __attribute__((ext_vector_type(2)));

constexpr int kVaTile = 64, kVaK = 32, kVaPitch = kVaTile + 4;

__global__ __launch_bounds__(256, 2) void tgemm_signacc_kernel(
    const float* __restrict__ A, int64_t M, int K, const uint32_t* __restrict__ codes, int KW,
    int N, const float* __restrict__ alpha, int alpha_raw, const float* __restrict__ bias,
    float* __restrict__ C) {
  __shared__ __attribute__((aligned(16))) float xs[kVaK][kVaPitch];
  __shared__ __attribute__((aligned(16))) float qs[kVaK][kVaPitch];
  const int t = threadIdx.x;
  const int n0 = blockIdx.x * kVaTile;
  const int64_t m0 = (int64_t)blockIdx.y * kVaTile;
  const int tr = t >> 4, tc = t & 15;
  f32x2v acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i][0] = acc[i][1] = f32x2v{0.f, 0.f};
  // loader roles: X -- float4 (row lr + 32 h, k 4 lk .. +3); codes -- thread < 128: column
  // t / 2, word t % 2 of the chunk (16 k each)
  const int lr = t >> 3, lk = 4 * (t & 7);
  for (int k0 = 0; k0 < K; k0 += kVaK) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int64_t row = m0 + lr + 32 * h;
      f32x4v v = f32x4v{0.f, 0.f, 0.f, 0.f};
      if (row < M && k0 + lk < K) v = *reinterpret_cast<const f32x4v*>(A + row * K + k0 + lk);
#pragma unroll
      for (int e = 0; e < 4; ++e) xs[lk + e][lr + 32 * h] = v[e];
    }
    if (t < 2 * kVaTile) {
      const int col = t >> 1, wd = t & 1;
      const int wi = (k0 >> 4) + wd;
      const uint32_t word = (n0 + col < N && wi < KW) ? codes[(int64_t)(n0 + col) * KW + wi] : 0u;
#pragma unroll
      for (int e = 0; e < 16; ++e) qs[16 * wd + e][col] = code_value((word >> (2 * e)) & 3u);
    }
    __syncthreads();
#pragma unroll 8
    for (int k = 0; k < kVaK; ++k) {
      const f32x4v xv = *reinterpret_cast<const f32x4v*>(&xs[k][4 * tr]);
      const f32x4v qv = *reinterpret_cast<const f32x4v*>(&qs[k][4 * tc]);
      const f32x2v q01 = f32x2v{qv[0], qv[1]}, q23 = f32x2v{qv[2], qv[3]};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const f32x2v xx = f32x2v{xv[i], xv[i]};
        acc[i][0] = __builtin_elementwise_fma(xx, q01, acc[i][0]);
        acc[i][1] = __builtin_elementwise_fma(xx, q23, acc[i][1]);
      }
    }
    __syncthreads();
  }
  const float a = effective_alpha(alpha, alpha_raw);
  const int c0 = n0 + 4 * tc;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t row = m0 + 4 * tr + i;
    if (row >= M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = c0 + j;
      if (col < N) {
        const float s = acc[i][j >> 1][j & 1];
        C[row * N + col] = fmaf(a, s, bias ? bias[col] : 0.0f);
      }
    }
  }
}

}  // namespace

bool launch_ternary_gemm_signacc(const float* A, int64_t M, int64_t K, const uint32_t* codes,
                                 int64_t N, const float* alpha, int alpha_raw, const float* bias,
                                 float* C, hipStream_t s) {
  if (K % 4 != 0 || M > ((int64_t)kVaTile << 30) || N > (1 << 24) || K > (1 << 24)) return false;
  if (M == 0 || N == 0) return true;
  const int KW = (int)((K + 15) / 16);
  const dim3 grid((unsigned)((N + kVaTile - 1) / kVaTile), (unsigned)((M + kVaTile - 1) / kVaTile));
  hipLaunchKernelGGL(tgemm_signacc_kernel, grid, dim3(256), 0, s, A, M, (int)K, codes, KW, (int)N,
                     alpha, alpha_raw, bias, C);
  return true;
}

}  // namespace ob
