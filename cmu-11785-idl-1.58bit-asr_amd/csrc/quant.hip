// quant.hip — weight quantizer kernels: pack (forward codes), dequant (quantize_weight
// forward) and the STE split-reduction finish (quantize_weight / BitLinear backward).
//
// Reference: onebit_asr/quant.py:44-92 (_QuantizeSTE.forward / .backward).
// All of these touch only the [N][K] weight-shaped tensors (<= 83k elements at
// Conformer-S), so they are launch-bound, not bandwidth-bound; they are written to be
// one launch each, deterministic and capture-safe.
#include "ob_launch.h"
#include "ob_quant.h"

namespace ob {

namespace {

constexpr int kThreads = 256;

// One thread per output word. Words [0, N*KW) are codes (row n, word w: K-contiguous);
// words [N*KW, N*KW + K*NW) are codes_t, indexed w-major / k-minor so that consecutive
// threads read consecutive W columns (coalesced) while building a transposed word.
__global__ __launch_bounds__(kThreads) void quant_pack_kernel(
    const float* __restrict__ W, const float* __restrict__ alpha, int alpha_raw, int bits,
    int64_t N, int64_t K, int64_t KW, int64_t NW, uint32_t* __restrict__ codes,
    uint32_t* __restrict__ codes_t) {
  const float a = effective_alpha(alpha, alpha_raw);
  int64_t t = blockIdx.x * (int64_t)kThreads + threadIdx.x;
  const int64_t n_codes = codes ? N * KW : 0;
  const int64_t n_codes_t = codes_t ? K * NW : 0;
  if (t < n_codes) {
    const int64_t n = t / KW;
    const int64_t w = t - n * KW;
    const float* row = W + n * K;
    uint32_t word = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int64_t k = 16 * w + j;
      if (k < K) word |= quant_code(row[k], a, bits) << (2 * j);
    }
    codes[n * KW + w] = word;
    return;
  }
  t -= n_codes;
  if (t < n_codes_t) {
    const int64_t w = t / K;
    const int64_t k = t - w * K;
    uint32_t word = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int64_t n = 16 * w + j;
      if (n < N) word |= quant_code(W[n * K + k], a, bits) << (2 * j);
    }
    codes_t[k * NW + w] = word;
  }
}

// quant.py:68 W_hat = alpha * Q, elementwise, grid-stride.
__global__ __launch_bounds__(kThreads) void quant_dequant_kernel(const float* __restrict__ W,
                                                                 const float* __restrict__ alpha,
                                                                 int alpha_raw, int bits,
                                                                 int64_t n,
                                                                 float* __restrict__ W_hat) {
  const float a = effective_alpha(alpha, alpha_raw);
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  for (int64_t i = blockIdx.x * (int64_t)kThreads + threadIdx.x; i < n; i += stride) {
    W_hat[i] = a * code_value(quant_code(W[i], a, bits));
  }
}

// Deterministic block sum: fixed xor-butterfly inside each wave, then wave 0 adds the
// four wave sums in wave order.
__device__ __forceinline__ float block_sum(float v, float* lds4) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) lds4[wave] = v;
  __syncthreads();
  float t = 0.0f;
  if (threadIdx.x == 0) {
#pragma unroll
    for (int i = 0; i < kThreads / 64; ++i) t += lds4[i];
  }
  return t;  // valid in thread 0 only
}

// quant.py:80-91 applied to the fixed-order sum of `chunks` partial slabs.
// Block = 64 elements x 4 chunk groups: group q sums chunks q, q+4, q+8, ... (independent,
// coalesced loads), the 4 group sums are added in group order through LDS, then wave 0
// applies the STE mask / alpha term and reduces its alpha partial. Deterministic.
constexpr int kReduceElems = 64;

__global__ __launch_bounds__(kThreads) void ste_reduce_kernel(
    const float* __restrict__ part, int chunks, int64_t nk, const float* __restrict__ part_db,
    int64_t n_db, const float* __restrict__ W, const float* __restrict__ alpha, int alpha_raw,
    int bits, float* __restrict__ dW, float* __restrict__ db, float* __restrict__ apart) {
  __shared__ float grp_sum[4][kReduceElems];
  const int lane = threadIdx.x & 63;
  const int grp = threadIdx.x >> 6;
  const int64_t e = blockIdx.x * (int64_t)kReduceElems + lane;
  const bool is_w = e < nk;
  const bool is_b = !is_w && e < nk + n_db;
  const float* src = is_w ? part + e : (is_b ? part_db + (e - nk) : nullptr);
  const int64_t stride = is_w ? nk : n_db;
  float s = 0.0f;
  if (src) {
    int c = grp;
    for (; c + 12 < chunks; c += 16) {
      const float v0 = src[(int64_t)c * stride];
      const float v1 = src[(int64_t)(c + 4) * stride];
      const float v2 = src[(int64_t)(c + 8) * stride];
      const float v3 = src[(int64_t)(c + 12) * stride];
      s += v0;
      s += v1;
      s += v2;
      s += v3;
    }
    for (; c < chunks; c += 4) s += src[(int64_t)c * stride];
  }
  grp_sum[grp][lane] = s;
  __syncthreads();
  if (grp != 0) return;
  const float g = ((grp_sum[0][lane] + grp_sum[1][lane]) + grp_sum[2][lane]) + grp_sum[3][lane];
  float prod = 0.0f;
  if (is_w) {
    const float a = effective_alpha(alpha, alpha_raw);
    const float wa = W[e] / a;
    dW[e] = g * ste_indicator(wa);  // quant.py:81-82 (multiply: inf*0 -> NaN as in torch)
    prod = g * alpha_term(wa, bits);  // quant.py:91 grad_out * term
  } else if (is_b) {
    db[e - nk] = g;
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) prod += __shfl_xor(prod, off, 64);
  if (lane == 0) apart[blockIdx.x] = prod;
}

// quant.py:91 .sum() finished over the block partials, then the abs() chain of
// quant.py:124 (torch abs backward multiplies by sgn(alpha)).
__global__ __launch_bounds__(kThreads) void ste_finalize_kernel(const float* __restrict__ apart,
                                                                int64_t nb,
                                                                const float* __restrict__ alpha,
                                                                int alpha_raw,
                                                                float* __restrict__ dalpha) {
  __shared__ float lds4[kThreads / 64];
  float s = 0.0f;
  for (int64_t i = threadIdx.x; i < nb; i += kThreads) s += apart[i];
  const float t = block_sum(s, lds4);
  if (threadIdx.x == 0) dalpha[0] = t * alpha_chain(alpha, alpha_raw);
}

}  // namespace

void launch_quant_pack(const float* W, const float* alpha, int alpha_raw, int bits, int64_t N,
                       int64_t K, uint32_t* codes, uint32_t* codes_t, hipStream_t s) {
  const int64_t KW = ceil_div(K, 16), NW = ceil_div(N, 16);
  const int64_t total = (codes ? N * KW : 0) + (codes_t ? K * NW : 0);
  if (total == 0) return;
  const int64_t blocks = ceil_div(total, kThreads);
  hipLaunchKernelGGL(quant_pack_kernel, dim3((unsigned)blocks), dim3(kThreads), 0, s, W, alpha,
                     alpha_raw, bits, N, K, KW, NW, codes, codes_t);
}

void launch_quant_dequant(const float* W, const float* alpha, int alpha_raw, int bits, int64_t n,
                          float* W_hat, hipStream_t s) {
  if (n == 0) return;
  int64_t blocks = ceil_div(n, kThreads);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(quant_dequant_kernel, dim3((unsigned)blocks), dim3(kThreads), 0, s, W,
                     alpha, alpha_raw, bits, n, W_hat);
}

int64_t ste_reduce_blocks(int64_t total) { return ceil_div(total, kReduceElems); }

void launch_ste_reduce(const float* part, int chunks, int64_t nk, const float* part_db,
                       int64_t n_db, const float* W, const float* alpha, int alpha_raw, int bits,
                       float* dW, float* db, float* apart, float* dalpha, hipStream_t s) {
  const int64_t nb = ste_reduce_blocks(nk + n_db);
  if (nb > 0) {
    hipLaunchKernelGGL(ste_reduce_kernel, dim3((unsigned)nb), dim3(kThreads), 0, s, part, chunks,
                       nk, part_db, n_db, W, alpha, alpha_raw, bits, dW, db, apart);
  }
  hipLaunchKernelGGL(ste_finalize_kernel, dim3(1), dim3(kThreads), 0, s, apart, nb, alpha,
                     alpha_raw, dalpha);
}

}  // namespace ob
