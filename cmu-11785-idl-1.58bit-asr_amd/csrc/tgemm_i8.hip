// tgemm_i8.hip — the north-star int8 path of BitLinear: per-tensor absmax int8 activations
// times ternary weights on the int8 matrix cores (v_mfma_i32_16x16x64_i8).
//
// The reference keeps activations fp32 (quant.py:126 F.linear(x, W_hat, b); SURVEY.md §0
// F3), so this is an OPT-IN mode (QuantizedLinear.act_quant = "absmax_int8"), used by the
// inference path and available to training. Its semantics (BitNet b1.58 activation
// quantizer, restated bit-exactly by oracle/quant_oracle.py::np_bitlinear_fwd_i8):
//
//   g   = max(max|X_p|, 1e-5)           per pass p (the tensor one reference call sees)
//   sx  = 127 / g                        fp32, correctly rounded
//   xq  = clamp(rint(x * sx), -127, 127) int8 (rint: round half to even, like torch.round)
//   acc = sum_k xq[m][k] * Q[n][k]       int32, exact (|acc| <= 127*K < 2^24)
//   y   = float(acc) * (a * (g / 127)) + b      two roundings (mul, then add), no fma
//
// so the GPU result is bit-identical to a numpy float32 restatement. Q is the same 2-bit
// code set as the fp32 path (bits 1 / 2, a = |alpha| + 1e-8).
//
// Kernel layout (block = 4 waves, 64 rows x 16*NT columns, persistent over row tiles like
// tgemm.hip): the block decodes its code rows into an int8 image of Q in LDS
// ([16*NT][64*NCH + 16] bytes, sign-extended codes); per 64-wide k chunk a lane loads 16
// consecutive fp32 of its row (4 x dwordx4), quantizes them in registers into one
// 16-byte fragment and issues one i8 MFMA per 16-column tile. A and B fragments take
// element j of lane (r, g) from k = 64c + 16g + j; any k permutation the hardware applies
// is the same for both operands, so the sum over k is unaffected.
#include "ob_fp.h"
#include "ob_launch.h"
#include "ob_quant.h"

namespace ob {

namespace {

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kThreads = 256;
constexpr int kRows = 64;
constexpr int kTargetBlocks = 512;
constexpr size_t kMaxLds = 64 * 1024;

__device__ __forceinline__ int xcd_logical(int b, int nb) {
  const int q = nb / 8, r = nb % 8, x = b % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

// 16 codes of one word -> 16 sign-extended int8 bytes (0 -> 0, 1 -> +1, 3 -> -1).
__device__ __forceinline__ u32x4 decode_i8(uint32_t word) {
  u32x4 out;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t v = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int j = 4 * q + e;
      const int c = (int)(word << (30 - 2 * j)) >> 30;  // two's-complement 2-bit field
      v |= ((uint32_t)c & 0xFFu) << (8 * e);
    }
    out[q] = v;
  }
  return out;
}

__device__ __forceinline__ uint32_t q4(const f32x4& x, float sx) {
  uint32_t v = 0;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float q = rintf(x[e] * sx);
    q = fminf(fmaxf(q, -127.0f), 127.0f);
    v |= ((uint32_t)(int)q & 0xFFu) << (8 * e);
  }
  return v;
}

// y = float(acc) * osc + b with two roundings: hipcc contracts a*b+c into an fma by
// default (-ffp-contract=fast), which would round once and differ from the restatement.
__device__ __forceinline__ float epilogue(int acc, float osc, float b) {
#pragma clang fp contract(off)
  const float p = (float)acc * osc;
  return p + b;
}

__device__ __forceinline__ float act_gamma(const float* amax, int p) {
  return fmaxf(amax[p], 1e-5f);
}

// Per-pass max|x|, two launches without atomics: kAbsParts blocks per pass each write the
// max of their slice (|x| >= 0, so comparing the fp32 bit patterns as unsigned is the
// float order), then one wave per pass reduces the partials. Max is order-independent,
// hence deterministic. (A single-address atomicMax from every wave serialised at the L2:
// 53 us for a 37 MB tensor, measured.)
constexpr int kAbsParts = 256;

__global__ __launch_bounds__(kThreads) void act_absmax_part_kernel(const float* __restrict__ X,
                                                                   int64_t n_per_pass,
                                                                   uint32_t* __restrict__ part) {
  __shared__ uint32_t red[kThreads / 64];
  const int p = blockIdx.y;
  const float* x = X + (int64_t)p * n_per_pass;
  const int64_t n4 = n_per_pass >> 2;
  uint32_t m0 = 0, m1 = 0;
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  for (; i + stride < n4; i += 2 * stride) {  // two loads in flight per thread
    const f32x4 a = reinterpret_cast<const f32x4*>(x)[i];
    const f32x4 b = reinterpret_cast<const f32x4*>(x)[i + stride];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      m0 = max(m0, __float_as_uint(a[e]) & 0x7FFFFFFFu);
      m1 = max(m1, __float_as_uint(b[e]) & 0x7FFFFFFFu);
    }
  }
  for (; i < n4; i += stride) {
    const f32x4 a = reinterpret_cast<const f32x4*>(x)[i];
#pragma unroll
    for (int e = 0; e < 4; ++e) m0 = max(m0, __float_as_uint(a[e]) & 0x7FFFFFFFu);
  }
  for (int64_t t = 4 * n4 + (int64_t)blockIdx.x * kThreads + threadIdx.x; t < n_per_pass;
       t += stride)
    m0 = max(m0, __float_as_uint(x[t]) & 0x7FFFFFFFu);
  uint32_t m = max(m0, m1);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0)
    part[(int64_t)p * gridDim.x + blockIdx.x] = max(max(red[0], red[1]), max(red[2], red[3]));
}

__global__ __launch_bounds__(64) void act_absmax_final_kernel(const uint32_t* __restrict__ part,
                                                              int nparts,
                                                              uint32_t* __restrict__ amax) {
  const int p = blockIdx.x;
  uint32_t m = 0;
  for (int i = threadIdx.x; i < nparts; i += 64) m = max(m, part[(int64_t)p * nparts + i]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o));
  if (threadIdx.x == 0) amax[p] = m;
}

// X_deq = xq * (g / 127): the activation the int8 forward actually multiplied (the
// backward's dW = dY^T X_deq under the straight-through estimator).
__global__ __launch_bounds__(kThreads) void act_dequant_kernel(const float* __restrict__ X,
                                                               int64_t n_per_pass,
                                                               const float* __restrict__ amax,
                                                               float* __restrict__ Xd) {
  const int p = blockIdx.y;
  const float g = act_gamma(amax, p);
  const float sx = 127.0f / g;
  const float ds = g / 127.0f;
  const float* x = X + (int64_t)p * n_per_pass;
  float* y = Xd + (int64_t)p * n_per_pass;
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n_per_pass; i += stride) {
    float q = rintf(x[i] * sx);
    q = fminf(fmaxf(q, -127.0f), 127.0f);
    y[i] = q * ds;
  }
}

// Fused epilogues of the inference call sites (the fp32 path's are in tgemm.hip):
//   I8_SWISH     C = silu(y) and the per-pass max|C| into amax_out (the int8 scale of the
//                next BitLinear, ff.lin2: conformer.py:36-45 at dropout 0);
//   I8_RESIDUAL  C = R + rscale * (row valid ? y : 0*y)  (ff.lin2 / mhsa.out_proj + x).
// Stores go row-coalesced through a per-wave LDS staging tile, as in tgemm.hip.
//   I8_SWISH_AMAX  only the per-pass max|silu(y)| (no store): the first of the two
//                launches that give ff.lin2 an int8 operand in HBM;
//   I8_SWISH_Q     the second: C8 = clamp(rint(silu(y) * 127 / max(amax_out[p], 1e-5)))
//                as int8 -- the same values and scale the in-register quantisation of
//                an fp32 silu(y) operand would produce, so ff.lin2 is bit-identical.
constexpr int kI8Plain = 0, kI8Swish = 1, kI8Residual = 2, kI8SwishAmax = 3, kI8SwishQ = 4;
struct I8Epi {
  const float* R;
  float rscale;
  const int* lens;
  int T;
  uint32_t* amax_out;
};

// silu(z) = z / (1 + exp(-z)) through v_exp_f32 and v_rcp_f32 (ob_fp.h fast_silu): the
// accurate expf + IEEE division cost ~40 VALU ops per element, which made the swish launches
// VALU-bound (ff.lin1's two int8-output launches 47 + 51 us at B = 256). Every int8 swish
// epilogue uses this one formula, so the fp32-operand and int8-operand paths agree bit for
// bit; against torch's silu it differs by a few ulp (the module path's int8 image of the FFN
// hidden can differ by one step where a value sits on a rounding boundary --
// tests/test_i8_fused_gpu.py bounds that).
__device__ __forceinline__ float silu_fast(float z) { return fast_silu(z); }

__host__ __device__ inline size_t i8_stage_off(int nt, int nch) {
  return (((size_t)(16 * nt) * (size_t)(64 * nch + 16)) + 15) & ~(size_t)15;
}
__host__ __device__ inline size_t i8_stage_bytes(int nt) {
  const int cw = nt < 4 ? nt : 4;
  return (size_t)4 * 16 * (16 * cw + 4) * sizeof(float);
}

// AI8: A is the int8 image of the activation ([M][K] bytes, quantised by its producer at
// the pass's scale 127 / max(amax[p], 1e-5)); else fp32, quantised here in registers.
// C is fp32 [M][N], or int8 for I8_SWISH_Q (C8).
template <int NT, int NCH, int EPI, bool AI8>
__global__ __launch_bounds__(kThreads) void tgemm_i8_kernel(
    const void* __restrict__ Av, int64_t M, int K, const uint32_t* __restrict__ codes, int KW,
    int N, int n_ct, int n_rt, int rgroups, const float* __restrict__ alpha, int alpha_raw,
    const float* __restrict__ amax, const float* __restrict__ bias, void* __restrict__ Cv,
    const uint32_t* __restrict__ codes1, const int* __restrict__ pass_bits, I8Epi ep) {
  const int64_t rowbase = pass_bits ? (int64_t)blockIdx.y * M : 0;
  const float* A = static_cast<const float*>(Av);
  const int8_t* A8 = static_cast<const int8_t*>(Av);
  float* C = static_cast<float*>(Cv);
  int8_t* C8 = static_cast<int8_t*>(Cv);
  int p = 0;
  if (pass_bits) {
    p = blockIdx.y;
    if (pass_bits[p] == 1) codes = codes1;
    A += (int64_t)p * M * K;
    A8 += (int64_t)p * M * K;
    C += (int64_t)p * M * N;
    C8 += (int64_t)p * M * N;
  }
  (void)rowbase;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int kpad = 64 * NCH;
  constexpr int stride = kpad + 16;  // bytes per image row
  constexpr int kwp = kpad / 16;     // code words per padded row

  const int L = xcd_logical(blockIdx.x, gridDim.x);
  const int ct = L % n_ct;
  const int rg = L / n_ct;
  const int n0 = ct * (16 * NT);

  constexpr int nwords = 16 * NT * kwp;
  for (int idx = threadIdx.x; idx < nwords; idx += kThreads) {
    const int nl = idx / kwp, w = idx - nl * kwp;
    const int n = n0 + nl;
    const uint32_t word = (n < N && w < KW) ? codes[(int64_t)n * KW + w] : 0u;
    *reinterpret_cast<u32x4*>(smem + nl * stride + 16 * w) = decode_i8(word);
  }
  __syncthreads();

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int r = lane & 15;
  const int g = lane >> 4;
  const char* brow = smem + r * stride + 16 * g;
  const float gam = act_gamma(amax, p);
  const float sx = 127.0f / gam;
  const float osc = __fmul_rn(effective_alpha(alpha, alpha_raw), gam / 127.0f);
  // I8_SWISH_Q: the output's int8 scale (amax_out holds the max of the I8_SWISH_AMAX launch)
  const float sx_out =
      EPI == kI8SwishQ ? 127.0f / fmaxf(__uint_as_float(ep.amax_out[p]), 1e-5f) : 0.0f;
  float bcol[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int col = n0 + 16 * t + r;
    bcol[t] = (bias && col < N) ? bias[col] : 0.0f;
  }
  float amx = 0.0f;  // I8_SWISH: this lane's max|C|

  for (int rt = rg; rt < n_rt; rt += rgroups) {
    const int64_t m0 = (int64_t)rt * kRows + wave * 16;
    const int64_t row = m0 + r < M ? m0 + r : M - 1;
    const float* arow = A + row * (int64_t)K;
    const int8_t* arow8 = A8 + row * (int64_t)K;
    i32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = i32x4{0, 0, 0, 0};

    // the chunk's 16 floats: clamped start (k >= K meets zero codes, K % 16 == 0)
    auto load16 = [&](int c, f32x4* v) {
      int k = 64 * c + 16 * g;
      k = k < K ? k : K - 16;
      const f32x4* src = reinterpret_cast<const f32x4*>(arow + k);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = src[e];
    };
    if constexpr (AI8) {
      // the chunk's 16 int8 of the row: one dwordx4 (all chunks of the row in flight)
      i32x4 qa[NCH];
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        int k = 64 * c + 16 * g;
        k = k < K ? k : K - 16;
        qa[c] = *reinterpret_cast<const i32x4*>(arow8 + k);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        i32x4 bq[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t)
          bq[t] = *reinterpret_cast<const i32x4*>(brow + t * 16 * stride + 64 * c);
#pragma unroll
        for (int t = 0; t < NT; ++t)
          acc[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(qa[c], bq[t], acc[t], 0, 0, 0);
      }
    } else {
      constexpr int kWin = NCH < 3 ? NCH : 3;
      f32x4 buf[NCH][4];
#pragma unroll
      for (int c = 0; c < kWin; ++c) load16(c, buf[c]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        if (c + kWin < NCH) load16(c + kWin, buf[c + kWin]);
        __builtin_amdgcn_sched_barrier(0);
        i32x4 bq[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t)
          bq[t] = *reinterpret_cast<const i32x4*>(brow + t * 16 * stride + 64 * c);
        i32x4 a;
#pragma unroll
        for (int e = 0; e < 4; ++e) a[e] = (int)q4(buf[c][e], sx);
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, bq[t], acc[t], 0, 0, 0);
      }
    }

    if constexpr (EPI == kI8Plain) {
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int col = n0 + 16 * t + r;
        if (col >= N) continue;
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
          const int64_t orow = m0 + 4 * g + reg;
          if (orow < M) C[orow * N + col] = epilogue(acc[t][reg], osc, bcol[t]);
        }
      }
    } else if constexpr (EPI == kI8SwishAmax) {
      // max only: fast_silu is non-decreasing on y >= 0 (v_exp_f32 / v_rcp_f32 monotone:
      // checked over every fp32 in [0, 128] by ob_silu_fast_monotone_check,
      // tests/test_i8_fused_gpu.py) and |fast_silu(y)| < 0.28 for y < 0 (its minimum is
      // -0.2785 at y = -1.2785), so this lane's max|silu| over the row tile is silu(max y)
      // whenever that is >= 0.28 -- one silu a lane instead of one an element, the same
      // float as the max over every element; otherwise every element (the exact fallback)
      float ym = -INFINITY;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int col = n0 + 16 * t + r;
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
          const int64_t orow = m0 + 4 * g + reg;
          const float y = epilogue(acc[t][reg], osc, bcol[t]);
          ym = (orow < M && col < N) ? fmaxf(ym, y) : ym;
        }
      }
      const float cand = silu_fast(ym);
      if (ym >= 0.0f && cand >= 0.28f) {
        amx = fmaxf(amx, cand);
      } else {
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const int col = n0 + 16 * t + r;
#pragma unroll
          for (int reg = 0; reg < 4; ++reg) {
            const int64_t orow = m0 + 4 * g + reg;
            const float v = fabsf(silu_fast(epilogue(acc[t][reg], osc, bcol[t])));
            amx = (orow < M && col < N) ? fmaxf(amx, v) : amx;
          }
        }
      }
    } else if constexpr (EPI == kI8SwishQ) {
      // int8 image through a per-wave byte tile [16 rows][16 NT + 16] in LDS: lane (r, g)
      // quantises rows 4g .. 4g+3 of column 16t + r in registers; the tile's rows then
      // leave as 16-byte segments (host-checked: N % 16 == 0, C8 16-B aligned)
      constexpr int kBP = 16 * NT + 16;
      uint8_t* bt = reinterpret_cast<uint8_t*>(smem + i8_stage_off(NT, NCH)) + wave * 16 * kBP;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
          float q = rintf(silu_fast(epilogue(acc[t][reg], osc, bcol[t])) * sx_out);
          q = fminf(fmaxf(q, -127.0f), 127.0f);
          bt[(4 * g + reg) * kBP + 16 * t + r] = (uint8_t)(int)q;
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      constexpr int kSeg = 16 * NT;  // 16 rows x NT segments
#pragma unroll
      for (int it = 0; it < (kSeg + 63) / 64; ++it) {
        const int idx = it * 64 + lane;
        const int row = idx / NT, seg = idx - row * NT;
        const int64_t orow = m0 + row;
        const int col = n0 + 16 * seg;
        if (idx < kSeg && orow < M && col < N)
          *reinterpret_cast<u32x4*>(C8 + orow * N + col) =
              *reinterpret_cast<const u32x4*>(bt + row * kBP + 16 * seg);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    } else {
      // row-coalesced (host-checked: N % 4 == 0, C / R 16-B aligned)
      constexpr int kCW = NT < 4 ? NT : 4, kCC = 16 * kCW, kLd = kCC + 4, kQ = kCC / 4;
      float* stg = reinterpret_cast<float*>(smem + i8_stage_off(NT, NCH)) + wave * 16 * kLd;
#pragma unroll
      for (int c0 = 0; c0 < NT; c0 += kCW) {
#pragma unroll
        for (int t = 0; t < kCW; ++t) {
          if (c0 + t >= NT) continue;
#pragma unroll
          for (int reg = 0; reg < 4; ++reg)
            stg[(4 * g + reg) * kLd + 16 * t + r] = epilogue(acc[c0 + t][reg], osc, bcol[c0 + t]);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int it = 0; it < kCW; ++it) {
          const int idx = it * 64 + lane, row = idx / kQ, c4 = idx - row * kQ;
          const int64_t orow = m0 + row;
          const int col = n0 + 16 * c0 + 4 * c4;
          const f32x4 y = *reinterpret_cast<const f32x4*>(stg + row * kLd + 4 * c4);
          if (orow < M && col < N && 4 * c4 < 16 * (NT - c0)) {
            f32x4 out;
            if constexpr (EPI == kI8Swish) {
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                out[e] = silu_fast(y[e]);
                amx = fmaxf(amx, fabsf(out[e]));
              }
            } else {
              bool valid = true;
              if (ep.lens) {
                const int64_t grow = rowbase + orow;
                const int64_t bb = grow / ep.T;
                valid = (grow - bb * ep.T) < ep.lens[bb];
              }
              const f32x4 rv = *reinterpret_cast<const f32x4*>(ep.R + (rowbase + orow) * N + col);
#pragma unroll
              for (int e = 0; e < 4; ++e) {
#pragma clang fp contract(off)
                const float v = valid ? y[e] : y[e] * 0.0f;
                out[e] = rv[e] + (ep.rscale == 1.0f ? v : ep.rscale * v);
              }
            }
            *reinterpret_cast<f32x4*>(C + orow * N + col) = out;
          }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
  if constexpr (EPI == kI8Swish || EPI == kI8SwishAmax) {
    // the block's max|C| -> one atomicMax per block (order-independent: deterministic)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) amx = fmaxf(amx, __shfl_xor(amx, o));
    __shared__ uint32_t bmax[kThreads / 64];
    if (lane == 0) bmax[wave] = __float_as_uint(amx);
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t m = bmax[0];
#pragma unroll
      for (int w2 = 1; w2 < kThreads / 64; ++w2) m = max(m, bmax[w2]);
      if (m != 0u) atomicMax(ep.amax_out + p, m);
    }
  }
}

// fast_silu(next float) >= fast_silu(x) for every fp32 x in [lo, hi) (bit patterns; both
// non-negative): the property the I8_SWISH_AMAX epilogue's one-silu-a-lane max relies on
__global__ __launch_bounds__(kThreads) void silu_monotone_kernel(uint32_t lo, uint32_t hi,
                                                                 uint32_t* __restrict__ bad) {
  uint32_t n = 0;
  const uint32_t stride = gridDim.x * kThreads;
  for (uint32_t b = lo + blockIdx.x * kThreads + threadIdx.x; b < hi; b += stride) {
    const float a = __uint_as_float(b), c = __uint_as_float(b + 1);
    n += silu_fast(c) < silu_fast(a) ? 1u : 0u;
  }
  for (int o = 32; o > 0; o >>= 1) n += __shfl_xor(n, o);
  if ((threadIdx.x & 63) == 0 && n) atomicAdd(bad, n);
}

size_t i8_image_bytes(int nt, int64_t K) {
  return (size_t)(16 * nt) * (size_t)(64 * ceil_div(K, 64) + 16);
}

// fused epilogues add the staging tiles; their total stays within 80 KB (2 blocks per CU)
int pick_nt_i8(int64_t N, int64_t K, bool epi = false) {
  static const int cands[] = {12, 9, 6, 4, 3, 2, 1};
  auto fits = [&](int nt) {
    return epi ? i8_stage_off(nt, (int)ceil_div(K, 64)) + i8_stage_bytes(nt) <= 80 * 1024
               : i8_image_bytes(nt, K) <= kMaxLds;
  };
  for (int nt : cands)
    if (N % (16 * nt) == 0 && fits(nt)) return nt;
  for (int nt : cands)
    if (16 * nt <= ((N + 15) & ~int64_t(15)) && fits(nt)) return nt;
  return 0;
}

template <int NT>
bool launch_i8_nt(const void* A, bool ai8, int P, int64_t M, int64_t K, const uint32_t* codes,
                  const uint32_t* codes1, const int* pass_bits, int64_t N, const float* alpha,
                  int alpha_raw, const float* amax, const float* bias, void* C, hipStream_t s,
                  int mode = kI8Plain, const I8Epi& ep = I8Epi{}) {
  const int n_ct = (int)ceil_div(N, 16 * NT);
  const int n_rt = (int)ceil_div(M, kRows);
  int rgroups = kTargetBlocks / (n_ct * P);
  if (rgroups < 1) rgroups = 1;
  if (rgroups > n_rt) rgroups = n_rt;
  const dim3 grid((unsigned)(rgroups * n_ct), (unsigned)P);
  const int KW = (int)ceil_div(K, 16);
#define OB_I8E(NCH, E, Q)                                                                     \
  hipLaunchKernelGGL((tgemm_i8_kernel<NT, NCH, E, Q>), grid, dim3(kThreads),                  \
                     i8_stage_off(NT, NCH) + (E == kI8Plain ? 0 : i8_stage_bytes(NT)), s, A, M, \
                     (int)K, codes, KW, (int)N, n_ct, n_rt, rgroups, alpha, alpha_raw, amax,     \
                     bias, C, codes1, pass_bits, ep);
  // int8 operands: the plain / residual consumers and the two swish producer launches;
  // fp32 operands: plain / swish (+ absmax) / residual
#define OB_I8(NCH)                                                         \
  if (ai8) {                                                               \
    if (mode == kI8Residual) { OB_I8E(NCH, kI8Residual, true) }            \
    else if (mode == kI8SwishAmax) { OB_I8E(NCH, kI8SwishAmax, true) }     \
    else if (mode == kI8SwishQ) { OB_I8E(NCH, kI8SwishQ, true) }           \
    else if (mode == kI8Plain) { OB_I8E(NCH, kI8Plain, true) }             \
    else return false;                                                     \
  } else {                                                                 \
    if (mode == kI8Swish) { OB_I8E(NCH, kI8Swish, false) }                 \
    else if (mode == kI8Residual) { OB_I8E(NCH, kI8Residual, false) }      \
    else if (mode == kI8Plain) { OB_I8E(NCH, kI8Plain, false) }            \
    else return false;                                                     \
  }                                                                        \
  return true;
  switch (ceil_div(K, 64)) {
    case 1: OB_I8(1)
    case 2: OB_I8(2)
    case 3: OB_I8(3)
    case 4: OB_I8(4)
    case 5: OB_I8(5)
    case 6: OB_I8(6)
    case 7: OB_I8(7)
    case 8: OB_I8(8)
    case 9: OB_I8(9)
    default: return false;
  }
#undef OB_I8
#undef OB_I8E
}

bool launch_i8_any(const void* A, bool ai8, int P, int64_t M, int64_t K, const uint32_t* codes,
                   const uint32_t* codes1, const int* pass_bits, int64_t N, const float* alpha,
                   int alpha_raw, const float* amax, const float* bias, void* C, hipStream_t s,
                   int mode, const I8Epi& ep) {
#define OB_I8NT(V)                                                                              \
  case V:                                                                                       \
    return launch_i8_nt<V>(A, ai8, P, M, K, codes, codes1, pass_bits, N, alpha, alpha_raw, amax, \
                           bias, C, s, mode, ep);
  switch (pick_nt_i8(N, K, mode != kI8Plain)) {
    OB_I8NT(12)
    OB_I8NT(9)
    OB_I8NT(6)
    OB_I8NT(4)
    OB_I8NT(3)
    OB_I8NT(2)
    OB_I8NT(1)
    default: return false;
  }
#undef OB_I8NT
}

}  // namespace

bool ternary_gemm_i8_supported(int64_t K, int64_t N) {
  return K >= 16 && K % 16 == 0 && K <= 576 && N >= 1 && pick_nt_i8(N, K) > 0;
}

size_t act_absmax_workspace(int P) { return sizeof(uint32_t) * (size_t)P * kAbsParts; }

void launch_silu_monotone_check(uint32_t lo, uint32_t hi, uint32_t* bad, hipStream_t s) {
  if (hi <= lo) return;
  hipLaunchKernelGGL(silu_monotone_kernel, dim3(2048), dim3(kThreads), 0, s, lo, hi, bad);
}

void launch_act_absmax(const float* X, int P, int64_t n_per_pass, float* amax, void* ws,
                       hipStream_t s) {
  uint32_t* part = static_cast<uint32_t*>(ws);
  hipLaunchKernelGGL(act_absmax_part_kernel, dim3(kAbsParts, (unsigned)P), dim3(kThreads), 0, s,
                     X, n_per_pass, part);
  hipLaunchKernelGGL(act_absmax_final_kernel, dim3((unsigned)P), dim3(64), 0, s,
                     (const uint32_t*)part, kAbsParts, reinterpret_cast<uint32_t*>(amax));
}

void launch_act_dequant(const float* X, int P, int64_t n_per_pass, const float* amax, float* Xd,
                        hipStream_t s) {
  if (n_per_pass == 0) return;
  int64_t blocks = ceil_div(n_per_pass, kThreads * 4);
  if (blocks > 2048 / P) blocks = 2048 / P > 0 ? 2048 / P : 1;
  hipLaunchKernelGGL(act_dequant_kernel, dim3((unsigned)blocks, (unsigned)P), dim3(kThreads), 0,
                     s, X, n_per_pass, amax, Xd);
}

bool launch_ternary_gemm_i8(const float* A, int P, int64_t M, int64_t K, const uint32_t* codes,
                            const uint32_t* codes1, const int* pass_bits, int64_t N,
                            const float* alpha, int alpha_raw, const float* amax,
                            const float* bias, float* C, hipStream_t s) {
  if (M == 0 || N == 0 || P == 0) return true;
  return launch_i8_any(A, false, P, M, K, codes, codes1, pass_bits, N, alpha, alpha_raw, amax,
                       bias, C, s, kI8Plain, I8Epi{});
}

bool launch_ternary_gemm_i8_epi(const float* A, int P, int64_t M, int64_t K,
                                const uint32_t* codes, const uint32_t* codes1,
                                const int* pass_bits, int64_t N, const float* alpha,
                                int alpha_raw, const float* amax, const float* bias, float* C,
                                int mode, const float* R, float rscale, const int* lens, int64_t T,
                                float* amax_out, hipStream_t s) {
  I8Epi ep{R, rscale, lens, (int)(T > 0 ? T : 1), reinterpret_cast<uint32_t*>(amax_out)};
  if (mode == kI8Swish) launch_zero_words(amax_out, P, s);
  if (M == 0 || N == 0 || P == 0) return true;
  return launch_i8_any(A, false, P, M, K, codes, codes1, pass_bits, N, alpha, alpha_raw, amax,
                       bias, C, s, mode, ep);
}

// int8 operand Aq (its producer's scale from amax). mode 0 plain / 2 residual: C fp32;
// mode 3 (swish -> int8): two launches over the same tiles -- the first only reduces the
// per-pass max|silu(y)| into amax_out, the second recomputes silu(y) and stores it as int8
// at that scale (C int8 [P*M][N]). Recomputing the K-wide product is cheaper than a round
// trip of the fp32 activation through HBM (4 bytes written + read per element).
bool launch_ternary_gemm_i8q(const int8_t* Aq, int P, int64_t M, int64_t K,
                             const uint32_t* codes, const uint32_t* codes1, const int* pass_bits,
                             int64_t N, const float* alpha, int alpha_raw, const float* amax,
                             const float* bias, void* C, int mode, const float* R, float rscale,
                             const int* lens, int64_t T, float* amax_out, hipStream_t s) {
  I8Epi ep{R, rscale, lens, (int)(T > 0 ? T : 1), reinterpret_cast<uint32_t*>(amax_out)};
  if (mode == 3) launch_zero_words(amax_out, P, s);
  if (M == 0 || N == 0 || P == 0) return true;
  if (mode == 3) {
    return launch_i8_any(Aq, true, P, M, K, codes, codes1, pass_bits, N, alpha, alpha_raw, amax,
                         bias, nullptr, s, kI8SwishAmax, ep) &&
           launch_i8_any(Aq, true, P, M, K, codes, codes1, pass_bits, N, alpha, alpha_raw, amax,
                         bias, C, s, kI8SwishQ, ep);
  }
  return launch_i8_any(Aq, true, P, M, K, codes, codes1, pass_bits, N, alpha, alpha_raw, amax,
                       bias, C, s, mode == 2 ? kI8Residual : kI8Plain, ep);
}

}  // namespace ob
