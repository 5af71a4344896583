// gemm.hip — the three BitLinear GEMMs on gfx950 matrix cores.
//
//   forward  Y  = a * X . Q^T + b     (quant.py:126, F.linear with W_hat = a*Q)
//   backward dX = a * dY . Q          (autograd of quant.py:126)
//   backward G  = dY^T . X            (autograd of quant.py:126, reduced over all rows)
//
// All three keep fp32 parity with the reference's fp32 F.linear:
//  * ternary GEMMs (forward, dX): each fp32 activation is split exactly into three bf16
//    parts x = hi + mid + lo (8+8+8 significand bits); Q in {-1,0,+1} is exact in bf16, so
//    three v_mfma_f32_16x16x32_bf16 per k-step accumulate exact products in fp32 -- the
//    result equals an fp32 GEMM up to summation order, at 3/16 of the fp32-MFMA cost.
//    The scale `a` is applied once in the epilogue (Y = a*(X.Q^T)).
//  * dW GEMM: v_mfma_f32_16x16x4_f32 (exact fp32 fma chain).
//  * OB_GEMM=f32 in the environment selects the fp32-MFMA ternary GEMM (A/B debugging).
//
// Fragment maps (lane l, r = l&15, g = l>>4), D[row=4g+reg][col=r] for both shapes:
//   16x16x4 f32 : A[i=r][kk=g],          B[kk=g][j=r]
//   16x16x32 bf16: A[i=r][kk=8g+j] (j<8), B[kk=8g+j][col=r]
// The kk index is free to permute as long as A and B agree.
#include <cstdlib>

#include "ob_launch.h"
#include "ob_quant.h"

namespace ob {

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kThreads = 256;  // 4 waves
constexpr int kGemmRows = 64;  // rows of X per block (16 per wave)

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// ---------------------------------------------------------------------------------
// Ternary GEMM: C[M][N] = a * (A[M][K] . Q^T) + bias, Q as codes [N][KW].
// Block: 4 waves stacked along M (64 rows) x NT 16-column tiles.
// Per 16-wide k chunk a lane loads X[row][kc+4g .. kc+4g+3] (one float4) and one code
// word per n tile; byte g of that word holds the 4 codes of k = kc+4g+e, e = 0..3.
// ---------------------------------------------------------------------------------
template <int NT, bool VEC>
__global__ __launch_bounds__(kThreads) void ternary_gemm_kernel(
    const float* __restrict__ A, int64_t M, int64_t K, const uint32_t* __restrict__ codes,
    int64_t KW, int64_t N, const float* __restrict__ alpha, int alpha_raw,
    const float* __restrict__ bias, float* __restrict__ C) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int r = lane & 15;
  const int g = lane >> 4;
  const int64_t m0 = (int64_t)blockIdx.x * kGemmRows + wave * 16;
  const int64_t n0 = (int64_t)blockIdx.y * (16 * NT);
  const int64_t row = m0 + r;
  const bool rvalid = row < M;
  const float* arow = A + (rvalid ? row : 0) * K;

  const uint32_t* crow[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int64_t n = n0 + 16 * t + r;
    crow[t] = (n < N) ? codes + n * KW : nullptr;
  }

  f32x4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};


  for (int64_t kc = 0; kc < K; kc += 16) {
    const int64_t k = kc + 4 * g;
    f32x4 xa;
    if (VEC) {
      xa = (rvalid && k < K) ? *reinterpret_cast<const f32x4*>(arow + k) : f32x4{0.f, 0.f, 0.f, 0.f};
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) xa[e] = (rvalid && k + e < K) ? arow[k + e] : 0.0f;
    }
    const int64_t w = kc >> 4;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const uint32_t word = crow[t] ? crow[t][w] : 0u;
      const uint32_t byte = word >> (8 * g);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        acc[t] = mfma4(xa[e], code_value((byte >> (2 * e)) & 3u), acc[t]);
      }
    }
  }

  const float a = effective_alpha(alpha, alpha_raw);
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int64_t col = n0 + 16 * t + r;
    if (col >= N) continue;
    const float b = bias ? bias[col] : 0.0f;
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      const int64_t orow = m0 + 4 * g + reg;
      if (orow < M) C[orow * N + col] = fmaf(a, acc[t][reg], b);
    }
  }
}

// ---------------------------------------------------------------------------------
// Ternary GEMM, bf16x3 split: C[M][N] = a * (A[M][K] . Q^T) + bias.
// Block: 4 waves stacked along M (64 rows) x NT 16-column tiles. At entry the block
// decodes its 16*NT code rows into a bf16 image of Q in LDS ([16*NT][Kpad+8], row pad
// keeps ds_read_b128 conflict-free at K = 144 / 576), then each wave streams its 16 rows
// of A in 32-wide k-chunks (two dwordx4 per lane, prefetched two chunks ahead), splits
// them into hi/mid/lo bf16 fragments and issues 3 MFMAs per n tile.
// ---------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t code_bf16(uint32_t c) {
  return ((c & 1u) * 0x3F80u) | ((c & 2u) << 14);  // 0 -> 0, 1 -> +1.0, 3 -> -1.0
}

__device__ __forceinline__ void split3(const f32x4& a, const f32x4& b, bf16x8& hi, bf16x8& mid,
                                       bf16x8& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float x = j < 4 ? a[j] : b[j - 4];
    const __bf16 h = (__bf16)x;
    const float r1 = x - (float)h;  // exact
    const __bf16 m = (__bf16)r1;
    const float r2 = r1 - (float)m;  // exact, fits in 8 bits
    hi[j] = h;
    mid[j] = m;
    lo[j] = (__bf16)r2;
  }
}

__device__ __forceinline__ f32x4 mfma_bf16(const bf16x8& a, const bf16x8& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// Loads are issued unconditionally from a clamped (always valid) address and zeroed
// afterwards with a select: a guarded `cond ? *p : 0` load makes hipcc branch around the
// load and wait vmcnt(0) at it, which serialises the prefetch pipeline.
__device__ __forceinline__ f32x4 zero_unless(bool ok, f32x4 v) {
  const f32x4 z = {0.f, 0.f, 0.f, 0.f};
  return ok ? v : z;
}

template <bool VEC>
__device__ __forceinline__ void load8(const float* __restrict__ arow, bool rvalid, int k, int K,
                                      f32x4& a, f32x4& b) {
  if (VEC) {  // K % 4 == 0, K >= 4
    const int ka = k < K - 4 ? k : K - 4;
    const int kb = k + 4 < K - 4 ? k + 4 : K - 4;
    const f32x4 va = *reinterpret_cast<const f32x4*>(arow + ka);
    const f32x4 vb = *reinterpret_cast<const f32x4*>(arow + kb);
    a = zero_unless(rvalid && k < K, va);
    b = zero_unless(rvalid && k + 4 < K, vb);
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k0 = k + e < K - 1 ? k + e : K - 1;
      const int k1 = k + 4 + e < K - 1 ? k + 4 + e : K - 1;
      const float v0 = arow[k0 < 0 ? 0 : k0];
      const float v1 = arow[k1 < 0 ? 0 : k1];
      a[e] = (rvalid && k + e < K) ? v0 : 0.0f;
      b[e] = (rvalid && k + 4 + e < K) ? v1 : 0.0f;
    }
  }
}

template <int NT, bool VEC, int NCH>
__global__ __launch_bounds__(kThreads) void tgemm_bf16x3_kernel(
    const float* __restrict__ A, int64_t M, int K, const uint32_t* __restrict__ codes, int KW,
    int N, const float* __restrict__ alpha, int alpha_raw, const float* __restrict__ bias,
    float* __restrict__ C) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __bf16* bimg = reinterpret_cast<__bf16*>(smem);
  const int kpad = (K + 31) & ~31;
  const int stride = kpad + 8;
  const int kwp = kpad >> 4;
  const int n0 = blockIdx.y * (16 * NT);

  // Decode this block's Q rows into LDS: one code word -> 16 bf16 (two 16-byte stores).
  for (int idx = threadIdx.x; idx < 16 * NT * kwp; idx += kThreads) {
    const int nl = idx / kwp, w = idx - nl * kwp;
    const int n = n0 + nl;
    const uint32_t word = (n < N && w < KW) ? codes[(int64_t)n * KW + w] : 0u;
    u32x4 lo4, hi4;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      lo4[p] = code_bf16((word >> (4 * p)) & 3u) | (code_bf16((word >> (4 * p + 2)) & 3u) << 16);
      hi4[p] = code_bf16((word >> (4 * p + 16)) & 3u) |
               (code_bf16((word >> (4 * p + 18)) & 3u) << 16);
    }
    u32x4* dst = reinterpret_cast<u32x4*>(bimg + nl * stride + 16 * w);
    dst[0] = lo4;
    dst[1] = hi4;
  }
  __syncthreads();

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int r = lane & 15;
  const int g = lane >> 4;
  const int64_t m0 = (int64_t)blockIdx.x * kGemmRows + wave * 16;
  const int64_t row = m0 + r;
  const bool rvalid = row < M;
  const float* arow = A + (rvalid ? row : M - 1) * (int64_t)K;
  const __bf16* brow = bimg + r * stride + 8 * g;

  f32x4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](const f32x4& x0, const f32x4& x1, int kc) {
    bf16x8 hi, mid, lo;
    split3(x0, x1, hi, mid, lo);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const bf16x8 bq = *reinterpret_cast<const bf16x8*>(brow + t * 16 * stride + kc);
      acc[t] = mfma_bf16(lo, bq, acc[t]);
      acc[t] = mfma_bf16(mid, bq, acc[t]);
      acc[t] = mfma_bf16(hi, bq, acc[t]);
    }
  };
  const int kg = 8 * g;
  if constexpr (NCH > 0) {
    // K is a compile-time chunk count: fully unrolled, a window of kWin chunks in flight,
    // every wait a counted vmcnt.
    constexpr int kWin = NCH < 6 ? NCH : 6;
    f32x4 buf[NCH > 0 ? NCH : 1][2];
#pragma unroll
    for (int c = 0; c < kWin; ++c) load8<VEC>(arow, rvalid, 32 * c + kg, K, buf[c][0], buf[c][1]);
    // sched_barrier keeps hipcc's scheduler from sinking each load next to its use
    // (which would leave one load in flight and a vmcnt(0) per chunk).
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      if (c + kWin < NCH)
        load8<VEC>(arow, rvalid, 32 * (c + kWin) + kg, K, buf[c + kWin][0], buf[c + kWin][1]);
      __builtin_amdgcn_sched_barrier(0);
      compute(buf[c][0], buf[c][1], 32 * c);
    }
  } else if (K > 0) {  // K == 0: A may have no storage at all
    // Generic K: three rotating register sets, unrolled so no register copy of an
    // in-flight load exists (a copy would make hipcc wait for it).
    f32x4 r0a, r0b, r1a, r1b, r2a, r2b;
    load8<VEC>(arow, rvalid, kg, K, r0a, r0b);
    load8<VEC>(arow, rvalid, 32 + kg, K, r1a, r1b);
    for (int kc = 0; kc < kpad; kc += 96) {
      load8<VEC>(arow, rvalid, kc + 64 + kg, K, r2a, r2b);
      compute(r0a, r0b, kc);
      load8<VEC>(arow, rvalid, kc + 96 + kg, K, r0a, r0b);
      if (kc + 32 < kpad) compute(r1a, r1b, kc + 32);
      load8<VEC>(arow, rvalid, kc + 128 + kg, K, r1a, r1b);
      if (kc + 64 < kpad) compute(r2a, r2b, kc + 64);
    }
  }

  const float a = effective_alpha(alpha, alpha_raw);
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int col = n0 + 16 * t + r;
    if (col >= N) continue;
    const float b = bias ? bias[col] : 0.0f;
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      const int64_t orow = m0 + 4 * g + reg;
      if (orow < M) C[orow * N + col] = fmaf(a, acc[t][reg], b);
    }
  }
}

// LDS bytes of the bf16 Q image for a column tile of 16*NT rows.
inline size_t bimg_bytes(int NT, int64_t K) {
  const int64_t kpad = (K + 31) & ~int64_t(31);
  return sizeof(uint16_t) * (size_t)(16 * NT) * (size_t)(kpad + 8);
}
constexpr size_t kMaxDynLds = 64 * 1024;

bool use_f32_gemm() {
  static const int v = [] {
    const char* e = getenv("OB_GEMM");
    return (e && e[0] == 'f') ? 1 : 0;
  }();
  return v != 0;
}

template <int NT>
void launch_gemm_nt(const float* A, int64_t M, int64_t K, const uint32_t* codes, int64_t N,
                    const float* alpha, int alpha_raw, const float* bias, float* C,
                    hipStream_t s) {
  const int64_t KW = ceil_div(K, 16);
  dim3 grid((unsigned)ceil_div(M, kGemmRows), (unsigned)ceil_div(N, 16 * NT));
  const bool vec = (K % 4 == 0) && K >= 4 && ((reinterpret_cast<uintptr_t>(A) & 15) == 0);
  const size_t lds = bimg_bytes(NT, K);
  if (!use_f32_gemm() && lds <= kMaxDynLds) {
#define OB_TGEMM(NCH)                                                                        \
  hipLaunchKernelGGL((tgemm_bf16x3_kernel<NT, true, NCH>), grid, dim3(kThreads), lds, s, A, M, \
                     (int)K, codes, (int)KW, (int)N, alpha, alpha_raw, bias, C)
    if (vec) {
      switch ((K + 31) / 32) {  // Conformer widths: 64, 144, 256, 576
        case 2: OB_TGEMM(2); break;
        case 5: OB_TGEMM(5); break;
        case 8: OB_TGEMM(8); break;
        case 18: OB_TGEMM(18); break;
        default: OB_TGEMM(0); break;
      }
    } else {
      hipLaunchKernelGGL((tgemm_bf16x3_kernel<NT, false, 0>), grid, dim3(kThreads), lds, s, A,
                         M, (int)K, codes, (int)KW, (int)N, alpha, alpha_raw, bias, C);
    }
#undef OB_TGEMM
    return;
  }
  // fp32-MFMA path: exact fma chain; also the fallback for K too large for the LDS image.
  if (vec)
    hipLaunchKernelGGL((ternary_gemm_kernel<NT, true>), grid, dim3(kThreads), 0, s, A, M, K,
                       codes, KW, N, alpha, alpha_raw, bias, C);
  else
    hipLaunchKernelGGL((ternary_gemm_kernel<NT, false>), grid, dim3(kThreads), 0, s, A, M, K,
                       codes, KW, N, alpha, alpha_raw, bias, C);
}

// ---------------------------------------------------------------------------------
// dW partial: part[c][n][k] = sum_{m in chunk c} dY[m][n] * X[m][k].
// Block = one 64x64 (n,k) output tile x one M chunk; its 4 waves split the chunk's rows
// in 16-row steps (wave w takes rows step+4w .. step+4w+3, lane row = g), and their
// tiles are summed in wave order through LDS (deterministic).
// A lane loads dY[m][n0+4r .. +3] and X[m][k0+4r .. +3]; MFMA (e,f) pairs element e of
// the first with element f of the second, so tile (e,f) covers n = n0+4i+e,
// k = k0+4j+f for its 16x16 (i,j).
// Waves of k-tile 0 also sum dY over their rows for db.
// ---------------------------------------------------------------------------------
constexpr int kDwTile = 64;

template <bool VEC, int S>
__global__ __launch_bounds__(kThreads) void dw_partial_kernel(
    const float* __restrict__ dY, const float* __restrict__ X, int64_t M, int64_t N, int64_t K,
    int64_t tiles_k, int64_t rows_per_chunk, float* __restrict__ part,
    float* __restrict__ part_db, uint32_t* __restrict__ ticket) {
  __shared__ float red[2][kDwTile * kDwTile];  // 32 KB: waves pair up (0+2, 1+3)
  __shared__ float dbred[4][kDwTile];

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int r = lane & 15;
  const int g = lane >> 4;
  const int64_t tn = blockIdx.x / tiles_k;
  const int64_t tk = blockIdx.x - tn * tiles_k;
  const int64_t n0 = tn * kDwTile, k0 = tk * kDwTile;
  const int64_t chunk = blockIdx.y;
  const int64_t m_begin = chunk * rows_per_chunk;
  const int64_t m_end = (m_begin + rows_per_chunk < M) ? m_begin + rows_per_chunk : M;
  const int64_t ncol = n0 + 4 * r;
  const int64_t kcol = k0 + 4 * r;
  const bool do_db = (part_db != nullptr) && (tk == 0);
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) *ticket = 0u;

  f32x4 acc[4][4];
#pragma unroll
  for (int e = 0; e < 4; ++e)
#pragma unroll
    for (int f = 0; f < 4; ++f) acc[e][f] = f32x4{0.f, 0.f, 0.f, 0.f};
  float dbacc[4] = {0.f, 0.f, 0.f, 0.f};


  // Rows are streamed with a two-step register prefetch so the dwordx4 latency hides
  // under the 16 MFMAs of the step before.
  // Unconditional loads from clamped addresses + selects (see zero_unless).
  const int64_t ncl = ncol < N - 4 ? ncol : (N >= 4 ? N - 4 : 0);
  const int64_t kcl = kcol < K - 4 ? kcol : (K >= 4 ? K - 4 : 0);
  auto load_step = [&](int64_t step, f32x4& dy, f32x4& x) {
    const int64_t m = step + g;
    const bool mv = m < m_end;
    const int64_t mc = mv ? m : M - 1;
    if (VEC) {
      dy = zero_unless(mv && ncol < N, *reinterpret_cast<const f32x4*>(dY + mc * N + ncl));
      x = zero_unless(mv && kcol < K, *reinterpret_cast<const f32x4*>(X + mc * K + kcl));
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int64_t nn = ncol + e < N ? ncol + e : N - 1;
        const int64_t kk = kcol + e < K ? kcol + e : (K > 0 ? K - 1 : 0);
        const float vy = dY[mc * N + nn];
        const float vx = K > 0 ? X[mc * K + kk] : 0.0f;
        dy[e] = (mv && ncol + e < N) ? vy : 0.0f;
        x[e] = (mv && kcol + e < K) ? vx : 0.0f;
      }
    }
  };
  auto compute = [&](const f32x4& dy, const f32x4& x) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
#pragma unroll
      for (int f = 0; f < 4; ++f) acc[e][f] = mfma4(dy[e], x[f], acc[e][f]);
    }
    if (do_db) {
#pragma unroll
      for (int e = 0; e < 4; ++e) dbacc[e] += dy[e];
    }
  };
  // The chunk is S steps of 16 rows (4 per wave): fully unrolled with a window of kWin
  // steps in flight; rows past the chunk / M load clamped and contribute zero.
  constexpr int kWin = S < 4 ? S : 4;
  const int64_t s0 = m_begin + 4 * wave;
  f32x4 bdy[S], bx[S];
#pragma unroll
  for (int i = 0; i < kWin; ++i) load_step(s0 + 16 * i, bdy[i], bx[i]);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < S; ++i) {
    if (i + kWin < S) load_step(s0 + 16 * (i + kWin), bdy[i + kWin], bx[i + kWin]);
    __builtin_amdgcn_sched_barrier(0);
    compute(bdy[i], bx[i]);
  }

  // Combine the 4 wave tiles in a fixed order: (w0 + w2) + (w1 + w3).
  // D row = 4g+reg -> n_local = 4*(4g+reg)+e; D col = r -> k_local = 4r+f.
  float* myred = red[wave & 1];
  if (wave >= 2) {
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int f = 0; f < 4; ++f)
#pragma unroll
        for (int reg = 0; reg < 4; ++reg)
          myred[(4 * (4 * g + reg) + e) * kDwTile + 4 * r + f] = acc[e][f][reg];
  }
  __syncthreads();
  if (wave < 2) {
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int f = 0; f < 4; ++f)
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
          float* p = &myred[(4 * (4 * g + reg) + e) * kDwTile + 4 * r + f];
          *p = acc[e][f][reg] + *p;
        }
  }
  if (do_db) {
    // rows g = 0..3 of this wave hold column partials; combine in fixed order.
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float v = dbacc[e];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      dbacc[e] = v;
    }
    if (g == 0) {
#pragma unroll
      for (int e = 0; e < 4; ++e) dbred[wave][4 * r + e] = dbacc[e];
    }
  }
  __syncthreads();

  float* out = part + chunk * (N * K);
#pragma unroll 4
  for (int q = 0; q < (kDwTile * kDwTile) / kThreads; ++q) {
    const int idx = q * kThreads + threadIdx.x;
    const int nl = idx / kDwTile, kl = idx - nl * kDwTile;
    const int64_t n = n0 + nl, k = k0 + kl;
    if (n < N && k < K) {
      const float v = red[0][idx] + red[1][idx];
      out[n * K + k] = v;
    }
  }
  if (do_db && threadIdx.x < kDwTile) {
    const int64_t n = n0 + threadIdx.x;
    if (n < N) {
      const int i = threadIdx.x;
      part_db[chunk * N + n] = ((dbred[0][i] + dbred[1][i]) + dbred[2][i]) + dbred[3][i];
    }
  }
}

}  // namespace

void launch_ternary_gemm(const float* A, int64_t M, int64_t K, const uint32_t* codes, int64_t N,
                         const float* alpha, int alpha_raw, const float* bias, float* C,
                         hipStream_t s) {
  if (M == 0 || N == 0) return;
  // Column tile: 48 divides the Conformer widths (144, 576); 64 / 32 for the rest.
  if (N % 48 == 0)
    launch_gemm_nt<3>(A, M, K, codes, N, alpha, alpha_raw, bias, C, s);
  else if (N % 64 == 0)
    launch_gemm_nt<4>(A, M, K, codes, N, alpha, alpha_raw, bias, C, s);
  else if (N <= 16)
    launch_gemm_nt<1>(A, M, K, codes, N, alpha, alpha_raw, bias, C, s);
  else if (N <= 32 || N % 32 == 0)
    launch_gemm_nt<2>(A, M, K, codes, N, alpha, alpha_raw, bias, C, s);
  else
    launch_gemm_nt<3>(A, M, K, codes, N, alpha, alpha_raw, bias, C, s);
}

DwPlan plan_dw(int64_t M, int64_t N, int64_t K) {
  DwPlan p;
  // At least one tile each way so that K = 0 still produces the bias partials.
  p.tiles_n = N > 0 ? ceil_div(N, kDwTile) : 1;
  p.tiles_k = K > 0 ? ceil_div(K, kDwTile) : 1;
  const int64_t tiles = p.tiles_n * p.tiles_k;
  // Chunk = S steps x 16 rows, S in {8, 16, 32}: the longest chunk that still gives
  // >= 256 blocks (one per CU), so the partial slabs stay few.
  int64_t steps = 32;
  while (steps > 8 && tiles * ceil_div(M, 16 * steps) < 256) steps /= 2;
  p.rows_per_chunk = 16 * steps;
  p.chunks = M > 0 ? ceil_div(M, p.rows_per_chunk) : 1;
  return p;
}

void launch_dw_partial(const float* dY, const float* X, int64_t M, int64_t N, int64_t K,
                       const DwPlan& p, float* part, float* part_db, uint32_t* ticket,
                       hipStream_t s) {
  if (M == 0 || N == 0) return;
  dim3 grid((unsigned)(p.tiles_n * p.tiles_k), (unsigned)p.chunks);
  const bool vec = (N % 4 == 0) && (K % 4 == 0) && N >= 4 && K >= 4 &&
                   ((reinterpret_cast<uintptr_t>(dY) & 15) == 0) &&
                   ((reinterpret_cast<uintptr_t>(X) & 15) == 0);
#define OB_DW(V, S)                                                                        \
  hipLaunchKernelGGL((dw_partial_kernel<V, S>), grid, dim3(kThreads), 0, s, dY, X, M, N, K,   \
                     p.tiles_k, p.rows_per_chunk, part, part_db, ticket)
  const int64_t steps = p.rows_per_chunk / 16;
  if (vec) {
    if (steps == 32) OB_DW(true, 32);
    else if (steps == 16) OB_DW(true, 16);
    else OB_DW(true, 8);
  } else {
    if (steps == 32) OB_DW(false, 32);
    else if (steps == 16) OB_DW(false, 16);
    else OB_DW(false, 8);
  }
#undef OB_DW
}

}  // namespace ob
