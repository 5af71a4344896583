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

template <bool VEC>
__device__ __forceinline__ void load8(const float* __restrict__ arow, bool rvalid, int k, int K,
                                      f32x4& a, f32x4& b) {
  const f32x4 z = {0.f, 0.f, 0.f, 0.f};
  if (VEC) {
    a = (rvalid && k < K) ? *reinterpret_cast<const f32x4*>(arow + k) : z;
    b = (rvalid && k + 4 < K) ? *reinterpret_cast<const f32x4*>(arow + k + 4) : z;
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      a[e] = (rvalid && k + e < K) ? arow[k + e] : 0.0f;
      b[e] = (rvalid && k + 4 + e < K) ? arow[k + 4 + e] : 0.0f;
    }
  }
}

template <int NT, bool VEC>
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
  const float* arow = A + (rvalid ? row : 0) * (int64_t)K;
  const __bf16* brow = bimg + r * stride + 8 * g;

  f32x4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};

  f32x4 c0, c1, n0v, n1v;
  load8<VEC>(arow, rvalid, 8 * g, K, c0, c1);
  load8<VEC>(arow, rvalid, 32 + 8 * g, K, n0v, n1v);
  for (int kc = 0; kc < kpad; kc += 32) {
    f32x4 p0, p1;
    load8<VEC>(arow, rvalid, kc + 64 + 8 * g, K, p0, p1);
    bf16x8 hi, mid, lo;
    split3(c0, c1, hi, mid, lo);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const bf16x8 bq = *reinterpret_cast<const bf16x8*>(brow + t * 16 * stride + kc);
      acc[t] = mfma_bf16(lo, bq, acc[t]);
      acc[t] = mfma_bf16(mid, bq, acc[t]);
      acc[t] = mfma_bf16(hi, bq, acc[t]);
    }
    c0 = n0v;
    c1 = n1v;
    n0v = p0;
    n1v = p1;
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
  const bool vec = (K % 4 == 0) && ((reinterpret_cast<uintptr_t>(A) & 15) == 0);
  const size_t lds = bimg_bytes(NT, K);
  if (!use_f32_gemm() && lds <= kMaxDynLds) {
    if (vec)
      hipLaunchKernelGGL((tgemm_bf16x3_kernel<NT, true>), grid, dim3(kThreads), lds, s, A, M,
                         (int)K, codes, (int)KW, (int)N, alpha, alpha_raw, bias, C);
    else
      hipLaunchKernelGGL((tgemm_bf16x3_kernel<NT, false>), grid, dim3(kThreads), lds, s, A, M,
                         (int)K, codes, (int)KW, (int)N, alpha, alpha_raw, bias, C);
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

template <bool VEC>
__global__ __launch_bounds__(kThreads) void dw_partial_kernel(
    const float* __restrict__ dY, const float* __restrict__ X, int64_t M, int64_t N, int64_t K,
    int64_t tiles_k, int64_t rows_per_chunk, float* __restrict__ part,
    float* __restrict__ part_db) {
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

  f32x4 acc[4][4];
#pragma unroll
  for (int e = 0; e < 4; ++e)
#pragma unroll
    for (int f = 0; f < 4; ++f) acc[e][f] = f32x4{0.f, 0.f, 0.f, 0.f};
  float dbacc[4] = {0.f, 0.f, 0.f, 0.f};


  // Rows are streamed with a two-step register prefetch so the dwordx4 latency hides
  // under the 16 MFMAs of the step before.
  auto load_step = [&](int64_t step, f32x4& dy, f32x4& x) {
    const int64_t m = step + g;
    const bool mv = m < m_end;
    if (VEC) {
      dy = (mv && ncol < N) ? *reinterpret_cast<const f32x4*>(dY + m * N + ncol)
                            : f32x4{0.f, 0.f, 0.f, 0.f};
      x = (mv && kcol < K) ? *reinterpret_cast<const f32x4*>(X + m * K + kcol)
                           : f32x4{0.f, 0.f, 0.f, 0.f};
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        dy[e] = (mv && ncol + e < N) ? dY[m * N + ncol + e] : 0.0f;
        x[e] = (mv && kcol + e < K) ? X[m * K + kcol + e] : 0.0f;
      }
    }
  };
  int64_t step = m_begin + 4 * wave;
  f32x4 dy0, x0, dy1, x1;
  load_step(step, dy0, x0);
  load_step(step + 16, dy1, x1);
  for (; step < m_end; step += 16) {
    f32x4 dy2, x2;
    load_step(step + 32, dy2, x2);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
#pragma unroll
      for (int f = 0; f < 4; ++f) acc[e][f] = mfma4(dy0[e], x0[f], acc[e][f]);
    }
    if (do_db) {
#pragma unroll
      for (int e = 0; e < 4; ++e) dbacc[e] += dy0[e];
    }
    dy0 = dy1;
    x0 = x1;
    dy1 = dy2;
    x1 = x2;
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
  // Aim for ~512 blocks (2 per CU, 8 waves) but keep >= 128 rows per chunk: fewer
  // partial slabs for the reduction to read back.
  int64_t chunks = ceil_div(512, tiles > 0 ? tiles : 1);
  const int64_t max_chunks = ceil_div(M, 128);
  if (chunks > max_chunks) chunks = max_chunks;
  if (chunks < 1) chunks = 1;
  int64_t rows = ceil_div(M, chunks);
  rows = ceil_div(rows, 16) * 16;
  p.rows_per_chunk = rows > 0 ? rows : 16;
  p.chunks = M > 0 ? ceil_div(M, p.rows_per_chunk) : 1;
  return p;
}

void launch_dw_partial(const float* dY, const float* X, int64_t M, int64_t N, int64_t K,
                       const DwPlan& p, float* part, float* part_db, hipStream_t s) {
  if (M == 0 || N == 0) return;
  dim3 grid((unsigned)(p.tiles_n * p.tiles_k), (unsigned)p.chunks);
  const bool vec = (N % 4 == 0) && (K % 4 == 0) &&
                   ((reinterpret_cast<uintptr_t>(dY) & 15) == 0) &&
                   ((reinterpret_cast<uintptr_t>(X) & 15) == 0);
  if (vec)
    hipLaunchKernelGGL(dw_partial_kernel<true>, grid, dim3(kThreads), 0, s, dY, X, M, N, K,
                       p.tiles_k, p.rows_per_chunk, part, part_db);
  else
    hipLaunchKernelGGL(dw_partial_kernel<false>, grid, dim3(kThreads), 0, s, dY, X, M, N, K,
                       p.tiles_k, p.rows_per_chunk, part, part_db);
}

}  // namespace ob
