// dw.hip — BitLinear weight-gradient GEMM, split over rows (M):
//   part[c] = dY[rows of chunk c]^T . X[rows of chunk c]      (autograd of quant.py:126)
// finished by ste_reduce (quant.hip), which applies quant.py:80-91.
//
// fp32 v_mfma_f32_16x16x4_f32 (exact fp32 fma chain). Fragment map (lane l, r = l&15,
// g = l>>4): A[i=r][kk=g], B[kk=g][j=r], D[row=4g+reg][col=r]; kk is free to permute as
// long as A and B agree, so every lane loads 4 contiguous fp32 (one dwordx4) of a row.
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
  // Loads are unconditional from clamped addresses (a guarded load makes hipcc branch and
  // wait vmcnt(0) at it); rows outside the chunk are zeroed at use, in compute().
  const int64_t ncl = ncol < N - 4 ? ncol : (N >= 4 ? N - 4 : 0);
  const int64_t kcl = kcol < K - 4 ? kcol : (K >= 4 ? K - 4 : 0);
  auto load_step = [&](int64_t step, f32x4& dy, f32x4& x) {
    const int64_t m = step + g;
    const int64_t mc = m < m_end ? m : M - 1;
    if (VEC) {
      dy = *reinterpret_cast<const f32x4*>(dY + mc * N + ncl);
      x = *reinterpret_cast<const f32x4*>(X + mc * K + kcl);
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int64_t nn = ncol + e < N ? ncol + e : N - 1;
        const int64_t kk = kcol + e < K ? kcol + e : (K > 0 ? K - 1 : 0);
        dy[e] = dY[mc * N + nn];
        x[e] = K > 0 ? X[mc * K + kk] : 0.0f;
      }
    }
  };
  const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};
  auto compute = [&](int64_t step, const f32x4& dy_raw, const f32x4& x_raw) {
    const bool mv = step + g < m_end;
    f32x4 dy = (mv && ncol < N) ? dy_raw : zero4;
    f32x4 x = (mv && kcol < K) ? x_raw : zero4;
    if (!VEC) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        dy[e] = (ncol + e < N) ? dy[e] : 0.0f;
        x[e] = (kcol + e < K) ? x[e] : 0.0f;
      }
    }
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
    compute(s0 + 16 * i, bdy[i], bx[i]);
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
