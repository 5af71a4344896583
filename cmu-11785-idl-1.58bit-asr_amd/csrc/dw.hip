// dw.hip — BitLinear weight-gradient GEMM, split over rows (M):
//   part[c] = dY[rows of chunk c]^T . X[rows of chunk c]      (autograd of quant.py:126)
// finished by ste_reduce (quant.hip), which applies quant.py:80-91.
//
// Default kernel: bf16x6 split MFMA. Both operands are dense fp32; each is split exactly
// into hi + mid + lo bf16 parts and the six products with combined weight >= 2^-16
// (hh, hm, mh, hl, lh, mm; each exact in fp32) are accumulated by
// v_mfma_f32_16x16x32_bf16 in fp32. The dropped terms (ml, lm, ll) are below 2^-24
// relative, so G matches an fp32 GEMM to fp32 rounding, at 6/16 of the fp32-MFMA cost.
// No LDS in the main loop: lane (r, g) loads VW consecutive columns of rows 8g..8g+7 of
// a 32-row step for both operands; element e of the VW columns is the operand of n-tile
// (or k-tile) e, so a 16*VW-wide tile needs no transpose (VW = 3: 48-wide tiles, which
// divide the Conformer widths 144 / 576; VW = 4: 64-wide).
// Fragment map of v_mfma_f32_16x16x32_bf16 (lane l, r = l&15, g = l>>4):
//   A[i=r][kk=8g+j], B[kk=8g+j][col=r], D[row=4g+reg][col=r].
//
// OB_GEMM=f32 selects the fp32 kernel (v_mfma_f32_16x16x4_f32, exact fp32 fma chain):
// A[i=r][kk=g], B[kk=g][j=r]; every lane loads 4 contiguous fp32 (one dwordx4) of a row.
#include <cstdlib>

#include "ob_launch.h"
#include "ob_quant.h"

namespace ob {

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kThreads = 256;  // 4 waves

// Bijective XCD-aware remap (cdna_hip_programming.md §5): consecutive logical ids land on
// one XCD under round-robin dispatch (hardware block b runs on XCD b % 8).
__device__ __forceinline__ int xcd_logical(int b, int nb) {
  const int q = nb / 8, r = nb % 8, x = b % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

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
    int64_t tiles_k, int64_t rows_per_chunk, int64_t cpp, float* __restrict__ part,
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
  // chunk -> (pass, chunk of the pass); M is the row count of one pass
  const int64_t chunk = blockIdx.y;
  const int64_t pass = chunk / cpp;
  const int64_t m_lim = (pass + 1) * M;
  const int64_t m_begin = pass * M + (chunk - pass * cpp) * rows_per_chunk;
  const int64_t m_end = (m_begin + rows_per_chunk < m_lim) ? m_begin + rows_per_chunk : m_lim;
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

// ---------------------------------------------------------------------------------
// dW partial, bf16x6: part[c][n][k] = sum_{m in chunk c} dY[m][n] * X[m][k].
// Block = one (16VW x 16VW) output tile x one M chunk of 4*S*32 rows; wave w takes the
// 32-row steps w, w+4, ...; the 4 wave tiles are summed in wave order through LDS.
// ---------------------------------------------------------------------------------
__device__ __forceinline__ f32x4 mfma_bf16(const bf16x8& a, const bf16x8& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// Buffer descriptor over [base, base + bytes): loads past the end return 0 (hardware
// range check), which zero-fills the rows past M without any per-lane test.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const float* base, int64_t bytes) {
  const uint32_t nrec = bytes > 0xFFFFFFF0ll ? 0xFFFFFFF0u : (uint32_t)bytes;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, (int)nrec,
                                           0x00020000);
}

// 4 fp32 -> 8-lane bf16 fragments, split exactly: x = hi + mid + lo.
template <int VW>
__device__ __forceinline__ void split_col(const f32x4 (&rows)[8], int e, bf16x8& hi, bf16x8& mid,
                                          bf16x8& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float x = rows[j][e];
    const __bf16 h = (__bf16)x;
    const float r1 = x - (float)h;
    const __bf16 m = (__bf16)r1;
    const float r2 = r1 - (float)m;
    hi[j] = h;
    mid[j] = m;
    lo[j] = (__bf16)r2;
  }
}

// Requires N % 4 == 0, K % 4 == 0 (dwordx4 rows); other shapes take the fp32 kernel.
// Lane (r, g) loads columns n0+4r..4r+3 (dY) and k0+4r..4r+3 (X) of rows 8g..8g+7 of a
// 32-row step: element e is the operand of n-tile (k-tile) e. Out-of-range rows read 0
// from the buffer descriptor; out-of-range columns only feed outputs that are never
// stored, so the main loop has no masks. Row and step offsets are scalar (soffset).
template <int S>
__global__ __launch_bounds__(kThreads, 2) void dw_bf16x6_kernel(
    const float* __restrict__ dY, const float* __restrict__ X, int64_t M, int N, int K,
    int tiles_n_arg, int tiles_k, int64_t rows_per_chunk, int64_t cpp, float* __restrict__ part,
    float* __restrict__ part_db, uint32_t* __restrict__ ticket) {
  constexpr int VW = 4, T = 64;
  __shared__ float red[2][T * T];
  __shared__ float dbred[4][T];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 15;
  const int g = lane >> 4;
  // 1-D grid, XCD-aware: consecutive logical ids (the tiles of one row chunk) run on one
  // XCD, so the chunk's dY/X rows are fetched into one L2 and re-read from there by all
  // its tiles (dispatch order x % 8 -> XCD; a chunk-major 2-D grid spread each chunk over
  // all 8 L2s: 19% L2 hit rate, measured).
  const int tiles = tiles_n_arg * tiles_k;
  const int L = xcd_logical((int)blockIdx.x, (int)gridDim.x);
  const int tile = L % tiles;
  const int tn = tile / tiles_k;
  const int tk = tile - tn * tiles_k;
  const int n0 = tn * T, k0 = tk * T;
  // chunk -> (pass, chunk of the pass); M is the row count of one pass
  const int64_t chunk = L / tiles;
  const int64_t pass = chunk / cpp;
  const int64_t m_lim = (pass + 1) * M;
  const int64_t m_begin = pass * M + (chunk - pass * cpp) * rows_per_chunk;
  const bool do_db = (part_db != nullptr) && (tk == 0);
  if (blockIdx.x == 0 && threadIdx.x == 0) *ticket = 0u;

  // Descriptors start at the chunk's first row and end at its pass's last row (rows past
  // it read 0), so every offset fits 32 bits.
  const __amdgpu_buffer_rsrc_t ry = make_rsrc(dY + m_begin * N, (m_lim - m_begin) * N * 4);
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(X + m_begin * K, (m_lim - m_begin) * K * 4);
  // Column offset clamped into the row (columns past N / K feed discarded outputs).
  const int nb = n0 + 4 * r < N - 4 ? n0 + 4 * r : N - 4;
  const int kb = k0 + 4 * r < K - 4 ? k0 + 4 * r : K - 4;
  const int voff_y = (8 * g * N + nb) * 4;
  const int voff_x = (8 * g * K + kb) * 4;

  f32x4 acc[VW][VW];
#pragma unroll
  for (int e = 0; e < VW; ++e)
#pragma unroll
    for (int f = 0; f < VW; ++f) acc[e][f] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 dbacc = {0.f, 0.f, 0.f, 0.f};

  struct Step {
    f32x4 dy[8];
    f32x4 x[8];
  };
  auto load = [&](int row0, Step& st) {  // row0: chunk-relative first row of the step
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      st.dy[j] = __builtin_amdgcn_raw_buffer_load_b128(ry, voff_y, (row0 + j) * N * 4, 0);
      st.x[j] = __builtin_amdgcn_raw_buffer_load_b128(rx, voff_x, (row0 + j) * K * 4, 0);
    }
  };
  auto compute = [&](const Step& st) {
    bf16x8 ah[VW], am[VW], al[VW];
#pragma unroll
    for (int e = 0; e < VW; ++e) split_col<VW>(st.dy, e, ah[e], am[e], al[e]);
    if (do_db) {
#pragma unroll
      for (int j = 0; j < 8; ++j) dbacc += st.dy[j];
    }
    // Product-major order: the VW MFMAs of one product term go to VW different
    // accumulators, so no MFMA waits on the one just issued (the e-major order chained six
    // dependent MFMAs per accumulator: 36% of wave time in issue stalls, measured).
#pragma unroll
    for (int f = 0; f < VW; ++f) {
      bf16x8 bh, bm, bl;
      split_col<VW>(st.x, f, bh, bm, bl);
#pragma unroll
      for (int e = 0; e < VW; ++e) acc[e][f] = mfma_bf16(am[e], bm, acc[e][f]);  // smallest first
#pragma unroll
      for (int e = 0; e < VW; ++e) acc[e][f] = mfma_bf16(al[e], bh, acc[e][f]);
#pragma unroll
      for (int e = 0; e < VW; ++e) acc[e][f] = mfma_bf16(ah[e], bl, acc[e][f]);
#pragma unroll
      for (int e = 0; e < VW; ++e) acc[e][f] = mfma_bf16(am[e], bh, acc[e][f]);
#pragma unroll
      for (int e = 0; e < VW; ++e) acc[e][f] = mfma_bf16(ah[e], bm, acc[e][f]);
#pragma unroll
      for (int e = 0; e < VW; ++e) acc[e][f] = mfma_bf16(ah[e], bh, acc[e][f]);
    }
  };

  // S steps per wave (wave w: steps w, w+4, ... of the chunk), one step in flight ahead.
  const int r0 = 32 * wave;
  Step bufA, bufB;
  load(r0, bufA);
#pragma unroll
  for (int i = 0; i < S; i += 2) {
    if (i + 1 < S) load(r0 + 128 * (i + 1), bufB);
    __builtin_amdgcn_sched_barrier(0);
    compute(bufA);
    if (i + 1 < S) {
      if (i + 2 < S) load(r0 + 128 * (i + 2), bufA);
      __builtin_amdgcn_sched_barrier(0);
      compute(bufB);
    }
  }

  // Combine the 4 wave tiles in a fixed order: (w0 + w2) + (w1 + w3).
  // Tile (e,f) D[row=4g+reg][col=r] -> G[n0 + 4*(4g+reg) + e][k0 + 4*r + f].
  float* myred = red[wave & 1];
  auto tile_index = [&](int e, int f, int reg) { return (VW * (4 * g + reg) + e) * T + VW * r + f; };
  if (wave >= 2) {
#pragma unroll
    for (int e = 0; e < VW; ++e)
#pragma unroll
      for (int f = 0; f < VW; ++f)
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) myred[tile_index(e, f, reg)] = acc[e][f][reg];
  }
  __syncthreads();
  if (wave < 2) {
#pragma unroll
    for (int e = 0; e < VW; ++e)
#pragma unroll
      for (int f = 0; f < VW; ++f)
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
          float* p = &myred[tile_index(e, f, reg)];
          *p = acc[e][f][reg] + *p;
        }
  }
  if (do_db) {
    // rows 8g..8g+7 of every step are in this lane's sums; add the 4 row groups in order
#pragma unroll
    for (int e = 0; e < VW; ++e) {
      float v = dbacc[e];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      dbacc[e] = v;
    }
    if (g == 0) {
#pragma unroll
      for (int e = 0; e < VW; ++e) dbred[wave][VW * r + e] = dbacc[e];
    }
  }
  __syncthreads();

  float* out = part + chunk * ((int64_t)N * K);
  for (int idx = threadIdx.x; idx < T * T; idx += kThreads) {
    const int nl = idx / T, kl = idx - nl * T;
    const int n = n0 + nl, k = k0 + kl;
    if (n < N && k < K) out[(int64_t)n * K + k] = red[0][idx] + red[1][idx];
  }
  if (do_db && threadIdx.x < T) {
    const int n = n0 + threadIdx.x;
    if (n < N) {
      const int i = threadIdx.x;
      part_db[chunk * N + n] = ((dbred[0][i] + dbred[1][i]) + dbred[2][i]) + dbred[3][i];
    }
  }
}

bool use_f32_dw() {
  static const int v = [] {
    const char* e = getenv("OB_GEMM");
    return (e && e[0] == 'f') ? 1 : 0;
  }();
  return v != 0;
}

}  // namespace

DwPlan plan_dw(int64_t M, int64_t N, int64_t K) { return plan_dw_passes(1, M, N, K); }

DwPlan plan_dw_passes(int64_t P, int64_t Mp, int64_t N, int64_t K) {
  DwPlan p;
  const int64_t M = P * Mp;  // chunk length is chosen for the whole stacked M
  if (use_f32_dw() || N % 4 != 0 || K % 4 != 0 || N < 4 || K < 4) {
    p.variant = 0;
    p.tiles_n = N > 0 ? ceil_div(N, kDwTile) : 1;  // >= 1 so K = 0 still yields db
    p.tiles_k = K > 0 ? ceil_div(K, kDwTile) : 1;
    const int64_t tiles = p.tiles_n * p.tiles_k;
    int64_t steps = 32;  // chunk = S steps x 16 rows
    while (steps > 8 && tiles * ceil_div(M, 16 * steps) < 256) steps /= 2;
    p.rows_per_chunk = 16 * steps;
  } else {
    // 64-wide tiles (one dwordx4 per lane per row). 48-wide tiles (which divide 144 / 576
    // without waste) measured slower: three strided dword loads per row.
    p.variant = 4;
    const int64_t t = 16 * p.variant;
    p.tiles_n = N > 0 ? ceil_div(N, t) : 1;
    p.tiles_k = K > 0 ? ceil_div(K, t) : 1;
    const int64_t tiles = p.tiles_n * p.tiles_k;
    // Chunk = 4 waves x S steps x 32 rows, S in {2, 4, 8}: the longest chunk that still
    // gives >= 256 blocks (one per CU), so the partial slabs stay few.
    static const int64_t max_steps = [] {  // OB_DW_MAXSTEPS: tuning experiments
      const char* e = getenv("OB_DW_MAXSTEPS");
      return (int64_t)(e ? atoi(e) : 8);
    }();
    int64_t steps = max_steps;
    while (steps > 2 && tiles * ceil_div(M, 128 * steps) < 256) steps /= 2;
    p.rows_per_chunk = 128 * steps;
  }
  p.passes = P;
  p.rows_per_pass = Mp;
  p.chunks_per_pass = Mp > 0 ? ceil_div(Mp, p.rows_per_chunk) : 1;
  p.chunks = P * p.chunks_per_pass;
  return p;
}

void launch_dw_partial(const float* dY, const float* X, int64_t M, int64_t N, int64_t K,
                       const DwPlan& p, float* part, float* part_db, uint32_t* ticket,
                       hipStream_t s) {
  if (p.rows_per_pass == 0 || N == 0) return;
  M = p.rows_per_pass;  // kernels index rows per pass (M given = passes * rows_per_pass)
  dim3 grid((unsigned)(p.tiles_n * p.tiles_k), (unsigned)p.chunks);
  const bool vec = (N % 4 == 0) && (K % 4 == 0) && N >= 4 && K >= 4 &&
                   ((reinterpret_cast<uintptr_t>(dY) & 15) == 0) &&
                   ((reinterpret_cast<uintptr_t>(X) & 15) == 0);
#define OB_DW(V, S)                                                                        \
  hipLaunchKernelGGL((dw_partial_kernel<V, S>), grid, dim3(kThreads), 0, s, dY, X, M, N, K,   \
                     p.tiles_k, p.rows_per_chunk, p.chunks_per_pass, part, part_db, ticket)
#define OB_DW6(S)                                                                          \
  hipLaunchKernelGGL((dw_bf16x6_kernel<S>), dim3((unsigned)(p.tiles_n * p.tiles_k * p.chunks)), \
                     dim3(kThreads), 0, s, dY, X, M, (int)N, (int)K, (int)p.tiles_n,            \
                     (int)p.tiles_k, p.rows_per_chunk, p.chunks_per_pass, part, part_db, ticket)
  if (p.variant != 0) {
    const int64_t steps = p.rows_per_chunk / 128;
    if (steps == 16) OB_DW6(16);
    else if (steps == 8) OB_DW6(8);
    else if (steps == 4) OB_DW6(4);
    else OB_DW6(2);
    return;
  }
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
#undef OB_DW6
#undef OB_DW
}

}  // namespace ob
