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
#include <type_traits>

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


// ---------------------------------------------------------------------------------
// dW partial, LDS-shared bf16x6 (shapes with N % 48 == 0 and K % 48 == 0, i.e. every
// Conformer width). Block = WN x WK waves, wave (wn, wk) owns the 48x48 output sub-tile
// n0 + 48wn.., k0 + 48wk..; block tile BN x BK = 48WN x 48WK; one M chunk per block.
// Per 32-row step the block loads dY[32][BN] and X[32][BK] once (fp32, coalesced), splits
// every element ONCE into hi/mid/lo bf16 (round-to-nearest, exact: x = hi + mid + lo) and
// stores the planes column-major in LDS (column = 32 rows of one n or k, 64 B per plane,
// slot pitch 224 B = 3 planes + 32 B: conflict-free ds_read_b128 for the
// MFMA fragments; the three planes of a column sit side by side in its 224-B slot). Every
// wave then reads its 16x16x32 A / B fragments from LDS, so a split
// element feeds WK (dY) or WN (X) waves instead of being re-split per output tile (the
// register-only kernel above split each dY element 3x and each X element 9x at lin1).
// Double-buffered: step s+1 is split and stored while step s's MFMAs run; one barrier per
// step. Loader unit = 4 rows x 4 columns of one operand (row quad fastest across lanes:
// conflict-free ds_write_b64).
// ---------------------------------------------------------------------------------
#ifdef OB_DW_STAMPS
// diagnostic build only (tools/dw_stamps.py): per wave the cycles of the prologue, the
// steps' MFMA phases, split / LDS-store phases, load issue and barrier waits, the partial /
// alpha epilogue and the db epilogue, and s_memrealtime at start and end
__device__ uint64_t g_dw_stamps[8 * 4096];
__device__ uint64_t g_dw_rt[2 * 4096];
#define DW_DECL \
  uint64_t dw_t = __builtin_amdgcn_s_memtime(), dw_rt0 = __builtin_amdgcn_s_memrealtime(), \
           dw_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define DW_STAMP(k)                                     \
  do {                                                  \
    const uint64_t dw_n = __builtin_amdgcn_s_memtime(); \
    dw_acc[k] += dw_n - dw_t;                           \
    dw_t = dw_n;                                        \
  } while (0)
#define DW_WRITE                                                                        \
  {                                                                                     \
    const uint64_t dw_rt1 = __builtin_amdgcn_s_memrealtime();                           \
    const size_t dw_w = (size_t)blockIdx.x * (blockDim.x / 64) + wave;                  \
    if (lane == 0 && dw_w < 4096) {                                                     \
      for (int k_ = 0; k_ < 8; ++k_) g_dw_stamps[dw_w * 8 + k_] = dw_acc[k_];           \
      g_dw_rt[dw_w * 2] = dw_rt0;                                                       \
      g_dw_rt[dw_w * 2 + 1] = dw_rt1;                                                   \
    }                                                                                   \
  }
#else
#define DW_DECL
#define DW_STAMP(k) \
  do {              \
  } while (0)
#define DW_WRITE
#endif

constexpr int kLdsPitch = 224;  // bytes per column slot: 3 planes x 32 bf16 rows + 32 B pad
constexpr int kStepRows = 32;

template <int WN, int WK>
struct DwLdsCfg {
  static constexpr int BN = 48 * WN, BK = 48 * WK;
  static constexpr int kThr = 64 * WN * WK;
  static constexpr int kCols = BN + BK;                       // dY columns then X columns
  static constexpr int kBuf = kCols * kLdsPitch;              // one step, three planes
  static constexpr int kUY = (BN * 4 + kThr - 1) / kThr;      // dY loader units per thread
  static constexpr int kUX = (BK * 4 + kThr - 1) / kThr;      // X loader units per thread
};

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

// Round two fp32 to bf16 (v_cvt_pk_bf16_f32), packed (a low, b high); also returns the two
// rounded values as fp32.
__device__ __forceinline__ uint32_t cvt2(float a, float b, float& ra, float& rb) {
  const bf16x2 v = __builtin_convertvector(f32x2{a, b}, bf16x2);
  const uint32_t u = __builtin_bit_cast(uint32_t, v);
  ra = __uint_as_float(u << 16);
  rb = __uint_as_float(u & 0xFFFF0000u);
  return u;
}

constexpr int kProdA[6] = {1, 2, 0, 1, 0, 0};  // plane of A per product: mm lh hl mh hm hh
constexpr int kProdB[6] = {1, 0, 2, 0, 1, 0};

// Layers sharing X (q / k / v of one LN output: dW_i = dY_i^T X) in one launch: the n-tiles
// of layer i follow those of layer i-1, and a block reads dY / writes the partials of its
// tile's layer. Every per-layer quantity (partial slab, db partials, alpha partial at
// (chunk, layer-local tile)) has the single-layer layout, so the finish is unchanged.
struct DwLdsGroup {
  const float* dY[kMaxDwGroup];
  float* part[kMaxDwGroup];
  float* part_db[kMaxDwGroup];
  DwAlpha al[kMaxDwGroup];
  int layers;
  // deferred finish: block 0 writes ent[0 .. layers) to table[slot ..] (table == nullptr: off)
  DwFinishEntry* table;
  int slot;
  DwFinishEntry ent[kMaxDwGroup];
};

template <int WN, int WK>
__global__ __launch_bounds__(64 * WN * WK) void dw_lds_kernel(
    const float* __restrict__ X, int64_t M, int N, int K, int tiles_k, int64_t rows_per_chunk,
    int64_t cpp, DwLdsGroup grp) {
  using C = DwLdsCfg<WN, WK>;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wn = wave / WK, wk = wave - wn * WK;
  DW_DECL
  const int r = lane & 15, g = lane >> 4;
  const int tiles_nl = N / C::BN;  // n-tiles of one layer
  const int tiles = grp.layers * tiles_nl * tiles_k;
  const int L = xcd_logical((int)blockIdx.x, (int)gridDim.x);
  const int tile = L % tiles;
  const int tng = tile / tiles_k, tk = tile - tng * tiles_k;
  const int layer = tng / tiles_nl, tn = tng - layer * tiles_nl;
  const float* __restrict__ dY = grp.dY[layer];
  float* __restrict__ part = grp.part[layer];
  float* __restrict__ part_db = grp.part_db[layer];
  const DwAlpha& al = grp.al[layer];
  const int n0 = tn * C::BN, k0 = tk * C::BK;
  const int64_t chunk = L / tiles;
  const int64_t pass = chunk / cpp;
  const int64_t m_lim = (pass + 1) * M;
  const int64_t m_begin = pass * M + (chunk - pass * cpp) * rows_per_chunk;
  const int64_t m_end = m_begin + rows_per_chunk < m_lim ? m_begin + rows_per_chunk : m_lim;
  const int steps = (int)((m_end - m_begin + kStepRows - 1) / kStepRows);
  if (grp.table && blockIdx.x == 0 && (int)threadIdx.x < grp.layers)
    grp.table[grp.slot + threadIdx.x] = grp.ent[threadIdx.x];
  const bool do_db = (part_db != nullptr) && (tk == 0);

  // Loader units: 2 rows x 4 columns of one operand, row pair fastest across lanes
  // (conflict-free ds_write_b32: the two columns a 32-lane group writes sit 32 banks
  // apart). Every thread owns UY dY units and UX X units, so each load instruction reads one
  // operand through one wave-uniform buffer descriptor (a per-lane choice compiles to a
  // waterfall loop). Rows at or past the chunk end read 0 (range check).
  const __amdgpu_buffer_rsrc_t ry = make_rsrc(dY + m_begin * N, (m_end - m_begin) * N * 4);
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(X + m_begin * K, (m_end - m_begin) * K * 4);
  constexpr int UY = C::kUY, UX = C::kUX;
  int y_voff[UY], y_c[UY], y_rp[UY], x_voff[UX], x_c[UX], x_rp[UX];
  bool y_ok[UY], x_ok[UX];
#pragma unroll
  for (int j = 0; j < UY; ++j) {
    const int u = threadIdx.x + j * C::kThr;
    y_ok[j] = u < C::BN * 4;           // (BN/4 column quads) x 16 row pairs
    const int uu = y_ok[j] ? u : 0;
    y_rp[j] = uu & 15;
    y_c[j] = 4 * (uu >> 4);
    y_voff[j] = (2 * y_rp[j] * N + n0 + y_c[j]) * 4;
  }
#pragma unroll
  for (int j = 0; j < UX; ++j) {
    const int u = threadIdx.x + j * C::kThr;
    x_ok[j] = u < C::BK * 4;
    const int uu = x_ok[j] ? u : 0;
    x_rp[j] = uu & 15;
    x_c[j] = 4 * (uu >> 4);
    x_voff[j] = (2 * x_rp[j] * K + k0 + x_c[j]) * 4;
  }
  struct Raw {
    f32x4 y[UY][2];
    f32x4 x[UX][2];
  };
  auto load = [&](Raw& raw, int step) {
    const int soy = step * kStepRows * N * 4, sox = step * kStepRows * K * 4;
#pragma unroll
    for (int j = 0; j < UY; ++j)
      if (y_ok[j])
#pragma unroll
        for (int i = 0; i < 2; ++i)
          raw.y[j][i] = __builtin_amdgcn_raw_buffer_load_b128(ry, y_voff[j] + i * N * 4, soy, 0);
#pragma unroll
    for (int j = 0; j < UX; ++j)
      if (x_ok[j])
#pragma unroll
        for (int i = 0; i < 2; ++i)
          raw.x[j][i] = __builtin_amdgcn_raw_buffer_load_b128(rx, x_voff[j] + i * K * 4, sox, 0);
  };
  f32x4 dbacc[UY];
#pragma unroll
  for (int j = 0; j < UY; ++j) dbacc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // split x = hi + mid + lo (each the bf16 rounding of what is left; exact) and store the
  // three planes of a 2-row x 4-column unit (one packed row pair per plane and column)
  auto put = [&](unsigned char* base, int col, int rp, const f32x4& r0, const f32x4& r1) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float h0, h1, m0, m1, l0, l1;
      const uint32_t ph = cvt2(r0[e], r1[e], h0, h1);
      const float s0 = r0[e] - h0, s1 = r1[e] - h1;
      const uint32_t pm = cvt2(s0, s1, m0, m1);
      const uint32_t pl = cvt2(s0 - m0, s1 - m1, l0, l1);
      unsigned char* cb = base + (col + e) * kLdsPitch + rp * 4;
      *reinterpret_cast<uint32_t*>(cb) = ph;
      *reinterpret_cast<uint32_t*>(cb + 64) = pm;
      *reinterpret_cast<uint32_t*>(cb + 128) = pl;
    }
  };
  auto store = [&](const Raw& raw, int buf) {
    unsigned char* base = lds + buf * C::kBuf;
#pragma unroll
    for (int j = 0; j < UY; ++j) {
      if (!y_ok[j]) continue;
      if (do_db) dbacc[j] += raw.y[j][0] + raw.y[j][1];
      put(base, y_c[j], y_rp[j], raw.y[j][0], raw.y[j][1]);
    }
#pragma unroll
    for (int j = 0; j < UX; ++j)
      if (x_ok[j]) put(base, C::BN + x_c[j], x_rp[j], raw.x[j][0], raw.x[j][1]);
  };

  f32x4 acc[3][3];
#pragma unroll
  for (int t = 0; t < 3; ++t)
#pragma unroll
    for (int u = 0; u < 3; ++u) acc[t][u] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto frag = [&](const unsigned char* base, int col, int plane) {
    return *reinterpret_cast<const bf16x8*>(base + col * kLdsPitch + 64 * plane + 16 * g);
  };
  auto compute = [&](int buf) {
    const unsigned char* base = lds + buf * C::kBuf;
    // B fragments (this wave's 3 k-tiles x 3 planes) for the whole step, A fragments one
    // n-tile at a time (register budget: 3 waves per SIMD); 16x16x32 bf16 MFMAs issue
    // back to back on one accumulator, so per tile row the products go
    // smallest first (mm, lh, hl, mh, hm, hh) over its 3 accumulators.
    bf16x8 b[3][3];
#pragma unroll
    for (int u = 0; u < 3; ++u)
#pragma unroll
      for (int q = 0; q < 3; ++q) b[u][q] = frag(base, C::BN + 48 * wk + 16 * u + r, q);
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      bf16x8 a[3];
#pragma unroll
      for (int q = 0; q < 3; ++q) a[q] = frag(base, 48 * wn + 16 * t + r, q);
#pragma unroll
      for (int p = 0; p < 6; ++p)
#pragma unroll
        for (int u = 0; u < 3; ++u)
          acc[t][u] = mfma_bf16(a[kProdA[p]], b[u][kProdB[p]], acc[t][u]);
    }
  };

  // Two register stages: step s+1's data is split into LDS while step s's MFMAs run, and
  // the loads of step s+2 / s+3 are already in flight (two steps of HBM latency covered).
  Raw ra, rb;
  load(ra, 0);
  if (steps > 1) load(rb, 1);
  store(ra, 0);
  if (steps > 2) load(ra, 2);
  __syncthreads();
  DW_STAMP(0);
  // Waves 0-3 compute before they store, waves 4.. store first (a stagger: the waves
  // sharing a SIMD -- w and w+4 -- then run their MFMA and their split/store phases at
  // different times instead of in lockstep between the barriers). Compute-first code issues
  // its fragment reads before the ds_writes (the compiler cannot tell the two buffers
  // apart and keeps program order).
  const bool late = wave >= 4;
  auto phase = [&](int cb, Raw& nxt, int sb, bool do_store, int ld_step) {
    if (late) {
      if (do_store) store(nxt, sb);
      DW_STAMP(2);
      compute(cb);
      DW_STAMP(1);
    } else {
      compute(cb);
      DW_STAMP(1);
      if (do_store) store(nxt, sb);
      DW_STAMP(2);
    }
    if (do_store && ld_step >= 0) load(nxt, ld_step);
    DW_STAMP(3);
  };
  for (int s = 0; s < steps; s += 2) {
    phase(0, rb, 1, s + 1 < steps, s + 3 < steps ? s + 3 : -1);
    __syncthreads();
    DW_STAMP(4);
    if (s + 1 >= steps) break;
    phase(1, ra, 0, s + 2 < steps, s + 4 < steps ? s + 4 : -1);
    __syncthreads();
    DW_STAMP(4);
  }
  // partial tile: D[row = 4g + reg][col = r] of tile (t, u) -> n = n0 + 48wn + 16t + 4g + reg,
  // k = k0 + 48wk + 16u + r. The same loop forms this block's share of the alpha gradient
  // (quant.py:84-91 is linear in G: sum_e G[e] term[e] = sum over chunks of the chunk
  // partial's dot with term), with the term at this chunk's pass bitwidth.
  // al.W == nullptr: a dense dW (dgemm.hip's pointwise convs) -- no alpha partials
  const bool has_al = al.W != nullptr;
  const float a = has_al ? effective_alpha(al.alpha, al.alpha_raw) : 1.0f;
  int bits = !has_al ? 2 : al.pass_bits ? al.pass_bits[pass] : (al.bits_dev ? *al.bits_dev : al.bits);
  bits = bits == 1 ? 1 : 2;
  float* out = part + chunk * ((int64_t)N * K);
  float prod = 0.0f;
  // two straight-line copies of the store loop (a per-element `if (has_al)` around the W
  // loads makes hipcc branch and wait for each load in turn)
  auto emit = [&](auto with_al) {
#pragma unroll
    for (int t = 0; t < 3; ++t)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int n = n0 + 48 * wn + 16 * t + 4 * g + reg;
#pragma unroll
        for (int u = 0; u < 3; ++u) {
          const int64_t e = (int64_t)n * K + k0 + 48 * wk + 16 * u + r;
          out[e] = acc[t][u][reg];
          if constexpr (decltype(with_al)::value)
            prod += acc[t][u][reg] * alpha_term(al.W[e] / a, bits);
        }
      }
  };
  if (has_al) emit(std::true_type{});
  else emit(std::false_type{});
  DW_STAMP(5);
  if (has_al) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) prod += __shfl_xor(prod, off, 64);
    float* wred = reinterpret_cast<float*>(lds) + 16 * C::BN;  // past the db scratch
    __syncthreads();  // (the loop's last barrier already ended all LDS reads)
    if (lane == 0) wred[wave] = prod;
    __syncthreads();
    if (threadIdx.x == 0) {
      float t = 0.0f;
      for (int w = 0; w < WN * WK; ++w) t += wred[w];
      // (chunk, layer-local tile): the finish kernel sums these in order
      al.apart[chunk * (tiles_nl * tiles_k) + tn * tiles_k + tk] = t;
    }
  }
  if (do_db) {
    // column sums: the 16 row pairs of each column quad, added in row-pair order via LDS
    float* red = reinterpret_cast<float*>(lds);  // [16][BN] (the step buffers are free now)
#pragma unroll
    for (int j = 0; j < UY; ++j)
      if (y_ok[j])
#pragma unroll
        for (int e = 0; e < 4; ++e) red[y_rp[j] * C::BN + y_c[j] + e] = dbacc[j][e];
    __syncthreads();
    for (int c = threadIdx.x; c < C::BN; c += C::kThr) {
      float v = 0.0f;
#pragma unroll
      for (int q = 0; q < 16; ++q) v += red[q * C::BN + c];
      part_db[chunk * N + n0 + c] = v;
    }
  }
  DW_STAMP(6);
  DW_WRITE
}


// ---------------------------------------------------------------------------------
// Finish of the LDS dW path (quant.py:80-91 given the chunk partials): dW[e] = (sum over
// chunks of part[c][e]) * 1[|W/a| <= 1], db = the same over part_db; the extra last block
// sums the dW blocks' alpha partials in logical-block order. Block = 64 elements x 4 chunk
// slices (slice q: chunks q, q+4, ... in order, 8 loads in flight), the slices added in a
// fixed order through LDS: deterministic, no atomics, and 4x the blocks of one element per
// thread (82 blocks for a 144 x 144 weight left most CUs idle: 6.4 us per launch).
// ---------------------------------------------------------------------------------
constexpr int kFinSlices = 4, kFinElems = kThreads / kFinSlices;
// One finish (chunk sum + STE mask, db, dalpha) as block `bid` of `nb` blocks.
__device__ __forceinline__ void dw_finish_body(const DwFinish& a, int bid, int nb) {
  if (bid == nb - 1) {  // alpha: fixed order over the dW blocks
    if (threadIdx.x >= 64 || !a.dalpha) return;  // (no alpha: a dense dW)
    float s2 = 0.0f;
    for (int i = threadIdx.x; i < a.n_apart; i += 64) s2 += a.apart[i];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) s2 += __shfl_xor(s2, off, 64);
    if (threadIdx.x == 0) a.dalpha[0] = s2 * alpha_chain(a.alpha, a.alpha_raw);
    return;
  }
  __shared__ float red[kFinSlices][kFinElems];
  const int el = threadIdx.x % kFinElems, sl = threadIdx.x / kFinElems;
  const int64_t nk = a.nk, n_db = a.n_db;
  const int chunks = a.chunks;
  const int64_t e = (int64_t)bid * kFinElems + el;
  const bool is_w = e < nk;
  const bool live = e < nk + n_db;
  const float* src = is_w ? a.part + e : a.part_db + (live ? e - nk : 0);
  const int64_t stride = is_w ? nk : n_db;
  constexpr int G = 8;
  float cur[G], nxt[G];
  auto fetch = [&](int c0, float (&v)[G]) {  // chunks c0 + kFinSlices * u of this slice
#pragma unroll
    for (int u = 0; u < G; ++u) {
      const int c = c0 + kFinSlices * u;
      v[u] = (live && c < chunks) ? src[(int64_t)c * stride] : 0.0f;
    }
  };
  float g = 0.0f;
  fetch(sl, cur);
  for (int c0 = sl; c0 < chunks; c0 += kFinSlices * G) {
    if (c0 + kFinSlices * G < chunks) fetch(c0 + kFinSlices * G, nxt);
#pragma unroll
    for (int u = 0; u < G; ++u)
      if (c0 + kFinSlices * u < chunks) g += cur[u];
#pragma unroll
    for (int u = 0; u < G; ++u) cur[u] = nxt[u];
  }
  red[sl][el] = g;
  __syncthreads();
  if (sl != 0 || !live) return;
  g = (red[0][el] + red[1][el]) + (red[2][el] + red[3][el]);
  if (is_w && !a.W) {
    a.dW[e] = g;  // dense dW (W == nullptr)
  } else if (is_w) {
    const float al = effective_alpha(a.alpha, a.alpha_raw);
    a.dW[e] = g * ste_indicator(a.W[e] / al);  // quant.py:81-82
  } else {
    a.db[e - nk] = g;
  }
}

int64_t finish_blocks(const DwFinish& a) { return ceil_div(a.nk + a.n_db, kFinElems) + 1; }

// Every deferred finish of a backward in one launch: block b runs the finish of the table
// entry whose [start, next start) holds b (binary search over the starts; the entries are in
// slot order with increasing starts).
__global__ __launch_bounds__(kThreads) void dw_finish_table_kernel(
    const DwFinishEntry* __restrict__ tab, int n, int64_t total) {
  const int64_t b = blockIdx.x;
  int lo = 0, hi = n - 1;
  while (lo < hi) {  // last entry with start <= b
    const int mid = (lo + hi + 1) >> 1;
    if (tab[mid].start <= b) lo = mid;
    else hi = mid - 1;
  }
  const int64_t st = tab[lo].start;
  const int64_t end = lo + 1 < n ? tab[lo + 1].start : total;
  const DwFinish f = tab[lo].f;
  dw_finish_body(f, (int)(b - st), (int)(end - st));
}

__global__ __launch_bounds__(kThreads) void dw_finish_kernel(DwFinish a) {
  dw_finish_body(a, blockIdx.x, gridDim.x);
}

// Several layers' finishes in one launch (the q/k/v projections of one input): block ranges
// [start[i], start[i+1]) belong to layer i; each layer's arithmetic is unchanged.
struct DwFinishGroup {
  DwFinish g[kMaxDwGroup];
  int start[kMaxDwGroup + 1];
  int n;
};

__global__ __launch_bounds__(kThreads) void dw_finish_group_kernel(DwFinishGroup G) {
  const int b = blockIdx.x;
  int i = 0;
  while (i + 1 < G.n && b >= G.start[i + 1]) ++i;
  dw_finish_body(G.g[i], b - G.start[i], G.start[i + 1] - G.start[i]);
}


// ---------------------------------------------------------------------------------
// Grouped deferred dW, stream-K (ob_dw_grouped). Every deferred weight gradient of a
// backward (N, K multiples of 144) in ONE persistent launch after the backward. The work
// space is linear in steps -- gemm-major, then 144 x 144 tile, then pass, then 32-row step
// -- and block b (one 9-wave block per CU) owns steps [b W / nb, (b + 1) W / nb). It walks
// its range tile by tile with the dw_lds_kernel<3,3> main loop (same LDS planes, same six
// products), so each segment runs hundreds of steps instead of the 12 a per-layer split-M
// launch gave one block, and no per-layer prologue / epilogue / finish launch remains.
//   * A tile one block covers entirely is finished from that block's registers: dW = G *
//     1[|W/a| <= 1] (quant.py:80-82), db, the tile's alpha partial.
//   * A tile split between blocks (only the first and the last tile of a block's range, so
//     <= 2 slabs per block) is finished by the block whose ticket add arrives last; it sums
//     the segments' slabs in block order (the partition is static: deterministic).
//   * Alpha (quant.py:84-91) is linear in G, so a segment that crosses a pass boundary i adds
//     sum_e A_i[e] (term_{b_i}[e] - term_{b_i+1}[e]) there (A_i = its accumulator at the
//     boundary) and sum_e A[e] term_b[e] at its end: the telescoped sum over passes of each
//     pass's rows against the term at that pass's bitwidth. Tiles' partials are summed in tile
//     order by the last tile of the gemm (second ticket).
// Hand-offs are write-through: sc1 stores, every storing wave's vmcnt(0), the block barrier,
// one agent-scope ticket add; the last arriver reads every handed-off byte with sc1 loads
// (MI355X_MICROARCH.md, Valid forms, row 1). The last arriver resets its ticket to 0.
// ---------------------------------------------------------------------------------
constexpr int kDwgSlotF = kDwgTile * kDwgTile + 256;  // floats: tile (fragment order), db, alpha
constexpr int kDwgDb = kDwgTile * kDwgTile;
constexpr int kDwgAl = kDwgDb + kDwgTile;
constexpr unsigned kSc1 = 16;  // buffer cache policy: sc1 (write-through store / L1-bypass load)

__device__ __forceinline__ int dwg_start(int b, int nb, int W) {
  return (int)((long long)b * W / nb);
}
// the block whose range holds linear step x (the largest b with dwg_start(b) <= x; nb <= W)
__device__ __forceinline__ int dwg_owner(int x, int nb, int W) {
  return (int)(((long long)(x + 1) * nb - 1) / W);
}

// An opaque copy of x: values derived from it cannot be hoisted above this point (keeps the
// epilogue's per-lane addresses out of the main loop's registers: hoisted out of the segment
// loop they stayed live across it and spilled the main loop).
// fp32 through the 32-bit buffer builtins (they move integers: bit-cast, not convert)
__device__ __forceinline__ float ld_f32(__amdgpu_buffer_rsrc_t r, int voff) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, 0, 0));
}
__device__ __forceinline__ void st_f32(float v, __amdgpu_buffer_rsrc_t r, int voff) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, voff, 0, 0);
}

__device__ __forceinline__ int opaque(int x) {
  asm volatile("" : "+v"(x));
  return x;
}

// 8 waves, two per SIMD: per 32-row step a SIMD issues the MFMAs of 21 or 20 16 x 16
// sub-tiles, against 27 on the busiest SIMD of the 9-wave dw_lds tiling (3/2/2/2 waves), and a
// wave may use 256 registers, which leaves the segment loop room (the 9-wave main loop needs
// all of its 168 and spilled inside the loop nest). Wave w owns the 3 x 3 block (w / 3, w % 3)
// of the 144 x 144 tile's 9 x 9 sub-tiles and sub-tile w of the ninth block (2, 2); wave 7 also
// owns that block's last sub-tile (8, 8).
constexpr int kDwgWaves = 8, kDwgThreads = 64 * kDwgWaves;
constexpr int kDwgBuf = 2 * kDwgTile * kLdsPitch;  // one step: dY columns, then X columns
constexpr int kDwgLds = 2 * kDwgBuf + 16 * kDwgTile * 4 + 16;

__global__ __launch_bounds__(kDwgThreads) void dw_grouped_kernel(
    const DwgDesc* __restrict__ descs, int G, int Wtot, float* __restrict__ slots,
    float* __restrict__ talpha, uint32_t* __restrict__ tickets, int total_tiles) {
  constexpr int BN = kDwgTile;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int bn = wave / 3, bk = wave - 3 * bn;  // main 3 x 3 block of sub-tiles
  const int tie = 6 + bn, tue = 6 + bk;         // extra sub-tile of block (2, 2)
  const bool two = wave == 7;                   // wave 7: also sub-tile (8, 8)
  const int r = lane & 15, g = lane >> 4;
  const int nb = gridDim.x, blk = blockIdx.x;
  const int beg = dwg_start(blk, nb, Wtot), end = dwg_start(blk + 1, nb, Wtot);
  // LDS: two step buffers, the db column partials [16 row pairs][144], a flag
  float* const s_db = reinterpret_cast<float*>(lds + 2 * kDwgBuf);
  int* const s_flag = reinterpret_cast<int*>(lds + 2 * kDwgBuf + 16 * kDwgTile * 4);
  float* const fl = reinterpret_cast<float*>(lds);  // epilogue scratch (step buffers free)
  // loader units (2 rows x 4 columns of each operand): unit tid, and for wave 0 also unit
  // 512 + tid (576 units per operand)
  const bool u2 = wave == 0;
  const int rp0 = threadIdx.x & 15, cq0 = 4 * (threadIdx.x >> 4);
  const int cq1 = 128 + cq0;  // the second unit (wave 0): same row pair, columns 128..143

  int gi = 0;  // the gemm holding `beg`
  {
    int lo = 0, hi = G - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (descs[mid].work0 <= beg) lo = mid;
      else hi = mid - 1;
    }
    gi = lo;
  }

  auto put = [&](unsigned char* base, int col, const f32x4& r0, const f32x4& r1) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float h0, h1, m0, m1, l0, l1;
      const uint32_t ph = cvt2(r0[e], r1[e], h0, h1);
      const float s0 = r0[e] - h0, s1 = r1[e] - h1;
      const uint32_t pm = cvt2(s0, s1, m0, m1);
      const uint32_t pl = cvt2(s0 - m0, s1 - m1, l0, l1);
      unsigned char* cb = base + (col + e) * kLdsPitch + rp0 * 4;
      *reinterpret_cast<uint32_t*>(cb) = ph;
      *reinterpret_cast<uint32_t*>(cb + 64) = pm;
      *reinterpret_cast<uint32_t*>(cb + 128) = pl;
    }
  };
  auto frag = [&](const unsigned char* base, int col, int plane) {
    return *reinterpret_cast<const bf16x8*>(base + col * kLdsPitch + 64 * plane + 16 * g);
  };

  int pos = beg;
  while (pos < end) {
    const DwgDesc& d = descs[gi];
    const int tsteps = d.P * d.spp;
    if (pos >= (int)d.work0 + tsteps * d.tiles) {
      ++gi;
      continue;
    }
    const int t = (pos - (int)d.work0) / tsteps;
    const int T0 = (int)d.work0 + t * tsteps, T1 = T0 + tsteps;
    const int send = end < T1 ? end : T1;
    const int N = d.N, K = d.K, Mp = d.Mp, spp = d.spp;
    const int tn = t / d.tiles_k, tk = t - tn * d.tiles_k;
    const int n0 = tn * kDwgTile, k0 = tk * kDwgTile;
    const bool has_al = d.W != nullptr;
    const bool do_db = d.db != nullptr && tk == 0;
    const float a = has_al ? effective_alpha(d.alpha, d.alpha_raw) : 1.0f;
    const __amdgpu_buffer_rsrc_t rw = make_rsrc(d.W, has_al ? (int64_t)N * K * 4 : 0);
    auto pass_bits = [&](int p) {
      const int b = d.pass_bits ? d.pass_bits[p] : d.bits;
      return b == 1 ? 1 : 2;
    };

    f32x4 acc[3][3], acce[2];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int u = 0; u < 3; ++u) acc[i][u] = f32x4{0.f, 0.f, 0.f, 0.f};
    acce[0] = acce[1] = f32x4{0.f, 0.f, 0.f, 0.f};
    // fn(accumulator, sub-tile row ti, sub-tile column tu) for every sub-tile of this wave
    auto for_tiles = [&](auto&& fn) {
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int u = 0; u < 3; ++u) fn(acc[i][u], 3 * bn + i, 3 * bk + u);
      fn(acce[0], tie, tue);
      if (two) fn(acce[1], 8, 8);
    };
    // byte offset of element (reg 0) of this lane in sub-tile (ti, tu): row 16 ti + 4g + reg,
    // column 16 tu + r (D[row = 4g + reg][col = r]); formed from an opaque lane id where used
    auto elem_base = [&]() {
      const int ln = opaque(lane);
      return ((n0 + 4 * (ln >> 4)) * K + k0 + (ln & 15)) * 4;
    };
    float aprod = 0.0f;
    // sum over this wave's elements of acc * (term_b1(W/a) - term_b2(W/a)) (b2 = 0: none)
    auto alpha_dot = [&](int b1, int b2) {
      const int eb = elem_base();
      for_tiles([&](f32x4& ac, int ti, int tu) {
        float w[4];
#pragma unroll
        for (int reg = 0; reg < 4; ++reg)
          w[reg] = ld_f32(rw, eb + ((16 * ti + reg) * K + 16 * tu) * 4);
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
          const float wa = w[reg] / a;
          aprod += ac[reg] * (alpha_term(wa, b1) - (b2 ? alpha_term(wa, b2) : 0.0f));
        }
      });
    };
    // db: each thread sums its units' columns into thread-private LDS slots
    f32x4* const db0 = reinterpret_cast<f32x4*>(s_db + rp0 * kDwgTile + cq0);
    f32x4* const db1 = reinterpret_cast<f32x4*>(s_db + rp0 * kDwgTile + cq1);

    __syncthreads();  // the previous segment's epilogue scratch is free
    if (do_db) {
      *db0 = f32x4{0.f, 0.f, 0.f, 0.f};
      if (u2) *db1 = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    int j = pos - T0;
    const int j1 = send - T0;
    while (j < j1) {
      // one pass piece: rows [r0, r1) of pass p
      const int p = j / spp;
      const int je = j1 < (p + 1) * spp ? j1 : (p + 1) * spp;
      const int r0 = p * Mp + (j - p * spp) * kStepRows;
      const int rl = p * Mp + (je - p * spp) * kStepRows;
      const int r1 = rl < (p + 1) * Mp ? rl : (p + 1) * Mp;
      const int steps = je - j;
      const __amdgpu_buffer_rsrc_t ry =
          make_rsrc(d.dY + (int64_t)r0 * N, (int64_t)(r1 - r0) * N * 4);
      const __amdgpu_buffer_rsrc_t rx =
          make_rsrc(d.X + (int64_t)r0 * K, (int64_t)(r1 - r0) * K * 4);
      // the second unit through descriptors of length 0 outside wave 0: those loads return 0
      // without touching memory, and every wave issues the same loads (a wave-dependent load
      // count made the compiler wait for all of them at every step)
      const __amdgpu_buffer_rsrc_t ry2 = u2 ? ry : make_rsrc(d.dY, 0);
      const __amdgpu_buffer_rsrc_t rx2 = u2 ? rx : make_rsrc(d.X, 0);
      const int yv0 = (2 * rp0 * N + n0 + cq0) * 4, xv0 = (2 * rp0 * K + k0 + cq0) * 4;
      struct Raw {
        f32x4 y[2][2];  // [unit][row]
        f32x4 x[2][2];
      };
      auto load = [&](Raw& raw, int step) {
        const int soy = step * kStepRows * N * 4, sox = step * kStepRows * K * 4;
#pragma unroll
        for (int i = 0; i < 2; ++i) {  // (row offset in soffset)
          raw.y[0][i] = __builtin_amdgcn_raw_buffer_load_b128(ry, yv0, soy + i * N * 4, 0);
          raw.x[0][i] = __builtin_amdgcn_raw_buffer_load_b128(rx, xv0, sox + i * K * 4, 0);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          raw.y[1][i] = __builtin_amdgcn_raw_buffer_load_b128(ry2, yv0 + 512, soy + i * N * 4, 0);
          raw.x[1][i] = __builtin_amdgcn_raw_buffer_load_b128(rx2, xv0 + 512, sox + i * K * 4, 0);
        }
      };
      auto store = [&](const Raw& raw, int buf) {
        unsigned char* base = lds + buf * kDwgBuf;
        if (do_db) *db0 = *db0 + (raw.y[0][0] + raw.y[0][1]);
        put(base, cq0, raw.y[0][0], raw.y[0][1]);
        put(base, BN + cq0, raw.x[0][0], raw.x[0][1]);
        if (u2) {
          if (do_db) *db1 = *db1 + (raw.y[1][0] + raw.y[1][1]);
          put(base, cq1, raw.y[1][0], raw.y[1][1]);
          put(base, BN + cq1, raw.x[1][0], raw.x[1][1]);
        }
      };
      auto compute = [&](int buf) {
        const unsigned char* base = lds + buf * kDwgBuf;
        bf16x8 bq[3][3];
#pragma unroll
        for (int u = 0; u < 3; ++u)
#pragma unroll
          for (int q = 0; q < 3; ++q) bq[u][q] = frag(base, BN + 48 * bk + 16 * u + r, q);
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          bf16x8 aq[3];
#pragma unroll
          for (int q = 0; q < 3; ++q) aq[q] = frag(base, 48 * bn + 16 * i + r, q);
#pragma unroll
          for (int pr = 0; pr < 6; ++pr)
#pragma unroll
            for (int u = 0; u < 3; ++u)
              acc[i][u] = mfma_bf16(aq[kProdA[pr]], bq[u][kProdB[pr]], acc[i][u]);
        }
        bf16x8 ae[3], be[3];
#pragma unroll
        for (int q = 0; q < 3; ++q) ae[q] = frag(base, 16 * tie + r, q);
#pragma unroll
        for (int q = 0; q < 3; ++q) be[q] = frag(base, BN + 16 * tue + r, q);
#pragma unroll
        for (int pr = 0; pr < 6; ++pr) acce[0] = mfma_bf16(ae[kProdA[pr]], be[kProdB[pr]], acce[0]);
        if (two) {
#pragma unroll
          for (int q = 0; q < 3; ++q) be[q] = frag(base, BN + 16 * 8 + r, q);
#pragma unroll
          for (int pr = 0; pr < 6; ++pr)
            acce[1] = mfma_bf16(ae[kProdA[pr]], be[kProdB[pr]], acce[1]);
        }
      };
      // Every phase issues its loads unconditionally: steps past the piece read zeros through
      // the descriptors' range check (no memory traffic). With the loads conditional the
      // compiler's wait counts had to cover the path without them, and each store then
      // waited for the NEXT step's loads too (one step of prefetch instead of two).
      // The next step's split and LDS store first, then this step's MFMAs: the split's VALU
      // runs while this step's fragment reads are in flight (compute-then-store measured
      // 2.5 % slower per launch; interleaving them with sched_group_barrier, no better:
      // profiles/r5/dwg_sched/). The two touch different LDS buffers.
      auto phase = [&](int cb, Raw& nxt, int sb, bool do_store, int ld_step) {
        (void)do_store;  // (the last phase stores the zeros read past the piece: never read)
        store(nxt, sb);
        compute(cb);
        load(nxt, ld_step);
      };
      Raw ra, rb;
      load(ra, 0);
      load(rb, 1);
      store(ra, 0);
      load(ra, 2);
      __syncthreads();
      // an even number of steps (an odd piece ends with a step of zeros: adds nothing), so
      // the loop body has no exit between its two phases (with one, the compiler's wait
      // counts at the loop head had to cover that path and waited for the next step's loads)
      for (int s = 0; s < steps; s += 2) {
        phase(0, rb, 1, true, s + 3);
        __syncthreads();
        phase(1, ra, 0, true, s + 4);
        __syncthreads();
      }
      if (has_al) {
        const int bp = pass_bits(p);
        if (je == j1) {
          alpha_dot(bp, 0);
        } else {
          const int bq = pass_bits(p + 1);
          if (bq != bp) alpha_dot(bp, bq);
        }
      }
      j = je;
    }

    // block sums of db and of the alpha partial (fixed order through LDS)
    const int tid = opaque((int)threadIdx.x);
    const int ln = tid & 63;
    if (has_al) {
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) aprod += __shfl_xor(aprod, off, 64);
      if (ln == 0) fl[wave] = aprod;
    }
    __syncthreads();
    float dbv = 0.0f, ap = 0.0f;
    if (do_db && tid < kDwgTile) {
#pragma unroll
      for (int q = 0; q < 16; ++q) dbv += s_db[q * kDwgTile + tid];
    }
    if (has_al && tid == 0) {
      for (int w = 0; w < kDwgWaves; ++w) ap += fl[w];
    }
    // slab offset of sub-tile (ti, tu) for this lane: [ti][tu][lane] f32x4
    auto slab_off = [&](int ti, int tu) { return ((ti * 9 + tu) * 64) * 16; };

    bool finish = pos == T0 && send == T1;  // the whole tile is this block's
    if (!finish) {
      // publish this segment's slab
      const int nsl = dwg_owner(T1 - 1, nb, Wtot) - dwg_owner(T0, nb, Wtot) + 1;
      float* slab = slots + (int64_t)(2 * blk + (beg >= T0 ? 0 : 1)) * kDwgSlotF;
      const __amdgpu_buffer_rsrc_t rs = make_rsrc(slab, (int64_t)kDwgSlotF * 4);
      for_tiles([&](f32x4& ac, int ti, int tu) {
        __builtin_amdgcn_raw_buffer_store_b128(ac, rs, ln * 16, slab_off(ti, tu), kSc1);
      });
      if (do_db && tid < kDwgTile)
        __hip_atomic_store(slab + kDwgDb + tid, dbv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (has_al && tid == 0)
        __hip_atomic_store(slab + kDwgAl, ap, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains
      __syncthreads();
      if (tid == 0) {
        const uint32_t old = __hip_atomic_fetch_add(tickets + d.tile0 + t, 1u, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
        *s_flag = old == (uint32_t)(nsl - 1);
      }
      __syncthreads();
      finish = *s_flag != 0;
      if (finish) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keep the loads below
        // sum the segments' slabs in block order (own slab included: read back)
        const int bf = dwg_owner(T0, nb, Wtot);
        dbv = 0.0f;
        ap = 0.0f;
        for (int q = 0; q < nsl; ++q) {
          const int bb = bf + q;
          const float* sl =
              slots + (int64_t)(2 * bb + (dwg_start(bb, nb, Wtot) >= T0 ? 0 : 1)) * kDwgSlotF;
          const __amdgpu_buffer_rsrc_t rl = make_rsrc(sl, (int64_t)kDwgSlotF * 4);
          for_tiles([&](f32x4& ac, int ti, int tu) {
            const f32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rl, ln * 16, slab_off(ti, tu), kSc1);
            ac = q == 0 ? v : ac + v;
          });
          if (do_db && tid < kDwgTile) {
            const float v =
                __hip_atomic_load(sl + kDwgDb + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            dbv = q == 0 ? v : dbv + v;
          }
          if (has_al && tid == 0) {
            const float v =
                __hip_atomic_load(sl + kDwgAl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            ap = q == 0 ? v : ap + v;
          }
        }
        if (tid == 0)
          __hip_atomic_store(tickets + d.tile0 + t, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    if (finish) {
      // dW = G * 1[|W/a| <= 1] (quant.py:80-82; dense: G)
      const __amdgpu_buffer_rsrc_t rd = make_rsrc(d.dW, (int64_t)N * K * 4);
      const int eb = elem_base();
      for_tiles([&](f32x4& ac, int ti, int tu) {
        float w[4];
        if (has_al) {
#pragma unroll
          for (int reg = 0; reg < 4; ++reg)
            w[reg] = ld_f32(rw, eb + ((16 * ti + reg) * K + 16 * tu) * 4);
        }
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
          float v = ac[reg];
          if (has_al) v *= ste_indicator(w[reg] / a);
          st_f32(v, rd, eb + ((16 * ti + reg) * K + 16 * tu) * 4);
        }
      });
      if (do_db && tid < kDwgTile) d.db[n0 + tid] = dbv;
      if (has_al && tid == 0) {
        const float chain = alpha_chain(d.alpha, d.alpha_raw);
        if (d.tiles == 1) {
          *d.dalpha = ap * chain;
        } else {
          __hip_atomic_store(talpha + d.tile0 + t, ap, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          uint32_t* gt = tickets + total_tiles + gi;
          const uint32_t old =
              __hip_atomic_fetch_add(gt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (old == (uint32_t)(d.tiles - 1)) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            float s2 = 0.0f;
            for (int q = 0; q < d.tiles; ++q)
              s2 += __hip_atomic_load(talpha + d.tile0 + q, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT);
            *d.dalpha = s2 * chain;
            __hip_atomic_store(gt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
        }
      }
    }
    pos = send;
  }
}

// descriptors per table launch (kernel arguments: 32 x 112 B + 16 B, inside the 4 KiB
// kernel-argument segment): 186 gemms a step in 6 launches instead of 12 (~4.5 us each)
constexpr int kDwgChunk = 32;
static_assert(sizeof(DwgDesc) * kDwgChunk + 64 <= 4096, "dwg_table_kernel arguments exceed 4 KiB");
struct DwgChunk {
  DwgDesc d[kDwgChunk];
};
__global__ void dwg_table_kernel(DwgDesc* table, int off, int n, DwgChunk c) {
  if ((int)threadIdx.x < n) table[off + threadIdx.x] = c.d[threadIdx.x];
}


}  // namespace

DwPlan plan_dw(int64_t M, int64_t N, int64_t K) { return plan_dw_passes(1, M, N, K); }

DwPlan plan_dw_passes(int64_t P, int64_t Mp, int64_t N, int64_t K) {
  DwPlan p;
  const int64_t M = P * Mp;  // chunk length is chosen for the whole stacked M
  if (N % 4 != 0 || K % 4 != 0 || N < 4 || K < 4) {
    p.variant = 0;
    p.tiles_n = N > 0 ? ceil_div(N, kDwTile) : 1;  // >= 1 so K = 0 still yields db
    p.tiles_k = K > 0 ? ceil_div(K, kDwTile) : 1;
    const int64_t tiles = p.tiles_n * p.tiles_k;
    int64_t steps = 32;  // chunk = S steps x 16 rows
    while (steps > 8 && tiles * ceil_div(M, 16 * steps) < 256) steps /= 2;
    p.rows_per_chunk = 16 * steps;
  } else if (N % 48 == 0 && K % 48 == 0) {
    // LDS-shared bf16x6: 144x144 block tiles (9 waves) where both widths allow it, else
    // 144x48 / 48x144 (3 waves) or 48x48 (1 wave); chunks of 32-row steps sized for ~256
    // blocks (one per CU).
    p.variant = (N % 144 == 0 && K % 144 == 0 && N * K > 144 * 144) ? 9
                : (N % 144 == 0) ? 31 : (K % 144 == 0) ? 13 : 11;
    const int64_t bn = p.variant == 9 || p.variant == 31 ? 144 : 48;
    const int64_t bk = p.variant == 9 || p.variant == 13 ? 144 : 48;
    p.tiles_n = N / bn;
    p.tiles_k = K / bk;
    const int64_t tiles = p.tiles_n * p.tiles_k;
    const int64_t want = ceil_div(256, tiles * P);  // chunks per pass
    p.rows_per_chunk = kStepRows * ceil_div(ceil_div(Mp > 0 ? Mp : 1, want), kStepRows);
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
    int64_t steps = 8;
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
                       hipStream_t s, const DwAlpha* al) {
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
  if (p.variant >= 9) {  // requires al (the finish is launch_dw_finish, not ste_reduce)
    launch_dw_partial_group(&dY, 1, X, M * p.passes, N, K, p, &part, &part_db, al, s);
    return;
  }
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

void launch_dw_partial_group(const float* const* dY, int G, const float* X, int64_t M,
                             int64_t N, int64_t K, const DwPlan& p, float* const* part,
                             float* const* part_db, const DwAlpha* al, hipStream_t s) {
  launch_dw_partial_group_defer(dY, G, X, M, N, K, p, part, part_db, al, nullptr, 0, nullptr, s);
}

void launch_dw_partial_group_defer(const float* const* dY, int G, const float* X, int64_t M,
                                   int64_t N, int64_t K, const DwPlan& p, float* const* part,
                                   float* const* part_db, const DwAlpha* al,
                                   DwFinishEntry* table, int slot, const DwFinishEntry* ent,
                                   hipStream_t s) {
  if (p.rows_per_pass == 0 || N == 0) return;
  M = p.rows_per_pass;
  DwLdsGroup grp{};
  grp.layers = G;
  grp.table = table;
  grp.slot = slot;
  if (table)
    for (int i = 0; i < G; ++i) grp.ent[i] = ent[i];
  for (int i = 0; i < G; ++i) {
    grp.dY[i] = dY[i];
    grp.part[i] = part[i];
    grp.part_db[i] = part_db[i];
    grp.al[i] = al[i];
  }
  // p.tiles_n counts the n-tiles of all G layers (plan of N_total = G * N)
  const unsigned nb = (unsigned)(p.tiles_n * p.tiles_k * p.chunks);
#define OB_DWL(WN, WK)                                                                        \
  hipLaunchKernelGGL((dw_lds_kernel<WN, WK>), dim3(nb), dim3(64 * WN * WK),                   \
                     (size_t)(2 * DwLdsCfg<WN, WK>::kBuf), s, X, M, (int)N, (int)K,           \
                     (int)p.tiles_k, p.rows_per_chunk, p.chunks_per_pass, grp)
  if (p.variant == 9) OB_DWL(3, 3);
  else if (p.variant == 31) OB_DWL(3, 1);
  else if (p.variant == 13) OB_DWL(1, 3);
  else OB_DWL(1, 1);
#undef OB_DWL
}

void launch_dw_finish(const float* part, int chunks, int64_t nk, const float* part_db,
                      int64_t n_db, const float* W, const float* alpha, int alpha_raw,
                      const float* apart, int n_apart, float* dW, float* db, float* dalpha,
                      hipStream_t s) {
  const DwFinish a{part, chunks, nk, part_db, n_db, W, alpha, alpha_raw, apart, n_apart,
                   dW, db, dalpha};
  const int64_t nb = finish_blocks(a);  // + the alpha block
  hipLaunchKernelGGL(dw_finish_kernel, dim3((unsigned)nb), dim3(kThreads), 0, s, a);
}

int64_t dw_finish_blocks(const DwFinish& a) { return finish_blocks(a); }

__global__ void dw_table_entry_kernel(DwFinishEntry* table, int slot, DwFinishEntry ent) {
  table[slot] = ent;
}

void launch_dw_table_entry(DwFinishEntry* table, int slot, const DwFinishEntry& ent,
                           hipStream_t s) {
  hipLaunchKernelGGL(dw_table_entry_kernel, dim3(1), dim3(1), 0, s, table, slot, ent);
}

void launch_dw_finish_table(const DwFinishEntry* table, int n, int64_t total_blocks,
                            hipStream_t s) {
  if (n <= 0 || total_blocks <= 0) return;
  hipLaunchKernelGGL(dw_finish_table_kernel, dim3((unsigned)total_blocks), dim3(kThreads), 0, s,
                     table, n, total_blocks);
}

int dwg_blocks(int64_t total_steps) {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      cus <= 0)
    cus = 256;
  return (int)(total_steps < cus ? total_steps : cus);
}

size_t dwg_slot_bytes() { return sizeof(float) * (size_t)kDwgSlotF; }

void launch_dw_grouped(const DwgDesc* host_descs, int G, int64_t total_steps, int blocks,
                       DwgDesc* table, float* slots, float* talpha, uint32_t* tickets,
                       int total_tiles, hipStream_t s) {
  // the descriptors reach the device as kernel arguments (capture-safe: no host copy)
  for (int off = 0; off < G; off += kDwgChunk) {
    DwgChunk c{};
    const int n = G - off < kDwgChunk ? G - off : kDwgChunk;
    for (int i = 0; i < n; ++i) c.d[i] = host_descs[off + i];
    hipLaunchKernelGGL(dwg_table_kernel, dim3(1), dim3(kDwgChunk), 0, s, table, off, n, c);
  }
  hipLaunchKernelGGL(dw_grouped_kernel, dim3((unsigned)blocks), dim3(kDwgThreads),
                     (size_t)kDwgLds, s, table, G, (int)total_steps, slots,
                     talpha, tickets, total_tiles);
}

void launch_dw_finish_group(const DwFinish* a, int n, hipStream_t s) {
  DwFinishGroup G{};
  G.n = n;
  int64_t total = 0;
  for (int i = 0; i < n; ++i) {
    G.g[i] = a[i];
    G.start[i] = (int)total;
    total += finish_blocks(a[i]);
  }
  G.start[n] = (int)total;
  hipLaunchKernelGGL(dw_finish_group_kernel, dim3((unsigned)total), dim3(kThreads), 0, s, G);
}

#ifdef OB_DW_STAMPS
extern "C" int ob_dw_stamps(void* host_stamps, void* host_rt) {  // diagnostic build only
  if (hipMemcpyFromSymbol(host_stamps, HIP_SYMBOL(g_dw_stamps), sizeof(g_dw_stamps)) != hipSuccess) return -6;
  return hipMemcpyFromSymbol(host_rt, HIP_SYMBOL(g_dw_rt), sizeof(g_dw_rt)) == hipSuccess ? 0 : -6;
}
#endif

}  // namespace ob
