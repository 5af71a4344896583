// dgemm.hip — the conv module's pointwise (kernel-size-1) Conv1d GEMMs on gfx950 matrix
// cores, fp32 in and out (conformer.py:143,147; onebit_asr/conv.py _PointwiseFn).
//
//   forward  Y  = X . W^T + b     (W [N][K]: the Conv1d weight viewed [out][in])
//   dgrad    dX = dY . W          (the same kernel, W read transposed: W [K][N])
//
// fp32 parity with the reference's fp32 conv: both operands are split exactly into three
// bf16 parts (x = hi + mid + lo, 8+8+8 significand bits) and six v_mfma_f32_16x16x32_bf16
// per k-step accumulate the products mm, lh, hl, mh, hm, hh in fp32. The dropped terms
// (ml, lm, ll) are below 2^-25 of |x||w|: an fp32 GEMM up to summation order.
//
// Block = WAVES waves, 16*WAVES rows x BN = 16*NT columns. At entry the block splits its BN
// columns of W (read straight from the fp32 weight, L2-resident) into a three-plane bf16
// image in LDS ([BN][3][Kpad+8]; the pad keeps the B-fragment ds_read_b128 conflict-free),
// then loops over its 16-row subtiles (an even share of M per block, dealt round-robin to
// the waves): each wave streams 16 rows of A (two dwordx4 per lane per
// 32-wide k-chunk, a window of chunks in flight across subtiles), splits them in
// registers and issues 6 MFMAs per 16-column tile. Blocks sharing a row tile are dealt to
// the same XCD (one L2 serves their A reads).
//
// Fragment map of v_mfma_f32_16x16x32_bf16 (lane l, r = l&15, g = l>>4):
//   A[i=r][kk=8g+j] (j<8), B[kk=8g+j][col=r], D[row=4g+reg][col=r].
#include <algorithm>
#include <cstdlib>

#include "ob_drop.h"
#include "ob_fp.h"
#include "ob_launch.h"

namespace ob {

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr size_t kLdsCU = 160 * 1024;  // LDS per CU

// x = hi + mid + lo exactly (RNE at each step; the residuals are exact in fp32).
__device__ __forceinline__ void split3x8(const f32x4& a, const f32x4& b, bf16x8& hi, bf16x8& mid,
                                         bf16x8& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float x = j < 4 ? a[j] : b[j - 4];
    const __bf16 h = (__bf16)x;
    const float r1 = x - (float)h;
    const __bf16 m = (__bf16)r1;
    hi[j] = h;
    mid[j] = m;
    lo[j] = (__bf16)(r1 - (float)m);
  }
}

__device__ __forceinline__ void split3x4(const f32x4& a, bf16x4& hi, bf16x4& mid, bf16x4& lo) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const __bf16 h = (__bf16)a[j];
    const float r1 = a[j] - (float)h;
    const __bf16 m = (__bf16)r1;
    hi[j] = h;
    mid[j] = m;
    lo[j] = (__bf16)(r1 - (float)m);
  }
}

__device__ __forceinline__ f32x4 mfma_bf16(const bf16x8& a, const bf16x8& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// Bijective XCD-aware remap: consecutive logical ids land on one XCD under round-robin
// dispatch (cdna_hip_programming.md §5).
__device__ __forceinline__ int xcd_logical(int b, int nb) {
  const int q = nb / 8, r = nb % 8, x = b % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

// Two dwordx4 of one row at k and k+4, the address clamped into the row (an unguarded load
// keeps the prefetch window in flight; clamped positions k >= K meet zero rows of the image).
__device__ __forceinline__ void load8(const float* __restrict__ arow, int k, int K, f32x4& a,
                                      f32x4& b) {
  const int ka = k < K - 4 ? k : K - 4;
  const int kb = k + 4 < K - 4 ? k + 4 : K - 4;
  a = *reinterpret_cast<const f32x4*>(arow + ka);
  b = *reinterpret_cast<const f32x4*>(arow + kb);
}

// products in the order they are accumulated (smallest first): plane of A, plane of B
// (0 = hi, 1 = mid, 2 = lo)
constexpr int kProdA[6] = {1, 2, 0, 1, 0, 0};
constexpr int kProdB[6] = {1, 0, 2, 0, 1, 0};

__host__ __device__ inline int dg_kpad(int K, int nch) { return nch > 0 ? 32 * nch : (K + 31) & ~31; }
__host__ __device__ inline size_t dg_lds_bytes(int nt, int kpad) {
  return (size_t)16 * nt * 3 * (kpad + 8) * sizeof(uint16_t);
}

template <int NT, int NCH, int WAVES, bool TRANS, bool RES = false>
__global__ __launch_bounds__(64 * WAVES, 2) void dgemm_kernel(
    const float* __restrict__ A, int64_t M, int K, const float* __restrict__ W, int N, int n_ct,
    int n16, int rgroups, const float* __restrict__ bias, float* __restrict__ C,
    const float* __restrict__ R, DropCfg dc, const uint64_t* __restrict__ rng, uint64_t rng_off) {
  constexpr int kThr = 64 * WAVES, BN = 16 * NT;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __bf16* bimg = reinterpret_cast<__bf16*>(smem);
  const int kpad = dg_kpad(K, NCH);
  const int stride = kpad + 8;   // bf16 per plane row
  const int cpitch = 3 * stride;  // bf16 per image column (three planes)

  const int L = xcd_logical(blockIdx.x, gridDim.x);
  const int ct = L % n_ct;
  const int rg = L / n_ct;
  const int n0 = ct * BN;
  // this block's 16-row subtiles [s0, s1) (an even share of the n16 subtiles of M), dealt
  // round-robin to its waves: a block's waves -- and so its SIMDs -- differ by at most one
  // subtile, where whole 16*WAVES-row tiles left half the blocks a second round
  const int s0 = (int)((int64_t)rg * n16 / rgroups), s1 = (int)((int64_t)(rg + 1) * n16 / rgroups);
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int r = lane & 15;
  const int g = lane >> 4;
  const int kg = 8 * g;

  // ---- B image: column c (output column n0 + c) holds W's values along k in 3 planes.
  // Loader unit = 4 consecutive k of one column, stored as one 8-byte write per plane:
  // !TRANS -> one dwordx4 of W row n (units column-major: a lane's 4 k are contiguous);
  // TRANS -> 4 dwords of W column n (units k-major: consecutive lanes read consecutive
  // columns of a W row, coalesced). Clamped loads; zeros selected for k >= K (K % 4 == 0,
  // so a unit is all in or all out) and for columns >= N.
  const int kq = kpad >> 2;
  const int units = BN * kq;
  auto unit_cols = [&](int u, int& c, int& k4) {
    if constexpr (TRANS) {
      k4 = u / BN;
      c = u - k4 * BN;
    } else {
      c = u / kq;
      k4 = u - c * kq;
    }
  };
  auto unit_load = [&](int u) -> f32x4 {
    u = u < units ? u : units - 1;
    int c, k4;
    unit_cols(u, c, k4);
    const int n = n0 + c < N ? n0 + c : N - 1;
    const int kk = 4 * k4 < K - 4 ? 4 * k4 : K - 4;
    if constexpr (TRANS) {
      const float* p = W + (int64_t)kk * N + n;
      return f32x4{p[0], p[N], p[2 * N], p[3 * N]};
    } else {
      return *reinterpret_cast<const f32x4*>(W + (int64_t)n * K + kk);
    }
  };
  auto unit_store = [&](int u, f32x4 v) {
    if (u >= units) return;
    int c, k4;
    unit_cols(u, c, k4);
    const bool ok = 4 * k4 < K && n0 + c < N;
    const f32x4 x = ok ? v : f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x4 h, m, l;
    split3x4(x, h, m, l);
    __bf16* col = bimg + c * cpitch + 4 * k4;
    *reinterpret_cast<bf16x4*>(col) = h;
    *reinterpret_cast<bf16x4*>(col + stride) = m;
    *reinterpret_cast<bf16x4*>(col + 2 * stride) = l;
  };
  auto arow_of = [&](int j) {  // row r of subtile j (clamped into M)
    const int64_t row = (int64_t)16 * j + r < M ? (int64_t)16 * j + r : M - 1;
    return A + row * (int64_t)K;
  };
  const int j0 = s0 + wave;  // this wave's first subtile (>= s1: no work)

  constexpr int kWmax = NT > 6 ? 3 : 5;
  constexpr int kWin = NCH > 0 ? (NCH < kWmax ? NCH : kWmax) : 1;
  f32x4 buf[NCH > 0 ? NCH : 1][2];
  if constexpr (NCH > 0) {
    constexpr int kUnits = BN * 8 * NCH;
    constexpr int kUpt = (kUnits + kThr - 1) / kThr;
    f32x4 wv[kUpt];
#pragma unroll
    for (int i = 0; i < kUpt; ++i) wv[i] = unit_load(threadIdx.x + i * kThr);
    const float* a0 = arow_of(j0 < s1 ? j0 : s0);  // (s0 < s1: a real subtile)
#pragma unroll
    for (int c = 0; c < kWin; ++c) load8(a0, 32 * c + kg, K, buf[c][0], buf[c][1]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < kUpt; ++i) unit_store(threadIdx.x + i * kThr, wv[i]);
  } else {
    for (int u = threadIdx.x; u < units; u += kThr) unit_store(u, unit_load(u));
  }
  __syncthreads();

  const __bf16* brow = bimg + r * cpitch + kg;
  const uint32_t dkey = (RES && dc.on) ? drop_key(rng[0], rng[1] + rng_off) : 0u;
  float bcol[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int col = n0 + 16 * t + r;
    bcol[t] = (bias && col < N) ? bias[col] : 0.0f;
  }

  for (int j = j0; j < s1; j += WAVES) {
    const int64_t m0 = (int64_t)16 * j;
    const float* arow = arow_of(j);
    f32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};

    // One k-chunk: the A split runs while the first group's B reads are in flight; tiles
    // go in groups of three (9 fragments = 36 VGPRs live), product-major inside a group so
    // consecutive MFMAs update different accumulators.
    auto compute = [&](const f32x4& x0, const f32x4& x1, int kc) {
      constexpr int kG = NT < 3 ? NT : 3;
#pragma unroll
      for (int t0 = 0; t0 < NT; t0 += kG) {
        bf16x8 b[kG][3];
#pragma unroll
        for (int t = 0; t < kG; ++t)
#pragma unroll
          for (int q = 0; q < 3; ++q)
            if (t0 + t < NT)
              b[t][q] = *reinterpret_cast<const bf16x8*>(brow + (t0 + t) * 16 * cpitch +
                                                          q * stride + kc);
        __builtin_amdgcn_sched_barrier(0);
        bf16x8 a[3];
        split3x8(x0, x1, a[0], a[1], a[2]);
#pragma unroll
        for (int p = 0; p < 6; ++p)
#pragma unroll
          for (int t = 0; t < kG; ++t)
            if (t0 + t < NT)
              acc[t0 + t] = mfma_bf16(a[kProdA[p]], b[t][kProdB[p]], acc[t0 + t]);
      }
    };

    if constexpr (NCH > 0) {
      // Fully unrolled; kWin chunks in flight, the next row tile's first chunks issued
      // while this tile computes its last ones (the last tile re-reads its own rows as the
      // "next" tile: L2 hits, never used).
      const float* anext = arow_of(j + WAVES < s1 ? j + WAVES : j);
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        if (c + kWin < NCH) load8(arow, 32 * (c + kWin) + kg, K, buf[c + kWin][0], buf[c + kWin][1]);
        __builtin_amdgcn_sched_barrier(0);
        compute(buf[c][0], buf[c][1], 32 * c);
        if (c + kWin >= NCH) {
          load8(anext, 32 * (c + kWin - NCH) + kg, K, buf[c + kWin - NCH][0],
                buf[c + kWin - NCH][1]);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    } else {
      // Generic K: three rotating register sets (no register copy of an in-flight load).
      f32x4 r0a, r0b, r1a, r1b, r2a, r2b;
      load8(arow, kg, K, r0a, r0b);
      load8(arow, 32 + kg, K, r1a, r1b);
      for (int kc = 0; kc < kpad; kc += 96) {
        load8(arow, kc + 64 + kg, K, r2a, r2b);
        compute(r0a, r0b, kc);
        load8(arow, kc + 96 + kg, K, r0a, r0b);
        if (kc + 32 < kpad) compute(r1a, r1b, kc + 32);
        load8(arow, kc + 128 + kg, K, r1a, r1b);
        if (kc + 64 < kpad) compute(r2a, r2b, kc + 64);
      }
    }

    __builtin_amdgcn_sched_barrier(0);
    // D[row = 4g + reg][col = r]: 16 lanes write 64 contiguous bytes of a row per store.
    // Residual epilogue (RES, its own instantiation: the plain kernels keep their registers):
    // per column tile, the four R values are loaded before the first store (the whole
    // tile's R in registers spills at NT 9).
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int col = n0 + 16 * t + r;
      if (col >= N) continue;
      float rv[4];
      if constexpr (RES) {
#pragma unroll
        for (int reg = 0; reg < 4; ++reg)
          rv[reg] = R[min(m0 + 4 * g + reg, M - 1) * N + col];
      }
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int64_t orow = m0 + 4 * g + reg;
        if (orow >= M) continue;
        const int64_t i = orow * N + col;
        const float y = acc[t][reg] + bcol[t];
        if constexpr (RES) {  // R + dropout(y), the operation sequence of residual_drop_fwd_kernel
          const float v = dc.on ? nc_mul(y, drop_keep(dkey, (uint64_t)i, dc.thresh) ? dc.scale : 0.0f) : y;
          C[i] = nc_add(rv[reg], v);
        } else {
          C[i] = y;
        }
      }
    }
  }
}


// ---------------------------------------------------------------------------------
// Long-K form (K too long for a whole-K image: the CTC head's input gradient, K = V = 5004,
// the reference's fp32 `g @ W` of linear.py / losses.py:41-47 through conformer.py:275):
// the block holds all 16 NT columns and walks K in chunks of kKc = 64, the chunk's B image
// (three planes, [BN][3][kKc + 8] bf16) double-buffered in LDS and built from W while the
// previous chunk's MFMAs run; each wave owns one 16-row subtile (a block = 16 WAVES rows).
// Same six products per k-step as dgemm_kernel, k in order: an fp32 GEMM up to summation
// order. Units of the loader: 4 consecutive k of one column (TRANS: W [K][N], consecutive
// lanes on consecutive columns of a W row; else W [N][K], one dwordx4).
// ---------------------------------------------------------------------------------
constexpr int kKc = 64;
constexpr int kKcStride = kKc + 8;  // bf16 per plane row (conflict-free ds_read_b128)

__host__ __device__ inline size_t dgkc_lds_bytes(int nt) {
  return (size_t)2 * 16 * nt * 3 * kKcStride * sizeof(uint16_t);
}

template <int NT, int WAVES, bool TRANS>
__global__ __launch_bounds__(64 * WAVES, 1) void dgemm_kc_kernel(
    const float* __restrict__ A, int64_t M, int K, const float* __restrict__ W, int N,
    const float* __restrict__ bias, float* __restrict__ C) {
  constexpr int kThr = 64 * WAVES, BN = 16 * NT;
  constexpr int kCpitch = 3 * kKcStride;            // bf16 per image column
  constexpr int kBuf = BN * kCpitch;                // bf16 per buffer
  constexpr int kUnits = BN * (kKc / 4);            // loader units per chunk
  constexpr int kUpt = (kUnits + kThr - 1) / kThr;  // units per thread
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __bf16* img = reinterpret_cast<__bf16*>(smem);
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4, kg = 8 * g;
  const int L = xcd_logical(blockIdx.x, gridDim.x);
  const int64_t m0 = ((int64_t)L * WAVES + wave) * 16;  // this wave's subtile
  const int64_t arow_i = m0 + r < M ? m0 + r : M - 1;
  const float* arow = A + arow_i * (int64_t)K;
  const int nck = (K + kKc - 1) / kKc;

  auto unit_cols = [&](int u, int& c, int& k4) {
    if constexpr (TRANS) {
      k4 = u / BN;
      c = u - k4 * BN;
    } else {
      c = u / (kKc / 4);
      k4 = u - c * (kKc / 4);
    }
  };
  auto unit_load = [&](int ch, int u) -> f32x4 {
    u = u < kUnits ? u : kUnits - 1;
    int c, k4;
    unit_cols(u, c, k4);
    const int n = c < N ? c : N - 1;
    int kk = ch * kKc + 4 * k4;
    kk = kk < K - 4 ? kk : K - 4;  // clamped (zeros selected at the store)
    if constexpr (TRANS) {
      const float* p = W + (int64_t)kk * N + n;
      return f32x4{p[0], p[N], p[2 * N], p[3 * N]};
    } else {
      return *reinterpret_cast<const f32x4*>(W + (int64_t)n * K + kk);
    }
  };
  // (u >= kUnits: the clamped unit again -- the same value to the same address, so the
  // store needs no branch, which would let hipcc sink the unit's load into it)
  auto unit_store = [&](int ch, int buf, int u, f32x4 v) {
    u = u < kUnits ? u : kUnits - 1;
    int c, k4;
    unit_cols(u, c, k4);
    const bool ok = ch * kKc + 4 * k4 < K && c < N;
    const f32x4 x = ok ? v : f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x4 h, m, l;
    split3x4(x, h, m, l);
    __bf16* col = img + buf * kBuf + c * kCpitch + 4 * k4;
    *reinterpret_cast<bf16x4*>(col) = h;
    *reinterpret_cast<bf16x4*>(col + kKcStride) = m;
    *reinterpret_cast<bf16x4*>(col + 2 * kKcStride) = l;
  };
  // A: two dwordx4 per lane per 32-wide k step (clamped: k >= K meets zero image rows)
  constexpr int kWin = 4;  // k steps in flight (2 chunks)
  f32x4 abuf[kWin][2];
  auto load_a = [&](int st, f32x4& x0, f32x4& x1) { load8(arow, 32 * st + kg, K, x0, x1); };

  f32x4 wv[kUpt];
#pragma unroll
  for (int i = 0; i < kUpt; ++i) wv[i] = unit_load(0, threadIdx.x + i * kThr);
#pragma unroll
  for (int w = 0; w < kWin; ++w) load_a(w, abuf[w][0], abuf[w][1]);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < kUpt; ++i) unit_store(0, 0, threadIdx.x + i * kThr, wv[i]);
  __syncthreads();

  f32x4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  // Chunks in pairs, so every A ring slot (2 * cc + hs) and LDS buffer (cc) is a static
  // index: a dynamic index into abuf makes hipcc move the ring through gpr-indexed copies
  // behind a vmcnt(0) per k step (every A load then waited for where it is issued). The
  // loads are unconditional (clamped addresses; k >= K meets zero image rows).
  for (int ch0 = 0; ch0 < nck; ch0 += 2) {
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
      const int ch = ch0 + cc;
      if (ch >= nck) break;  // block-uniform
      // the next chunk's W units in flight over this chunk's MFMAs
      const int chn = ch + 1 < nck ? ch + 1 : ch;
#pragma unroll
      for (int i = 0; i < kUpt; ++i) wv[i] = unit_load(chn, threadIdx.x + i * kThr);
      const __bf16* brow = img + cc * kBuf + r * kCpitch + kg;
#pragma unroll
      for (int hs = 0; hs < 2; ++hs) {
        const int st = 2 * ch + hs, slot = 2 * cc + hs;
        const f32x4 x0 = abuf[slot][0], x1 = abuf[slot][1];
        load_a(st + kWin, abuf[slot][0], abuf[slot][1]);
        __builtin_amdgcn_sched_barrier(0);
        constexpr int kG = NT < 3 ? NT : 3;
#pragma unroll
        for (int t0 = 0; t0 < NT; t0 += kG) {
          bf16x8 b[kG][3];
#pragma unroll
          for (int t = 0; t < kG; ++t)
#pragma unroll
            for (int q = 0; q < 3; ++q)
              if (t0 + t < NT)
                b[t][q] = *reinterpret_cast<const bf16x8*>(brow + (t0 + t) * 16 * kCpitch +
                                                            q * kKcStride + 32 * hs);
          __builtin_amdgcn_sched_barrier(0);
          bf16x8 a[3];
          split3x8(x0, x1, a[0], a[1], a[2]);
#pragma unroll
          for (int p = 0; p < 6; ++p)
#pragma unroll
            for (int t = 0; t < kG; ++t)
              if (t0 + t < NT) acc[t0 + t] = mfma_bf16(a[kProdA[p]], b[t][kProdB[p]], acc[t0 + t]);
        }
      }
      // (unconditional, so hipcc keeps the W loads where they are issued instead of sinking
      // them into a guarded store: after the last chunk the idle buffer -- whose readers all
      // passed the previous barrier -- just takes a copy of that chunk)
#pragma unroll
      for (int i = 0; i < kUpt; ++i) unit_store(chn, cc ^ 1, threadIdx.x + i * kThr, wv[i]);
      __syncthreads();  // the next buffer is complete; this buffer's reads are done
    }
  }
  // D[row = 4g + reg][col = r]
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int col = 16 * t + r;
    if (col >= N) continue;
    const float bc = bias ? bias[col] : 0.0f;
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      const int64_t orow = m0 + 4 * g + reg;
      if (orow < M) C[orow * N + col] = acc[t][reg] + bc;
    }
  }
}

struct DgCfg {
  int nt, waves;
};

// Widest column tile whose image fits one CU's LDS (8 waves) or half of it (4 waves, two
// blocks per CU), preferring tiles that divide N.
DgCfg pick_cfg(int64_t N, int64_t K) {
  const int kpad = dg_kpad((int)K, 0);
  const bool k_special = kpad == 160 || kpad == 288;
  static const int cands[] = {9, 6, 3, 2, 1};
  for (int pass = 0; pass < 2; ++pass)
    for (int nt : cands) {
      if (pass == 0 && N % (16 * nt) != 0) continue;
      if (16 * nt > ((N + 15) & ~int64_t(15))) continue;
      // instantiated combinations (launch_dense_gemm's switch)
      const bool inst = kpad == 160 ? (nt == 9 || nt == 6 || nt == 3)
                        : kpad == 288 ? (nt == 3 || nt == 2 || nt == 1)
                                      : (nt == 3 || nt == 1);
      if (!inst && k_special) continue;
      if (!k_special && !(nt == 3 || nt == 1)) continue;
      const size_t lds = dg_lds_bytes(nt, kpad);
      int waves = lds <= kLdsCU / 2 ? 4 : lds <= kLdsCU ? 8 : 0;
      if (waves) return DgCfg{nt, waves};
    }
  return DgCfg{0, 0};
}

}  // namespace

// the long-K form: every column in one block (N <= 144), K past what the whole-K image holds
static bool dense_kc_shape(int64_t K, int64_t N) {
  return N >= 4 && N <= 144 && N % 4 == 0 && K >= 4 && K % 4 == 0 && K <= (1 << 20) &&
         pick_cfg(N, K).nt == 0;
}

bool dense_gemm_supported(int64_t K, int64_t N) {
  return (K >= 4 && N >= 4 && K % 4 == 0 && N % 4 == 0 && K <= (1 << 20) && N <= (1 << 20) &&
          pick_cfg(N, K).nt > 0) ||
         dense_kc_shape(K, N);
}

bool launch_dense_gemm(const float* A, int64_t M, int64_t K, const float* W, int trans,
                       const float* bias, int64_t N, float* C, hipStream_t s,
                       const DenseEpi* epi) {
  if (!dense_gemm_supported(K, N)) return false;
  if (M == 0) return true;
  if (dense_kc_shape(K, N)) {  // long K: K-chunked images (epilogue: bias only)
    if (epi && epi->R) return false;
    constexpr int kW = 8;
    const dim3 grid((unsigned)ceil_div(M, 16 * kW));
    const size_t lds = dgkc_lds_bytes(9);
    if (trans)
      hipLaunchKernelGGL((dgemm_kc_kernel<9, kW, true>), grid, dim3(64 * kW), lds, s, A, M, (int)K,
                         W, (int)N, bias, C);
    else
      hipLaunchKernelGGL((dgemm_kc_kernel<9, kW, false>), grid, dim3(64 * kW), lds, s, A, M,
                         (int)K, W, (int)N, bias, C);
    return true;
  }
  const DgCfg cfg = pick_cfg(N, K);
  const int kpad = dg_kpad((int)K, 0);
  const size_t lds = dg_lds_bytes(cfg.nt, kpad);
  const int n_ct = (int)ceil_div(N, 16 * cfg.nt);
  const int n16 = (int)ceil_div(M, 16);
  const int per_cu = (int)std::min<size_t>(kLdsCU / lds, (size_t)(8 / cfg.waves));
  // row groups: fill every CU, but give each block at least one subtile per wave (more
  // blocks than that only repeat the B-image prologue: measured +0.5 us at N = 144). The
  // conv module's pw1 forward (N = 288, two column tiles): 128 groups of 11-12 subtiles,
  // three per SIMD at most, where whole 128-row tiles left half the blocks a second round of
  // two per SIMD: 21.9 -> 18.9 us; pw1 dX (three tiles) 22.6 -> 20.1 us; the decoder's
  // K = 1024 linear 36.2 -> 26.8 us (tools/dense_bench.py, profiles/r6/dense_ab/)
  int rgroups = 256 * per_cu / n_ct;
  rgroups = std::min<int64_t>(rgroups, ceil_div(n16, cfg.waves));
  if (rgroups < 1) rgroups = 1;
  const dim3 grid((unsigned)(rgroups * n_ct));
  const int nch = kpad == 160 ? 5 : kpad == 288 ? 9 : 0;
  const float* R = epi ? epi->R : nullptr;
  const DropCfg dc = make_drop(R ? epi->p_drop : 0.0f);
  const uint64_t* rng = R ? epi->rng : nullptr;
  const uint64_t rng_off = R ? epi->rng_off : 0;
#define OB_DG(NT, NCH, WV)                                                                       \
  if (cfg.nt == NT && nch == NCH && cfg.waves == WV) {                                           \
    if (trans)                                                                                   \
      hipLaunchKernelGGL((dgemm_kernel<NT, NCH, WV, true>), grid, dim3(64 * WV), lds, s, A, M,    \
                         (int)K, W, (int)N, n_ct, n16, rgroups, bias, C, nullptr, dc,    \
                         nullptr, 0);                                                            \
    else                                                                                         \
      hipLaunchKernelGGL((dgemm_kernel<NT, NCH, WV, false>), grid, dim3(64 * WV), lds, s, A, M,   \
                         (int)K, W, (int)N, n_ct, n16, rgroups, bias, C, nullptr, dc,    \
                         nullptr, 0);                                                            \
    return true;                                                                                 \
  }
#define OB_DG2(NT, NCH) OB_DG(NT, NCH, 4) OB_DG(NT, NCH, 8)
  if (R && !trans && cfg.nt == 9 && nch == 5) {  // the conv module's pw2 (K, N = 144)
#define OB_DGR(WV)                                                                               \
    if (cfg.waves == WV) {                                                                       \
      hipLaunchKernelGGL((dgemm_kernel<9, 5, WV, false, true>), grid, dim3(64 * WV), lds, s, A,   \
                         M, (int)K, W, (int)N, n_ct, n16, rgroups, bias, C, R, dc, rng,         \
                         rng_off);                                                               \
      return true;                                                                               \
    }
    OB_DGR(4)
    OB_DGR(8)
#undef OB_DGR
  }
  if (R) {  // other shapes: the plain GEMM, then the residual-dropout pass in place
    DenseEpi none{nullptr, 0.0f, nullptr, 0};
    if (!launch_dense_gemm(A, M, K, W, trans, bias, N, C, s, &none)) return false;
    launch_residual_drop_fwd(R, C, M, N, 1.0f, epi->p_drop, rng, rng_off, nullptr, 0, C, s);
    return true;
  }
  OB_DG2(9, 5)
  OB_DG2(6, 5)
  OB_DG2(3, 5)
  OB_DG2(3, 9)
  OB_DG2(2, 9)
  OB_DG2(1, 9)
  OB_DG2(3, 0)
  OB_DG2(1, 0)
#undef OB_DG2
#undef OB_DG
  return false;
}

}  // namespace ob
