// relattn.hip — the relative-position attention core of MHSA, fused (forward + backward).
//
// Reference: onebit_asr/conformer.py:115-130 (MHSA.forward between the projections):
//   ac = (q + u) k^T                    matrix_ac
//   bd = rel_shift((q + v) p^T)         matrix_bd, rel_shift of :97-103
//   S  = (ac + bd) / sqrt(d); S[i][j] = -inf where frame i or j is padding (mask :121-122)
//   A  = nan_to_num(softmax(S))         fully masked rows -> 0 (:123-125)
//   A  = dropout(A); ctx = A v          (:126-127)
// torch materialises ac, bd (padded, shifted copies), S, A and the dropout mask as
// [B,H,T,T] fp32 tensors, ~10 full passes per block per pass. Here the forward is one
// kernel that keeps a query tile's scores in registers and writes only ctx and the
// softmax probabilities (kept for the backward). The backward is a query-side kernel (dq,
// dS' to global) and a key-side kernel (dk, dv, per-row dpos over all queries: no
// per-query-tile partials), plus one launch holding two fixed-order reductions (du/dvb over tiles,
// dpos over the pass's batch rows).
//
// rel_shift as a FLAT re-reading (conformer.py:97-103 pads a zero column on the left of X =
// (q + v) p^T, views the [T][T+1] result as [T+1][T] and drops the first row): with
// Xpad[r] = [0, X[r][0 .. T-1]] stored row after row at pitch T+1,
//   bd[i][j] = Xpad.flat[T + i*T + j]
// so the forward reads bd at a lane base + an immediate offset (no per-element branch), and
// the adjoint is the same map backwards: dX[r][m] = dS'.flat[r*(T+1) + m + 1 - T] (0 where
// that index is negative, i.e. only in row 0), read from a row-major dS' band at pitch T.
//
// Layout: q, k, v, ctx, dq, dk, dv [Bt][T][H*d]; pos, dpos [P][T][H*d] (batch row b uses
// pass b / (Bt/P)); u, vb, du, dvb [H][d]; lens int32 [Bt].
// probs: MFMA-fragment tiles [Bt*H][nt][nt][64 lanes][4], nt = ceil(T/16): tile (a, t) holds
// P[16a + r][16t + 4g + e] in lane r + 16g, element e -- the layout the forward's scores
// are in, so every lane writes (and the query-side backward reads) one dwordx4 per 16x16
// tile, 1 KB contiguous per wave instruction. Rows / keys >= T hold 0.
// Products on v_mfma_f32_16x16x4_f32 (exact fp32 fma chain, like torch's fp32 matmul).
// Dropout keeps (i, j) by the pair hash of ob_drop.h on index (bh*T + i)*Te + j, Te = T
// rounded up to even (so the two keys of a pair share a row); the forward stores each kept
// probability as P and each dropped one as -P (P >= 0, so the sign bit is free), and the
// backward kernels read the keep bit back with the probability.
#include <atomic>
#include <math.h>

#include <algorithm>

#include "ob_drop.h"
#include "ob_launch.h"

namespace {
// Sums / max / or over the four 16-lane rows of a wave (x op x[lane ^ 16], then ^ 32) on the
// gfx950 lane-swap instructions (VALU) instead of ds_bpermute round trips through the LDS
// pipe this kernel's fragments keep busy. permlane16_swap(x, x) returns, per lane, x of
// both lanes {l, l ^ 16} (in row order) and permlane32_swap those of {l, l ^ 32}; the
// operations are commutative, so the results are the xor shuffles' bits.
template <typename F>
__device__ __forceinline__ uint32_t xrows_1632(uint32_t x, F op) {
  const auto a = __builtin_amdgcn_permlane16_swap(x, x, false, false);
  x = op(a[0], a[1]);
  const auto b = __builtin_amdgcn_permlane32_swap(x, x, false, false);
  return op(b[0], b[1]);
}
__device__ __forceinline__ float xsum_1632(float v) {
  return __builtin_bit_cast(float, xrows_1632(__builtin_bit_cast(uint32_t, v), [](uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(float, a) + __builtin_bit_cast(float, b));
  }));
}
__device__ __forceinline__ float xmax_1632(float v) {
  return __builtin_bit_cast(float, xrows_1632(__builtin_bit_cast(uint32_t, v), [](uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, fmaxf(__builtin_bit_cast(float, a), __builtin_bit_cast(float, b)));
  }));
}
__device__ __forceinline__ uint32_t xor_1632(uint32_t v) {
  return xrows_1632(v, [](uint32_t a, uint32_t b) { return a | b; });
}
}  // namespace

namespace ob {

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kThreads = 256;
constexpr int kTile = 64;  // query rows per block (16 per wave)
constexpr int kFwdKeyChunk = 256;  // keys of v staged per pass of the forward's ctx product

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// bf16x6 products: exact fp32 from bf16 MFMA (every operand x = hi + mid + lo)
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma_bf(const bf16x8_t& a, const bf16x8_t& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// x = hi + mid + lo exactly (each part the bf16 rounding of what is left)
__device__ __forceinline__ void split3(float x, __bf16& h, __bf16& m, __bf16& l) {
  h = (__bf16)x;
  const float r1 = x - (float)h;
  m = (__bf16)r1;
  l = (__bf16)(r1 - (float)m);
}

__device__ __forceinline__ void split8(const float (&x)[8], bf16x8_t (&p)[3]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    __bf16 h, m, l;
    split3(x[j], h, m, l);
    p[0][j] = h;
    p[1][j] = m;
    p[2][j] = l;
  }
}

// the six products of weight >= 2^-16 (smallest first), as dw.hip's bf16x6 GEMM
__device__ __forceinline__ f32x4 mfma_x6(const bf16x8_t (&a)[3], const bf16x8_t (&b)[3], f32x4 c) {
  c = mfma_bf(a[1], b[1], c);
  c = mfma_bf(a[2], b[0], c);
  c = mfma_bf(a[0], b[2], c);
  c = mfma_bf(a[1], b[0], c);
  c = mfma_bf(a[0], b[1], c);
  return mfma_bf(a[0], b[0], c);
}

// hi / mid / lo of two values as three packed dwords (value 0 in the low half)
__device__ __forceinline__ void split_pair(float x0, float x1, uint32_t (&w)[3]) {
  __bf16 h0, m0, l0, h1, m1, l1;
  split3(x0, h0, m0, l0);
  split3(x1, h1, m1, l1);
  w[0] = (uint32_t)__builtin_bit_cast(uint16_t, h0) | ((uint32_t)__builtin_bit_cast(uint16_t, h1) << 16);
  w[1] = (uint32_t)__builtin_bit_cast(uint16_t, m0) | ((uint32_t)__builtin_bit_cast(uint16_t, m1) << 16);
  w[2] = (uint32_t)__builtin_bit_cast(uint16_t, l0) | ((uint32_t)__builtin_bit_cast(uint16_t, l1) << 16);
}

// N consecutive floats from a 4-byte-aligned address as dwordx4 runs + a dword tail
// (gfx950 global loads take unaligned vector addresses).
typedef f32x4 f32x4u __attribute__((aligned(4)));
template <int N>
__device__ __forceinline__ void load_run(const float* __restrict__ p, float (&out)[N]) {
#pragma unroll
  for (int i = 0; i + 4 <= N; i += 4) {
    const f32x4 v = *(const f32x4u*)(p + i);
    out[i] = v[0];
    out[i + 1] = v[1];
    out[i + 2] = v[2];
    out[i + 3] = v[3];
  }
#pragma unroll
  for (int i = N & ~3; i < N; ++i) out[i] = p[i];
}

// A operands of key/position tiles t0 .. t0+3 for the 16x16x4 MFMA: lane (r, g) takes
// columns g*DQ .. g*DQ+DQ-1 of row 16t+r (rows clamped to T-1).
template <int DQ>
__device__ __forceinline__ void load_group(const float* __restrict__ base, int C, int t0, int r,
                                           int g, int T, float (&dst)[4][DQ]) {
#pragma unroll
  for (int u = 0; u < 4; ++u)
    load_run<DQ>(base + (size_t)min(16 * (t0 + u) + r, T - 1) * C + g * DQ, dst[u]);
}

// Buffer descriptor over one (batch row or pass, head) slice of a [rows][H*d] tensor:
// [base, base + bytes); loads past it return 0 (hardware range check), so rows >= T need no
// clamp, and every offset is a 32-bit VGPR / SGPR / immediate sum (no 64-bit address math
// per load).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t slice_rsrc(const float* base, int T, int C,
                                                             int D) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0,
                                           (int)(((size_t)(T - 1) * C + D) * sizeof(float)),
                                           0x00020000);
}

// A operands of key/position tiles t0 .. t0+3 for the 16x16x4 MFMA from a slice: lane
// (r, g) takes columns g*DQ .. g*DQ+DQ-1 of row 16t+r (voff = (r*C + g*DQ) * 4; rows >= T
// read 0).
template <int DQ>
__device__ __forceinline__ void load_group_buf(__amdgpu_buffer_rsrc_t rs, int voff, int C, int t0,
                                               float (&dst)[4][DQ]) {
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int soff = 64 * (t0 + u) * C;  // 16 rows
#pragma unroll
    for (int i = 0; i + 4 <= DQ; i += 4) {
      const f32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, voff + 4 * i, soff, 0);
      dst[u][i] = v[0];
      dst[u][i + 1] = v[1];
      dst[u][i + 2] = v[2];
      dst[u][i + 3] = v[3];
    }
#pragma unroll
    for (int i = DQ & ~3; i < DQ; ++i)
      dst[u][i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, voff + 4 * i, soff, 0));
  }
}

// Bijective XCD-aware remap (hardware block b runs on XCD b % 8): consecutive logical ids
// share an XCD, so the query tiles and heads of one batch row -- which read the same
// q/k/v/pos cache lines (heads are column slices of one row) -- share one L2.
__device__ __forceinline__ int xcd_logical(int b, int nb) {
  const int q = nb / 8, r = nb % 8, x = b % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

struct BlockId {
  int qt, h, b;
};

// 1-D grid of nqt * H * Bt blocks -> (query tile, head, batch row), tile fastest.
__device__ __forceinline__ BlockId block_id(int nqt, int H) {
  const int L = xcd_logical((int)blockIdx.x, (int)gridDim.x);
  BlockId id;
  id.qt = L % nqt;
  const int rest = L / nqt;
  id.h = rest % H;
  id.b = rest / H;
  return id;
}

// first float of probs fragment tile (a, t) of (batch row, head) bh
__device__ __forceinline__ size_t frag_off(int bh, int a, int t, int nt) {
  return (((size_t)bh * nt + a) * nt + t) * 256;
}

__device__ __forceinline__ uint64_t drop_row_base(int bh, int T, int i) {  // even
  return ((uint64_t)bh * T + i) * (uint64_t)(T + (T & 1));
}

#ifdef OB_ATTN_STAMPS
// diagnostic build only (tools/attn_stamps.py): per-wave cycles of up to 10 phases of ONE
// kernel (OB_ATTN_STAMPS = 1 flash-style backward, 2 query-side backward, 3 forward,
// 4 key-side backward), written to a buffer nothing else reads
__device__ uint64_t g_attn_stamps[65536];
__device__ uint64_t g_attn_rt[16384];  // per wave: s_memrealtime (100 MHz) at start and end
#define OB_STAMP_DECL(K)                                                       \
  constexpr bool st_on = OB_ATTN_STAMPS == (K);                                \
  uint64_t st_t = st_on ? __builtin_amdgcn_s_memtime() : 0,                   \
           st_rt0 = st_on ? __builtin_amdgcn_s_memrealtime() : 0,             \
           st_acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#define OB_STAMP(k)                                          \
  do {                                                       \
    if constexpr (st_on) {                                   \
      const uint64_t st_n = __builtin_amdgcn_s_memtime();    \
      st_acc[k] += st_n - st_t;                              \
      st_t = st_n;                                           \
    }                                                        \
  } while (0)
#define OB_STAMP_WRITE(NWV)                                                             \
  if constexpr (st_on) {                                                                \
    const uint64_t st_rt1 = __builtin_amdgcn_s_memrealtime();                           \
    const size_t st_w = (size_t)blockIdx.x * (NWV) + w;                                 \
    if (lane == 0 && st_w * 10 + 10 <= 65536)                                           \
      for (int k_ = 0; k_ < 10; ++k_) g_attn_stamps[st_w * 10 + k_] = st_acc[k_];       \
    if (lane == 0 && st_w * 2 + 2 <= 16384) {                                           \
      g_attn_rt[st_w * 2] = st_rt0;                                                     \
      g_attn_rt[st_w * 2 + 1] = st_rt1;                                                 \
    }                                                                                   \
  }
#else
#define OB_STAMP_DECL(K)
#define OB_STAMP(k) \
  do {              \
  } while (0)
#define OB_STAMP_WRITE(NWV)
#endif

// ------------------------------------------------------------------------------------
// Forward: block = (query tile of 64, head, batch row). The Xpad image of rows i0 .. i0+64
// lives in LDS (row 64 = the next tile's first query, read by the last rows' j >= i+2
// entries), then the same space holds v for the context product.
// ------------------------------------------------------------------------------------
template <int DQ, int NTT>
__global__ __launch_bounds__(kThreads) void relattn_fwd_kernel(
    const float* __restrict__ q, const float* __restrict__ k, const float* __restrict__ v,
    const float* __restrict__ pos, const float* __restrict__ u, const float* __restrict__ vbias,
    const int* __restrict__ lens, int Bp, int T, int H, float inv_sqrt_d, DropCfg dc,
    const uint64_t* __restrict__ rng, uint64_t rng_off, float* __restrict__ probs,
    float* __restrict__ stats, uint32_t* __restrict__ kbits, float* __restrict__ anchors,
    float* __restrict__ ctx) {
  constexpr int D = 4 * DQ;
  constexpr int CT = (D + 15) / 16;
  extern __shared__ float img[];
  const int nt = (T + 15) >> 4;
  const int ldi = T + 1;  // Xpad pitch
  const BlockId bid = block_id((T + kTile - 1) / kTile, H);
  const int b = bid.b, h = bid.h, i0 = bid.qt * kTile;
  const int bh = b * H + h;
  const int pass = b / Bp;
  const int C = H * D;
  const int L = min(lens[b], T);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 15, g = lane >> 4;
  const float* qb = q + (size_t)b * T * C + h * D;
  const float* kb = k + (size_t)b * T * C + h * D;
  const float* vbp = v + (size_t)b * T * C + h * D;
  const float* pb = pos + (size_t)pass * T * C + h * D;
  const float* ub = u + h * D;
  const float* vbb = vbias + h * D;
  const __amdgpu_buffer_rsrc_t rs_p = slice_rsrc(pb, T, C, D), rs_k = slice_rsrc(kb, T, C, D);
  const int voff_a = (r * C + g * DQ) * 4;  // this lane's A-operand run in a 16-row group
  OB_STAMP_DECL(3)

  const int ir = 16 * w + r;  // this lane's query row in the tile (scores phase)
  const int qi = i0 + ir;
  const int qic = min(qi, T - 1);
  float qu[DQ], qv[DQ];
  {
    float x[DQ];
    load_run<DQ>(qb + (size_t)qic * C + g * DQ, x);
#pragma unroll
    for (int s = 0; s < DQ; ++s) {
      const int c = g * DQ + s;
      qu[s] = x[s] + ub[c];
      qv[s] = x[s] + vbb[c];
    }
  }

  // X = (q + v) p^T for the wave's 16 rows: D[pos][query] with A = p rows, B = (q+v),
  // four position tiles at a time (next group's p rows loading meanwhile), stored as
  // Xpad rows: img[ir][1 + m] = X[qi][m], img[ir][0] = 0.
  // (two operand buffers used alternately by the fully unrolled group loop: no copies)
  float opb[2][4][DQ];
  load_group_buf<DQ>(rs_p, voff_a, C, 0, opb[0]);
  OB_STAMP(0);
#pragma unroll
  for (int t0 = 0; t0 < NTT; t0 += 4) {
    if (t0 >= nt) continue;
    float (&opa)[4][DQ] = opb[(t0 >> 2) & 1];
    if (t0 + 4 < NTT && t0 + 4 < nt) load_group_buf<DQ>(rs_p, voff_a, C, t0 + 4, opb[((t0 >> 2) + 1) & 1]);
    f32x4 acc[4];
#pragma unroll
    for (int uu = 0; uu < 4; ++uu) acc[uu] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < DQ; ++s)
#pragma unroll
      for (int uu = 0; uu < 4; ++uu) acc[uu] = mfma4(opa[uu][s], qv[s], acc[uu]);
#pragma unroll
    for (int uu = 0; uu < 4; ++uu) {
      const int t = t0 + uu;
      if (t >= nt) continue;
      float* dst = img + ir * ldi + 1 + 16 * t + 4 * g;
      if (16 * t + 15 < T) {
#pragma unroll
        for (int j = 0; j < 4; ++j) dst[j] = acc[uu][j];
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (16 * t + 4 * g + j < T) dst[j] = acc[uu][j];  // (m >= T: the next row's zero)
      }
    }
  }
  if (g == 0) img[ir * ldi] = 0.0f;
  OB_STAMP(1);
  // the first key group of the scores phase, in flight over the row-64 work and barrier
  load_group_buf<DQ>(rs_k, voff_a, C, 0, opb[0]);
  // Xpad row 64: the next tile's first query (fp32 fma chain on the VALU)
  if (i0 + kTile < T) {
    const float* qe = qb + (size_t)(i0 + kTile) * C;
    for (int m = threadIdx.x; m < T; m += kThreads) {
      float pr[D];
      load_run<D>(pb + (size_t)m * C, pr);
      // (columns in order: this row only feeds the upper rel_shift part of row 63 of the tile;
      // the flash-style backward recomputes that row from the MFMA-computed anchor, which can
      // differ from this one in the last bit)
      float a = 0.0f;
#pragma unroll
      for (int c = 0; c < D; ++c) a = fmaf(qe[c] + vbb[c], pr[c], a);
      img[kTile * ldi + 1 + m] = a;
    }
    if (threadIdx.x == 0) img[kTile * ldi] = 0.0f;
  }
  OB_STAMP(2);
  __syncthreads();
  OB_STAMP(3);
  // X rows of the queries 32, 64, 96, ... (< T): the rows just below each 32-query chunk of
  // the flash-style backward, which reads them instead of recomputing them
  if (anchors) {
    const int nchk = (16 * nt + 31) / 32;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const int row = i0 + 32 * half;
      if (row < 32 || row >= T) continue;
      float* dst = anchors + ((size_t)bh * nchk + row / 32 - 1) * T;
      for (int m = threadIdx.x; m < T; m += kThreads) dst[m] = img[32 * half * ldi + 1 + m];
    }
  }

  // scores for (query qi, keys 16t+4g+j): ac by MFMA (A = k rows, B = q+u); bd read flat
  float sreg[NTT][4];
  float mx = -INFINITY;
  const float* bdp = img + (T + ir * T + 4 * g - i0);  // bd[qi][16t+4g+j] = bdp[16t + j]
  const int Lq = qi < L ? L : 0;                        // valid keys of this row
#pragma unroll
  for (int t0 = 0; t0 < NTT; t0 += 4) {
    if (t0 >= nt) continue;
    float (&opa)[4][DQ] = opb[(t0 >> 2) & 1];
    if (t0 + 4 < NTT && t0 + 4 < nt) load_group_buf<DQ>(rs_k, voff_a, C, t0 + 4, opb[((t0 >> 2) + 1) & 1]);
    f32x4 acc4[4];
#pragma unroll
    for (int uu = 0; uu < 4; ++uu) acc4[uu] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < DQ; ++s)
#pragma unroll
      for (int uu = 0; uu < 4; ++uu) acc4[uu] = mfma4(opa[uu][s], qu[s], acc4[uu]);
#pragma unroll
    for (int uu = 0; uu < 4; ++uu) {
      const int t = t0 + uu;
      if (t >= nt) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float sc = (acc4[uu][j] + bdp[16 * t + j]) * inv_sqrt_d;
        sreg[t][j] = 16 * t + 4 * g + j < Lq ? sc : -INFINITY;
        mx = fmaxf(mx, sreg[t][j]);
      }
    }
  }
  mx = xmax_1632(mx);
  OB_STAMP(4);
  // v rows of the ctx product's first key chunk, in flight over the softmax (DQ <= 9: the
  // registers are free; wider heads load at staging)
  constexpr int kVSlots = (kFwdKeyChunk / 2 * DQ + kThreads - 1) / kThreads;
  constexpr bool kVPre = DQ <= 9;
  const int nkp0 = min(kFwdKeyChunk, 32 * ((nt + 1) >> 1)) / 2;  // key pairs of chunk 0
  f32x4 vpre[kVPre ? kVSlots : 1][2];
  if constexpr (kVPre) {
#pragma unroll
    for (int sl = 0; sl < kVSlots; ++sl) {
      const int e = threadIdx.x + kThreads * sl;
      const int kp = e / DQ, cq = e - kp * DQ;
      const bool ok = e < nkp0 * DQ;
      vpre[sl][0] = ok && 2 * kp < T ? *(const f32x4u*)(vbp + (size_t)(2 * kp) * C + 4 * cq)
                                     : f32x4{0.f, 0.f, 0.f, 0.f};
      vpre[sl][1] = ok && 2 * kp + 1 < T ? *(const f32x4u*)(vbp + (size_t)(2 * kp + 1) * C + 4 * cq)
                                         : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  const bool row_live = mx != -INFINITY;  // all -inf -> softmax NaN -> nan_to_num 0
  const float mxs = row_live ? mx : 0.0f;
  float sum = 0.0f;
#pragma unroll
  for (int t = 0; t < NTT; ++t) {
    if (t >= nt) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float e = __expf(sreg[t][j] - mxs);  // exp(-inf) = 0
      sreg[t][j] = e;
      sum += e;
    }
  }
  sum = xsum_1632(sum);
  const float rsum = row_live ? 1.0f / sum : 0.0f;
  const int Tp = 16 * nt;  // rows / keys of the saved state
  if (stats && g == 0 && qi < Tp) {
    stats[2 * ((size_t)bh * Tp + qi)] = mxs;
    stats[2 * ((size_t)bh * Tp + qi) + 1] = rsum;
  }
  const uint32_t dkey = dc.on ? drop_key(rng[0], rng[1] + rng_off) : 0u;
  // keys 16t+4g .. +3 are the element pairs pb + 8t and pb + 8t + 1 of the row's hash index
  // (drop_row_base is even): 32-bit pair arithmetic, the hashes keep4 draws
  const DropPairRow dr = drop_pair_row(dkey, (drop_row_base(bh, T, qi) + 4 * g) >> 1);
  const bool want_kw = kbits != nullptr && dc.on;  // keep bits saved (flash-style backward)
  uint32_t kw[(NTT + 1) / 2];  // keep bits of keys 32wd .. 32wd + 31 (this lane's share)
#pragma unroll
  for (int wd = 0; wd < (NTT + 1) / 2; ++wd) kw[wd] = 0u;
  // this wave's row tile of probs (waves past the last row tile -- T not a multiple of
  // 64 -- store nothing); the test is wave-uniform
  const int arow = (i0 >> 4) + __builtin_amdgcn_readfirstlane(w);
  const bool store_p = probs != nullptr && arow < nt;
  float* pf = probs + (store_p ? frag_off(bh, arow, 0, nt) : 0) + 4 * lane;
#pragma unroll
  for (int t = 0; t < NTT; ++t) {
    if (t >= nt) continue;
    // dropout off: thresh 0, every field keeps
    uint32_t h0 = 0xFFFFFFFFu, h1 = 0xFFFFFFFFu;
    if (dc.on) {
      h0 = drop_hash_at(dr, 8 * t);
      h1 = drop_hash_at(dr, 8 * t + 1);
    }
    const bool keep[4] = {(h0 & 0xFFFFu) >= dc.thresh, (h0 >> 16) >= dc.thresh,
                          (h1 & 0xFFFFu) >= dc.thresh, (h1 >> 16) >= dc.thresh};
    if (want_kw) {
      const uint32_t nib = (keep[0] ? 1u : 0u) | (keep[1] ? 2u : 0u) | (keep[2] ? 4u : 0u) |
                           (keep[3] ? 8u : 0u);
      kw[t >> 1] |= nib << (16 * (t & 1) + 4 * g);
    }
    f32x4 st;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float pr = sreg[t][j] * rsum;
      // the keep decision rides in the sign bit (P >= 0): the backward kernels read it
      // back instead of re-hashing every element
      st[j] = keep[j] ? pr : -pr;
      // (dropout off: every element keeps and dc.scale is 1, so this is pr)
      sreg[t][j] = keep[j] ? pr * dc.scale : 0.0f;
    }
    if (store_p) *reinterpret_cast<f32x4*>(pf + 256 * t) = st;
  }
  if (want_kw) {
    const int W = (nt + 1) >> 1;
#pragma unroll
    for (int wd = 0; wd < (NTT + 1) / 2; ++wd) {
      uint32_t x = kw[wd];
      x = xor_1632(x);
      if (wd < W && g == 0 && qi < Tp) kbits[((size_t)bh * Tp + qi) * W + wd] = x;
    }
  }

  // ctx = A v on bf16x6 (16x16x32, exact fp32 products): k step c = keys 32c .. 32c+31;
  // A = the lane's 8 probabilities of its query (keys 32c+4g..+3 of tile 2c and
  // 32c+16+4g..+3 of tile 2c+1: a permuted k order), split in registers; B = v^T parts
  // [col][key] in LDS read in the same order (two ds_read_b64 per part). v of (b, h) is staged
  // into the image space (free once every wave has passed the scores phase), up to
  // kFwdKeyChunk keys at a time: each thread splits two consecutive keys of 4 columns, one
  // packed dword per part.
  constexpr int DPc = 16 * CT;
  const int KPc = 32 * ((nt + 1) >> 1);      // keys covered by the k steps (zero past T)
  const int VP = min(KPc, kFwdKeyChunk) + 8;  // bf16 per part row (pad: conflict-free b64 reads)
  __bf16* vpl = reinterpret_cast<__bf16*>(img);
  f32x4 o[CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) o[ct] = f32x4{0.f, 0.f, 0.f, 0.f};
  // keys in chunks of kFwdKeyChunk (one chunk up to T = 256): stage, then the chunk's k steps
#pragma unroll
  for (int ch = 0; ch < (16 * NTT + kFwdKeyChunk - 1) / kFwdKeyChunk; ++ch) {
    const int kb0 = ch * kFwdKeyChunk;
    if (kb0 >= KPc) continue;
    const int nkp = min(kFwdKeyChunk, KPc - kb0) / 2;  // key pairs staged
    OB_STAMP(5);
    __syncthreads();  // the image (first chunk) / the previous chunk's parts are read
    OB_STAMP(6);
    auto put_v = [&](int kp, int cq, const f32x4& v0, const f32x4& v1) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        uint32_t wds[3];
        split_pair(v0[j], v1[j], wds);
#pragma unroll
        for (int p = 0; p < 3; ++p)
          *reinterpret_cast<uint32_t*>(vpl + ((size_t)p * DPc + 4 * cq + j) * VP + 2 * kp) = wds[p];
      }
    };
    if (kVPre && ch == 0) {
#pragma unroll
      for (int sl = 0; sl < kVSlots; ++sl) {
        const int e = threadIdx.x + kThreads * sl;
        if (e < nkp * DQ) put_v(e / DQ, e % DQ, vpre[sl][0], vpre[sl][1]);
      }
    } else {
      for (int e = threadIdx.x; e < nkp * DQ; e += kThreads) {
        const int kp = e / DQ, cq = e - kp * DQ;
        const int key = kb0 + 2 * kp;
        f32x4 v0 = f32x4{0.f, 0.f, 0.f, 0.f}, v1 = f32x4{0.f, 0.f, 0.f, 0.f};
        if (key < T) v0 = *(const f32x4u*)(vbp + (size_t)key * C + 4 * cq);
        if (key + 1 < T) v1 = *(const f32x4u*)(vbp + (size_t)(key + 1) * C + 4 * cq);
        put_v(kp, cq, v0, v1);
      }
    }
    if constexpr (DPc > D) {
      for (int e = threadIdx.x; e < 3 * (DPc - D) * nkp; e += kThreads) {  // columns >= D
        const int pc = e / nkp, kp = e - pc * nkp;
        const int p = pc / (DPc - D), col = D + pc % (DPc - D);
        *reinterpret_cast<uint32_t*>(vpl + ((size_t)p * DPc + col) * VP + 2 * kp) = 0u;
      }
    }
    OB_STAMP(7);
    __syncthreads();
    OB_STAMP(8);
#pragma unroll
    for (int kl = 0; kl < kFwdKeyChunk / 32; ++kl) {
      const int kc = ch * (kFwdKeyChunk / 32) + kl;  // k step: keys 32kc .. 32kc+31
      if (kc >= (NTT + 1) / 2 || 2 * kc >= nt) continue;
      float a8[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        a8[j] = sreg[2 * kc][j];
        a8[4 + j] = 2 * kc + 1 < nt ? sreg[2 * kc + 1][j] : 0.0f;
      }
      bf16x8_t af[3];
      split8(a8, af);
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        bf16x8_t bfr[3];
#pragma unroll
        for (int p = 0; p < 3; ++p) {
          const __bf16* row = vpl + ((size_t)p * DPc + 16 * ct + r) * VP + 32 * kl + 4 * g;
          const bf16x4_t lo = *reinterpret_cast<const bf16x4_t*>(row);
          const bf16x4_t hi = *reinterpret_cast<const bf16x4_t*>(row + 16);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            bfr[p][j] = lo[j];
            bfr[p][4 + j] = hi[j];
          }
        }
        o[ct] = mfma_x6(af, bfr, o[ct]);
      }
    }
  }
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    const int col = 16 * ct + r;
    if (col >= D) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = i0 + 16 * w + 4 * g + j;
      if (row < T) ctx[((size_t)b * T + row) * C + h * D + col] = o[ct][j];
    }
  }
  OB_STAMP(9);
  OB_STAMP_WRITE(kThreads / 64)
}

// ------------------------------------------------------------------------------------
// Backward, query side: block = (query tile, head, batch row). Writes dq (final), the
// tile's du / dvb partials (summed by relattn_reduce_kernel) and dS' = dS / sqrt(d)
// to global for the key-side kernel. The softmax backward's row term is
//   delta_i = sum_j Pd_ij dPd_ij = dO_i . ctx_i
// (ctx = Pd v), so each score's dS' is formed as soon as its dP tile is: no parking of dP.
// LDS holds dS' rows i0-1 .. i0+63 at pitch T (band row 0 = query i0-1, recomputed here on
// the VALU; zero when i0 == 0) -- the rows the rel_shift adjoint of the tile reads.
// ------------------------------------------------------------------------------------
template <int DQ, int NTT>
__global__ __launch_bounds__(kThreads) void relattn_bwd_kernel(
    const float* __restrict__ dctx, const float* __restrict__ ctxo, const float* __restrict__ k,
    const float* __restrict__ v, const float* __restrict__ pos, int Bp, int T, int H,
    float inv_sqrt_d, DropCfg dc, const float* __restrict__ probs, float* __restrict__ dq,
    float* __restrict__ dsg, float* __restrict__ du_part, float* __restrict__ dvb_part) {
  constexpr int D = 4 * DQ;
  constexpr int CT = (D + 15) / 16;
  extern __shared__ float band[];
  __shared__ float red[kThreads / 64][2][64];
  const int nt = (T + 15) >> 4;
  const int nqt = (T + kTile - 1) / kTile;
  const BlockId bid = block_id(nqt, H);
  const int b = bid.b, h = bid.h, qt = bid.qt, i0 = qt * kTile;
  const int bh = b * H + h;
  const int pass = b / Bp;
  const int C = H * D;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 15, g = lane >> 4;
  const size_t bo = (size_t)b * T * C + h * D;
  const float* kb = k + bo;
  const float* vbp = v + bo;
  const float* dob = dctx + bo;
  const float* cob = ctxo + bo;
  const float* pb = pos + (size_t)pass * T * C + h * D;
  const __amdgpu_buffer_rsrc_t rs_v = slice_rsrc(vbp, T, C, D), rs_k = slice_rsrc(kb, T, C, D),
                               rs_p = slice_rsrc(pb, T, C, D);
  const int voff_a = (r * C + g * DQ) * 4;  // this lane's A-operand run in a 16-row group
  // dropout backward factor from a stored probability's sign bit (the forward's keep bit)
  auto keep_scale = [&](float pv) -> float {
    if (!dc.on) return 1.0f;
    return __builtin_signbit(pv) ? 0.0f : dc.scale;
  };
  // the band's slack past its 65 rows (read only by rows >= T and padded positions)
  if (threadIdx.x < 128) band[(kTile + 1) * T + threadIdx.x] = 0.0f;
  OB_STAMP_DECL(2)

  const int ir = 16 * w + r;
  const int qi = i0 + ir;
  const int qic = min(qi, T - 1);
  float dor[DQ];
  load_run<DQ>(dob + (size_t)qic * C + g * DQ, dor);
  float delta;
  {
    float cr[DQ];
    load_run<DQ>(cob + (size_t)qic * C + g * DQ, cr);
    float a = 0.0f;
#pragma unroll
    for (int s = 0; s < DQ; ++s) a = fmaf(dor[s], cr[s], a);
    a = xsum_1632(a);
    delta = a;
  }
  OB_STAMP(0);

  // dPd[query qi][key] = dO . v (A = v rows, B = dO row); P from the fragment tiles;
  // dS' = P (dPd * keep * scale - delta) / sqrt(d) (softmax backward, then the 1/sqrt(d))
  // (waves past the last row tile of probs -- T not a multiple of 64 -- read zeros)
  const bool arow_ok = (i0 >> 4) + w < nt;
  const float* pf = probs + frag_off(bh, arow_ok ? (i0 >> 4) + w : 0, 0, nt) + 4 * lane;
  float* brow = band + (1 + ir) * T + 4 * g;  // band row of query qi
  float dsr[NTT][4];
  float opb[2][4][DQ];
  load_group_buf<DQ>(rs_v, voff_a, C, 0, opb[0]);
#pragma unroll
  for (int t0 = 0; t0 < NTT; t0 += 4) {
    if (t0 >= nt) continue;
    float (&opa)[4][DQ] = opb[(t0 >> 2) & 1];
    if (t0 + 4 < NTT && t0 + 4 < nt) load_group_buf<DQ>(rs_v, voff_a, C, t0 + 4, opb[((t0 >> 2) + 1) & 1]);
    f32x4 p4[4];
#pragma unroll
    for (int uu = 0; uu < 4; ++uu)
      p4[uu] = arow_ok && t0 + uu < nt ? *reinterpret_cast<const f32x4*>(pf + 256 * (t0 + uu))
                                       : f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 acc4[4];
#pragma unroll
    for (int uu = 0; uu < 4; ++uu) acc4[uu] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < DQ; ++s)
#pragma unroll
      for (int uu = 0; uu < 4; ++uu) acc4[uu] = mfma4(opa[uu][s], dor[s], acc4[uu]);
#pragma unroll
    for (int uu = 0; uu < 4; ++uu) {
      const int t = t0 + uu;
      if (t >= nt) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float pv = p4[uu][j];
        const float dp = acc4[uu][j] * keep_scale(pv);  // dropout backward
        const float ds = (fabsf(pv) * (dp - delta)) * inv_sqrt_d;
        dsr[t][j] = ds;
      }
      if (16 * t + 15 < T) {
#pragma unroll
        for (int j = 0; j < 4; ++j) brow[16 * t + j] = dsr[t][j];
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (16 * t + 4 * g + j < T) brow[16 * t + j] = dsr[t][j];
      }
    }
  }

  OB_STAMP(1);
  // band row 0: query i0-1 on the VALU, the same formula (zero row when i0 == 0)
  if (i0 > 0) {
    const int ip = i0 - 1;
    const float* drow = dob + (size_t)ip * C;
    const float* crow = cob + (size_t)ip * C;
    float dl = 0.0f;
#pragma unroll
    for (int c = 0; c < D; ++c) dl = fmaf(drow[c], crow[c], dl);
    const float* pr = probs + frag_off(bh, ip >> 4, 0, nt) + 4 * (ip & 15);
    for (int jj = threadIdx.x; jj < T; jj += kThreads) {
      float vr[D];
      load_run<D>(vbp + (size_t)jj * C, vr);
      float a = 0.0f;
#pragma unroll
      for (int c = 0; c < D; ++c) a = fmaf(vr[c], drow[c], a);
      const float pv = pr[256 * (jj >> 4) + 64 * ((jj & 15) >> 2) + (jj & 3)];
      band[jj] = (fabsf(pv) * (a * keep_scale(pv) - dl)) * inv_sqrt_d;
    }
  } else {
    for (int jj = threadIdx.x; jj < T; jj += kThreads) band[jj] = 0.0f;
  }
  OB_STAMP(2);

  // dQu = dS' k (A = dS' row r, k = 4g+j of tile t; B = k rows)
  f32x4 oq[CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) oq[ct] = f32x4{0.f, 0.f, 0.f, 0.f};
  // (B operands k[16t+4g+j][16ct+r] of tile t+1 load while tile t's MFMAs issue)
  // (rows >= T read 0; columns >= D of a head read the next head's values, which only
  // feed output columns that are never stored)
  const int voff_b = (4 * g * C + r) * 4;
  auto load_b = [&](int t, float (&dst)[4][CT]) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int ct = 0; ct < CT; ++ct)
        dst[j][ct] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                   rs_k, voff_b + 4 * (j * C + 16 * ct), 64 * t * C, 0));
  };
  {
    float kbb[2][4][CT];
    load_b(0, kbb[0]);
#pragma unroll
    for (int t = 0; t < NTT; ++t) {
      if (t >= nt) continue;
      if (t + 1 < NTT && t + 1 < nt) load_b(t + 1, kbb[(t + 1) & 1]);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) oq[ct] = mfma4(dsr[t][j], kbb[t & 1][j][ct], oq[ct]);
    }
  }
  OB_STAMP(3);
  __syncthreads();  // the band is complete (row 0 and every wave's rows)
  OB_STAMP(4);

  // dQv = dX p, dX read flat from the band: dX[qi][m] = dS'.flat[qi(T+1) + m + 1 - T]
  // = band[i0 + 1 + ir(T+1) + m] (band row 0 = query i0-1, zero for the first tile).
  // Positions m = 4mk+g go eight MFMA steps at a time, the next eight's p operands loading
  // meanwhile; positions past T multiply p = 0.
  f32x4 ov[CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) ov[ct] = f32x4{0.f, 0.f, 0.f, 0.f};
  const float* xrow = band + i0 + 1 + ir * (T + 1) + g;  // dX[qi][4mk + g] = xrow[4mk]
  const int nk = (T + 3) >> 2;
  constexpr int kMK = 8;  // eight MFMA steps per round, the next round's p loading meanwhile
  // p[4mk + g][16ct + r]: positions >= T read 0 (range check)
  const int voff_pm = (g * C + r) * 4;
  auto load_p = [&](int mk0, float (&dst)[kMK][CT]) {
#pragma unroll
    for (int qq = 0; qq < kMK; ++qq)
#pragma unroll
      for (int ct = 0; ct < CT; ++ct)
        dst[qq][ct] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                    rs_p, voff_pm + 64 * ct, 16 * (mk0 + qq) * C, 0));
  };
  float pv_cur[kMK][CT];
  load_p(0, pv_cur);
  for (int mk0 = 0; mk0 < nk; mk0 += kMK) {
    float pv_nxt[kMK][CT];
    if (mk0 + kMK < nk) load_p(mk0 + kMK, pv_nxt);
#pragma unroll
    for (int qq = 0; qq < kMK; ++qq) {
      const float av = mk0 + qq < nk ? xrow[4 * (mk0 + qq)] : 0.0f;
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) ov[ct] = mfma4(av, pv_cur[qq][ct], ov[ct]);
    }
#pragma unroll
    for (int qq = 0; qq < kMK; ++qq)
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) pv_cur[qq][ct] = pv_nxt[qq][ct];
  }
  OB_STAMP(5);
  // dq = dQu + dQv; per-tile column sums of dQu / dQv for du / dvb
  float su[CT], sv[CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    const int col = 16 * ct + r;
    su[ct] = 0.0f;
    sv[ct] = 0.0f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = i0 + 16 * w + 4 * g + j;
      if (row < T) {
        su[ct] += oq[ct][j];
        sv[ct] += ov[ct][j];
        if (col < D) dq[bo + (size_t)row * C + col] = oq[ct][j] + ov[ct][j];
      }
    }
    su[ct] = xsum_1632(su[ct]);
    sv[ct] = xsum_1632(sv[ct]);
  }
  const size_t tile_id = ((size_t)b * H + h) * nqt + qt;
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    const int col = 16 * ct + r;
    if (g == 0 && col < D) {
      red[w][0][col] = su[ct];
      red[w][1][col] = sv[ct];
    }
  }
  OB_STAMP(6);
  __syncthreads();
  OB_STAMP(7);
  if (threadIdx.x < D) {
    const int c = threadIdx.x;
    du_part[tile_id * D + c] = ((red[0][0][c] + red[1][0][c]) + red[2][0][c]) + red[3][0][c];
    dvb_part[tile_id * D + c] = ((red[0][1][c] + red[1][1][c]) + red[2][1][c]) + red[3][1][c];
  }

  // dS' rows of this tile to global for the key-side kernel: band rows 1 .. 64 are the
  // global rows i0 .. i0+63 at the same pitch T, i.e. one contiguous run -- copied by the
  // whole block, consecutive lanes on consecutive floats (conflict-free LDS reads, 256-B
  // store segments), 8 loads in flight per thread
  float* dsb = dsg + (size_t)bh * T * T + (size_t)i0 * T;
  const int n = min(kTile, T - i0) * T;
  const float* src = band + T;
  for (int e0 = 0; e0 < n; e0 += 8 * kThreads) {
    float v8[8];
#pragma unroll
    for (int q8 = 0; q8 < 8; ++q8) {
      const int e = e0 + q8 * kThreads + threadIdx.x;
      v8[q8] = src[e < n ? e : 0];
    }
#pragma unroll
    for (int q8 = 0; q8 < 8; ++q8) {
      const int e = e0 + q8 * kThreads + threadIdx.x;
      if (e < n) dsb[e] = v8[q8];
    }
  }
  OB_STAMP(8);
  OB_STAMP_WRITE(kThreads / 64)
}

// ------------------------------------------------------------------------------------
// Backward, key side: block = (key tile of 64, head, batch row), wave w = keys 16w..16w+15
// of the tile; every query row is visited (no per-query-tile partials):
//   dK[key]  = sum_i dS'[i][key] (q+u)[i]       dV[key] = sum_i Pd[i][key] dO[i]
//   dpos[m]  = sum_i dX[i][m] (q+v)[i]          (per batch row; summed over the pass later)
// Queries go in chunks of 32. Per chunk the block stages, once for its 4 waves, the A tiles
// dS' / Pd (dropout applied) / dX [32 queries][64 keys] (dwordx4 rows, dX gathered by the
// rel_shift adjoint) and the B tiles q+u / q+v / dO [32 queries][D] in LDS; the next
// chunk's global loads are in flight in registers while the current chunk's MFMAs
// (16x16x4: A[key r][query g], B[query g][column r]) issue. Query order per accumulator is
// ascending, four per MFMA step, as in a plain loop over i.
// ------------------------------------------------------------------------------------
template <int D>
struct KvStage {
  static constexpr int kQ = 32;                       // queries per chunk
  static constexpr int kAP = 80;                      // A pitch (= 16 mod 32: conflict-free)
  static constexpr int kBP = ((D + 16) / 32) * 32 + 16;  // B pitch (= 16 mod 32, >= D)
  static constexpr int kBVec = kQ * (D / 4);          // float4s per B source (q or dO)
  static constexpr int kBSlots = (2 * kBVec + kThreads - 1) / kThreads;
  alignas(16) float ak[kQ][kAP];
  alignas(16) float av[kQ][kAP];
  alignas(16) float ap[kQ][kAP];
  alignas(16) float qu[kQ][kBP];
  alignas(16) float qv[kQ][kBP];
  alignas(16) float dob[kQ][kBP];
};

template <int DQ>
__global__ __launch_bounds__(kThreads) void relattn_bwd_kv_kernel(
    const float* __restrict__ dsg, const float* __restrict__ probs, const float* __restrict__ q,
    const float* __restrict__ dctx, const float* __restrict__ u, const float* __restrict__ vbias,
    int T, int H, DropCfg dc, float* __restrict__ dk, float* __restrict__ dv,
    float* __restrict__ dp_part) {
  constexpr int D = 4 * DQ;
  constexpr int CT = (D + 15) / 16;
  using St = KvStage<D>;
  constexpr int kQ = St::kQ;
  __shared__ St st;
  const int nt = (T + 15) >> 4;
  const int nkt = (T + kTile - 1) / kTile;
  const BlockId bid = block_id(nkt, H);
  const int b = bid.b, h = bid.h, k0 = bid.qt * kTile;
  const int bh = b * H + h;
  const int C = H * D;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 15, g = lane >> 4;
  const size_t bo = (size_t)b * T * C + h * D;
  const float* qb = q + bo;
  const float* dob = dctx + bo;
  const float* ub = u + h * D;
  const float* vbb = vbias + h * D;
  const float* dsb = dsg + (size_t)bh * T * T;
  const float* prb = probs + frag_off(bh, 0, 0, nt);

  // pad columns of the B tiles stay zero (their MFMA columns are discarded anyway)
  for (int e = threadIdx.x; e < kQ * St::kBP; e += kThreads) {
    (&st.qu[0][0])[e] = 0.0f;
    (&st.qv[0][0])[e] = 0.0f;
    (&st.dob[0][0])[e] = 0.0f;
  }

  // staging roles: A -- thread t owns query row t/16, keys k0 + 4(t%16) .. +3;
  // B -- float4 slot e = t + 256 j: q (e < kBVec) or dO, row e/(D/4), columns 4(e%(D/4))..
  constexpr int kAH = kQ / 16;  // A rows per thread (ai, ai + 16, ...)
  const int ai = threadIdx.x >> 4, ax = 4 * (threadIdx.x & 15);
  const int key0 = k0 + ax;
  // P[i][key0 .. +3] is element 0..3 of lane (i & 15) + 16 ((key0 & 15) >> 2) of fragment
  // tile (i / 16, key0 / 16): one aligned dwordx4
  const size_t pcol = (size_t)256 * (key0 >> 4) + 64 * ((key0 & 15) >> 2);
  f32x4 ra_k[kAH], ra_v[kAH], ra_p[kAH], rb[St::kBSlots];
  // buffer descriptors: dS' of (b, h) [T][T], its probs fragment tiles, q / dO slices
  // (loads past a descriptor return 0: rows >= T need no test)
  const __amdgpu_buffer_rsrc_t rs_ds = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(dsb), (short)0, (int)((size_t)T * T * sizeof(float)), 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_pr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(prb), (short)0, (int)((size_t)nt * nt * 256 * sizeof(float)), 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_q = slice_rsrc(qb, T, C, D), rs_do = slice_rsrc(dob, T, C, D);
  const bool kfull = key0 + 3 < T;  // this thread's 4 keys all < T (false only in the last tile)
  auto fetch = [&](int i0) {
#pragma unroll
    for (int hf = 0; hf < kAH; ++hf) {
      const int i = i0 + ai + 16 * hf;
      // dS'[i][key0 .. +3] and dX[i][key0 .. +3] = dS'.flat[i(T+1) + key0 + 1 - T + j] (the
      // rel_shift adjoint read flat; 0 where that index is negative: row 0 only)
      const int fk = i * T + key0, fx = i * (T + 1) + key0 + 1 - T;
      if (kfull && i < T && fx >= 0) {
        ra_k[hf] = __builtin_amdgcn_raw_buffer_load_b128(rs_ds, 4 * fk, 0, 0);
        ra_p[hf] = __builtin_amdgcn_raw_buffer_load_b128(rs_ds, 4 * fx, 0, 0);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const bool ok = i < T && key0 + j < T;
          const float xk = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs_ds, 4 * (fk + j), 0, 0));
          const float xp = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs_ds, 4 * max(fx + j, 0), 0, 0));
          ra_k[hf][j] = ok ? xk : 0.0f;
          ra_p[hf][j] = ok && fx + j >= 0 ? xp : 0.0f;
        }
      }
      // P[i][key0 .. +3]: one aligned dwordx4 of fragment tile (i/16, key0/16) (zeros past T)
      ra_v[hf] = key0 < 16 * nt
                     ? __builtin_amdgcn_raw_buffer_load_b128(
                           rs_pr, 4 * (int)((size_t)(i >> 4) * nt * 256 + pcol + 4 * (i & 15)), 0, 0)
                     : f32x4{0.f, 0.f, 0.f, 0.f};
      // Pd = P * keep * scale, the keep bit from the stored probability's sign
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (dc.on) ra_v[hf][j] = __builtin_signbit(ra_v[hf][j]) ? 0.0f : ra_v[hf][j] * dc.scale;
      }
    }
#pragma unroll
    for (int sl = 0; sl < St::kBSlots; ++sl) {
      const int e = threadIdx.x + kThreads * sl;
      const int e2 = e < St::kBVec ? e : e - St::kBVec;
      const int row = i0 + e2 / DQ, c4 = 4 * (e2 % DQ);
      if (e < 2 * St::kBVec) {
        rb[sl] = __builtin_amdgcn_raw_buffer_load_b128(e < St::kBVec ? rs_q : rs_do,
                                                       4 * (row * C + c4), 0, 0);
      } else {
        rb[sl] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  };
  auto stage = [&]() {
#pragma unroll
    for (int hf = 0; hf < kAH; ++hf) {  // 16-B aligned rows: ds_write_b128
      *(f32x4*)&st.ak[ai + 16 * hf][ax] = ra_k[hf];
      *(f32x4*)&st.av[ai + 16 * hf][ax] = ra_v[hf];
      *(f32x4*)&st.ap[ai + 16 * hf][ax] = ra_p[hf];
    }
#pragma unroll
    for (int sl = 0; sl < St::kBSlots; ++sl) {
      const int e = threadIdx.x + kThreads * sl;
      if (e >= 2 * St::kBVec) continue;
      const int e2 = e < St::kBVec ? e : e - St::kBVec;
      const int row = e2 / DQ, c4 = 4 * (e2 % DQ);
      if (e < St::kBVec) {
        f32x4 xu, xv;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          xu[j] = rb[sl][j] + ub[c4 + j];
          xv[j] = rb[sl][j] + vbb[c4 + j];
        }
        *(f32x4*)&st.qu[row][c4] = xu;
        *(f32x4*)&st.qv[row][c4] = xv;
      } else {
        *(f32x4*)&st.dob[row][c4] = rb[sl];
      }
    }
  };

  f32x4 ak[CT], av[CT], ap[CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    ak[ct] = f32x4{0.f, 0.f, 0.f, 0.f};
    av[ct] = f32x4{0.f, 0.f, 0.f, 0.f};
    ap[ct] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const int kl = 16 * w + r;  // the lane's key within the tile (A row)
  OB_STAMP_DECL(4)
  fetch(0);
  OB_STAMP(0);
  for (int i0 = 0; i0 < T; i0 += kQ) {
    __syncthreads();  // the previous chunk's LDS reads are done
    OB_STAMP(1);
    stage();
    OB_STAMP(2);
    __syncthreads();
    OB_STAMP(3);
    if (i0 + kQ < T) fetch(i0 + kQ);
#pragma unroll
    for (int s4 = 0; s4 < kQ / 4; ++s4) {
      const int qq = 4 * s4 + g;
      const float a_k = st.ak[qq][kl], a_v = st.av[qq][kl], a_p = st.ap[qq][kl];
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        const int col = 16 * ct + r;
        ak[ct] = mfma4(a_k, st.qu[qq][col], ak[ct]);
        av[ct] = mfma4(a_v, st.dob[qq][col], av[ct]);
        ap[ct] = mfma4(a_p, st.qv[qq][col], ap[ct]);
      }
    }
    OB_STAMP(4);
  }
  float* dkb = dk + bo;
  float* dvb = dv + bo;
  float* dpb = dp_part + ((size_t)b * H + h) * T * D;  // [b][h][T][D]
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    const int col = 16 * ct + r;
    if (col >= D) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int kk = k0 + 16 * w + 4 * g + j;
      if (kk >= T) continue;
      dkb[(size_t)kk * C + col] = ak[ct][j];
      dvb[(size_t)kk * C + col] = av[ct][j];
      dpb[(size_t)kk * D + col] = ap[ct][j];
    }
  }
  OB_STAMP(5);
  OB_STAMP_WRITE(kThreads / 64)
}

// ------------------------------------------------------------------------------------
// Backward, flash style (T <= 256): ONE block per (batch row, head) walks the query rows in
// chunks of 32 and recomputes each chunk's probabilities from the forward's row statistics
// (max, 1/sum) and keep bits -- no [T][T] tensor is read or written in HBM. Per chunk:
//   X  = (q+v) pos^T rows (the rel_shift source, LDS image at pitch T+1) and
//   S  = (q+u) k^T + bd, P = exp(S/sqrt(d) - max) / sum   (bitwise the forward's P: same
//        MFMA k order, same VALU expressions),
//   dP = dO v^T, dS' = P (dP keep scale - dO.ctx) / sqrt(d), Pd = P keep scale,
// in the "key on the lane" orientation D[query][key]: lane (key r, queries 4g+e of two
// 16-query tiles) holds 8 queries of one key, which is exactly the A fragment (permuted k
// order) of the key-side products
//   dK += dS'^T (q+u),  dV += Pd^T dO          (bf16x6 on 16x16x32 MFMA, accumulated over
//                                              the chunks in registers: exact fp32 products)
// and dS' goes to an LDS band (pitch T, the previous chunk's last row kept as row 0) for
//   dpos += dX^T (q+v)  (dX = the rel_shift adjoint, read flat from the band; bf16x6)
//   dq    = dS' k + dX pos   (fp32 16x16x4 MFMA, one 16x16 tile per job; K = all keys)
// Wave w owns key tiles / position tiles w*KPW .. w*KPW+KPW-1; the dq tiles are 4*CT jobs
// dealt round-robin (waves w and w+4 share a SIMD: 3 jobs per SIMD at CT = 3, NW = 8).
// du / dvb: per-(b, h) column sums of the dq parts (relattn_reduce_kernel, nqt = 1).
// ------------------------------------------------------------------------------------
constexpr int kFQ = 32;        // query rows per chunk
constexpr int kPlanePitch = 40;  // bf16 per column row of a B plane (80 B: 16-B aligned rows)

// acc[ct] += A^T B for one key tile: A = the lane's 8 queries of its key (fp32, split here),
// B = the chunk's plane (3 parts, [col][query], part stride 16 CT * kPlanePitch) read in the
// same k order: queries 4g..4g+3, then 16+4g..16+4g+3
template <int CT>
__device__ __forceinline__ void key_side(const float (&a8)[8], const __bf16* pl, int g, int r,
                                         f32x4 (&acc)[CT]) {
  bf16x8_t a[3];
  split8(a8, a);
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    bf16x8_t bb[3];
#pragma unroll
    for (int pp = 0; pp < 3; ++pp) {
      const __bf16* pu = pl + (size_t)pp * 16 * CT * kPlanePitch + (16 * ct + r) * kPlanePitch + 4 * g;
      const bf16x4_t u0 = *(const bf16x4_t*)pu, u1 = *(const bf16x4_t*)(pu + 16);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        bb[pp][j] = u0[j];
        bb[pp][4 + j] = u1[j];
      }
    }
    acc[ct] = mfma_x6(a, bb, acc[ct]);
  }
}

// One 16x16 dq tile over all nk k steps of 4 (keys or positions) on 16x16x4 fp32 MFMA: four
// independent accumulation chains (step s = 4n + chain), summed in a fixed order by the
// caller; the next 4 steps' operands load while the current 4 MFMAs issue (two register
// sets, no copies; loads past the last step stay inside LDS / the buffer's range).
// WHICH 0: B from the k image (pitch DP); 1: B = pos rows through the buffer descriptor.
template <int WHICH, int DP>
__device__ __forceinline__ void dq_job(const float* __restrict__ arow, float live,
                                       const float* __restrict__ brow,
                                       __amdgpu_buffer_rsrc_t rs_p, int voff, int C, int sb,
                                       int se, f32x4 (&ac4)[4]) {
#pragma unroll
  for (int qq = 0; qq < 4; ++qq) ac4[qq] = f32x4{0.f, 0.f, 0.f, 0.f};
  arow += 4 * sb;
  if (WHICH == 0) brow += 4 * sb * DP;
  const int nk = se - sb;
  const int sbase = 16 * sb * C;  // (WHICH 1: byte offset of row 4 sb)
  auto ld = [&](int s0, float (&A)[4], float (&B)[4]) {
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
      A[qq] = arow[4 * (s0 + qq)];
      if (WHICH == 0)
        B[qq] = brow[4 * (s0 + qq) * DP];
      else
        B[qq] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                              rs_p, voff, sbase + 16 * (s0 + qq) * C, 0));
    }
  };
  float A0[4], B0[4], A1[4], B1[4];
  ld(0, A0, B0);
  for (int s0 = 0; s0 < nk; s0 += 8) {
    ld(s0 + 4, A1, B1);
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) ac4[qq] = mfma4(A0[qq] * live, B0[qq], ac4[qq]);
    ld(s0 + 8, A0, B0);
    if (s0 + 4 < nk)
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) ac4[qq] = mfma4(A1[qq] * live, B1[qq], ac4[qq]);
  }
}

struct FusedLds {  // float offsets into the dynamic LDS of relattn_bwd_fused_kernel
  int kimg, reg, qu, qv, dO, planes, stats, delta, dpart, kb, comb, sums, total;
  __host__ __device__ FusedLds(int T, int D, int CT, int nch, int W) {
    const int Tp16 = 16 * ((T + 15) / 16);
    const int ap = D + 1;                      // A-image pitch
    kimg = 0;                                  // k rows [Tp][16 CT] (zero pad)
    reg = kimg + Tp16 * 16 * CT;               // prev row [T] + X image / dS' band
    qu = reg + T + 33 * (T + 1);               // (q+u) rows [32][ap]
    qu = (qu + 3) & ~3;
    qv = qu + kFQ * ap;                        // (q+v) rows [32][ap]
    dO = qv + kFQ * ap;                        // dO rows [32][ap]
    planes = dO + kFQ * ap;                    // bf16 [3 tensors][3 parts][16 CT][40]
    planes = (planes + 3) & ~3;                // 16-B aligned
    stats = planes + (9 * 16 * CT * kPlanePitch) / 2;
    delta = stats + 2 * kFQ * nch;             // [32]
    dpart = delta + kFQ;                       // dO.ctx partials [32][D/4]
    kb = dpart + kFQ * (D / 4);                // keep bits [32][W]
    comb = kb + kFQ * W;                       // dq parts [2 which][2 a][CT][2 half][256]
    sums = comb + 2 * 2 * CT * 2 * 256;        // column sums [2 which][2 a][2 half][16 CT]
    total = sums + 8 * 16 * CT;
  }
};


template <int DQ, int NW>
__global__ __launch_bounds__(64 * NW) void relattn_bwd_fused_kernel(
    const float* __restrict__ dctx, const float* __restrict__ ctxo, const float* __restrict__ q,
    const float* __restrict__ k, const float* __restrict__ v, const float* __restrict__ pos,
    const float* __restrict__ u, const float* __restrict__ vbias, const int* __restrict__ lens,
    const float* __restrict__ stats, const uint32_t* __restrict__ kbits,
    const float* __restrict__ anchors, int Bp, int T_, int H, int ns, float inv_sqrt_d,
    DropCfg dc, float* __restrict__ dq, float* __restrict__ dk, float* __restrict__ dv,
    size_t kv_split_stride, float* __restrict__ dp_part, float* __restrict__ du_part,
    float* __restrict__ dvb_part) {
  const int T = T_;
  constexpr int D = 4 * DQ;
  constexpr int CT = (D + 15) / 16;
  constexpr int DP = 16 * CT;           // padded columns
  constexpr int KPW = 16 / NW;          // key / position tiles per wave
  constexpr int NTH = 64 * NW;
  constexpr int NJ = 8 * CT;            // dq jobs (which, a, ct, half of the k range)
  constexpr int JPW = (NJ + NW - 1) / NW;
  extern __shared__ float lds[];
  const int nt = (T + 15) >> 4;
  const int Tp = 16 * nt;
  const int W = (nt + 1) >> 1;
  const int nch = (Tp + kFQ - 1) / kFQ;
  const FusedLds off(T, D, CT, nch, W);
  float* kimg = lds + off.kimg;
  float* R = lds + off.reg;
  float* qu_a = lds + off.qu;
  float* qv_a = lds + off.qv;
  float* do_a = lds + off.dO;
  __bf16* planes = reinterpret_cast<__bf16*>(lds + off.planes);
  float* st_s = lds + off.stats;
  float* delta_s = lds + off.delta;
  float* dpart = lds + off.dpart;
  uint32_t* kb_s = reinterpret_cast<uint32_t*>(lds + off.kb);
  float* comb = lds + off.comb;
  float* sums = lds + off.sums;
  constexpr int AP = D + 1;
  // B plane (tensor z: 0 = q+u, 1 = q+v, 2 = dO; part p): [col][query] bf16
  auto plane = [&](int z, int p) { return planes + (size_t)(3 * z + p) * DP * kPlanePitch; };

  // block = (batch row, head, split of the chunks): the ns splits of one (b, h) are
  // consecutive logical ids (one XCD: they read the same k / v / pos rows)
  const int L0 = xcd_logical((int)blockIdx.x, (int)gridDim.x);
  const int sp = L0 % ns, bhl = L0 / ns;
  const int h = bhl % H, b = bhl / H;
  const int bh = b * H + h;
  const int cps = (nch + ns - 1) / ns;  // chunks per split
  const int c0 = sp * cps, c1 = min(nch, c0 + cps);
  const int pass = b / Bp;
  const int C = H * D;
  const int L = min(lens[b], T);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 15, g = lane >> 4;
  const size_t bo = (size_t)b * T * C + h * D;
  const float* qb = q + bo;
  const float* kb = k + bo;
  const float* vb = v + bo;
  const float* dob = dctx + bo;
  const float* cob = ctxo + bo;
  const float* pb = pos + (size_t)pass * T * C + h * D;
  const float* ub = u + h * D;
  const float* vbb = vbias + h * D;
  const __amdgpu_buffer_rsrc_t rs_p = slice_rsrc(pb, T, C, D);
  float* xim = R + T;  // X image: row x (query i0 + x) at pitch T+1, column 0 = 0

  // ---- block setup: k image, statistics, this wave's v / pos rows (B operands, registers)
  for (int e = threadIdx.x; e < Tp * CT * 4; e += NTH) {
    const int row = e / (CT * 4), c4 = 4 * (e - row * (CT * 4));
    f32x4 x4 = f32x4{0.f, 0.f, 0.f, 0.f};
    if (row < T && c4 < D) x4 = *(const f32x4u*)(kb + (size_t)row * C + c4);
    *(f32x4*)(kimg + row * DP + c4) = x4;
  }
  for (int e = threadIdx.x; e < kFQ * nch; e += NTH) {
    const bool in = e < Tp;
    st_s[2 * e] = in ? stats[2 * ((size_t)bh * Tp + e)] : 0.0f;
    st_s[2 * e + 1] = in ? stats[2 * ((size_t)bh * Tp + e) + 1] : 0.0f;
  }
  float vreg[KPW][DQ], preg[KPW][DQ];
#pragma unroll
  for (int i = 0; i < KPW; ++i) {
    const int row = 16 * (w * KPW + i) + r;
    if (row < T) {
      load_run<DQ>(vb + (size_t)row * C + g * DQ, vreg[i]);
      load_run<DQ>(pb + (size_t)row * C + g * DQ, preg[i]);
    } else {
#pragma unroll
      for (int s = 0; s < DQ; ++s) vreg[i][s] = preg[i][s] = 0.0f;
    }
  }
  f32x4 acc_k[KPW][CT], acc_v[KPW][CT], acc_p[KPW][CT];
#pragma unroll
  for (int i = 0; i < KPW; ++i)
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) acc_k[i][ct] = acc_v[i][ct] = acc_p[i][ct] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int e = threadIdx.x; e < 8 * DP; e += NTH) sums[e] = 0.0f;

  // band row 0 of the first chunk: dS' of query i0 - 1, zero or (split > 0) recomputed:
  // X[ip][j], X[ip+1][j], (q+u)[ip].k[j], dO[ip].v[j] in the MFMA's k order (bitwise the
  // values the previous split's tiles hold), dO[ip].ctx[ip] as the staging partials sum it
  if (c0 > 0) {
    const int ip = kFQ * c0 - 1, j = threadIdx.x;
    if (j < T) {
      const float* qr = qb + (size_t)ip * C;
      const float* qn = qb + (size_t)(ip + 1) * C;
      const float* dr = dob + (size_t)ip * C;
      const float* cr = cob + (size_t)ip * C;
      float prow[D];
      load_run<D>(pb + (size_t)j * C, prow);
      float xs = 0.0f, xn = 0.0f, as = 0.0f, ds = 0.0f, dl = 0.0f;
#pragma unroll
      for (int s2 = 0; s2 < DQ; ++s2)
#pragma unroll
        for (int gg = 0; gg < 4; ++gg) {
          const int cc = gg * DQ + s2;
          xs = fmaf(qr[cc] + vbb[cc], prow[cc], xs);
          xn = fmaf(qn[cc] + vbb[cc], prow[cc], xn);
          as = fmaf(qr[cc] + ub[cc], kimg[j * DP + cc], as);
          ds = fmaf(dr[cc], vb[(size_t)j * C + cc], ds);
        }
#pragma unroll
      for (int c4i = 0; c4i < DQ; ++c4i) {
        float a4 = 0.0f;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) a4 = fmaf(dr[4 * c4i + jj], cr[4 * c4i + jj], a4);
        dl += a4;
      }
      comb[j] = xs;
      comb[T + j] = xn;
      comb[2 * T + j] = as;
      comb[3 * T + j] = ds;
      if (j == 0) comb[4 * T] = dl;
    }
    __syncthreads();
    if (j < T) {
      // bd[ip][j] = X.flat[T + ip*T + j]: X[ip][T-1-ip+j] (j <= ip), 0 (j = ip+1),
      // X[ip+1][j-ip-2] (j >= ip+2)
      const float bd = j <= ip ? comb[T - 1 - ip + j] : (j == ip + 1 ? 0.0f : comb[T + j - ip - 2]);
      float sc = (comb[2 * T + j] + bd) * inv_sqrt_d;
      sc = j < (ip < L ? L : 0) ? sc : -INFINITY;
      const float p = __expf(sc - st_s[2 * ip]) * st_s[2 * ip + 1];
      float ks = 1.0f;
      if (dc.on)
        ks = (kbits[((size_t)bh * Tp + ip) * W + (j >> 5)] >> (j & 31)) & 1u ? dc.scale : 0.0f;
      R[j] = (p * (comb[3 * T + j] * ks - comb[4 * T])) * inv_sqrt_d;
    }
  } else {
    for (int e = threadIdx.x; e < T; e += NTH) R[e] = 0.0f;
  }

  OB_STAMP_DECL(1)
  for (int c = c0; c < c1; ++c) {
    const int i0 = kFQ * c;
    // LDS addresses derived from T are recomputed per chunk (a few VALU ops) instead of
    // being hoisted out of the loop and spilled under the register pressure
    int T = T_;
    asm volatile("" : "+s"(T));
    OB_STAMP(0);
    __syncthreads();  // the previous chunk's band / image / plane / comb reads are done
    OB_STAMP(1);
    // ---- phase 0a: the previous chunk's dq; this chunk's rows, dO.ctx partials, X row 32
    if (c > c0) {
      const int ip = i0 - kFQ;
      for (int e = threadIdx.x; e < kFQ * D; e += NTH) {
        const int x = e / D, col = e - x * D;
        const int a = x >> 4, xr = x & 15, ct = col >> 4, cr = col & 15;
        if (ip + x < T) {
          // dq = (dS' k) + (dX pos), each the sum of its two k-range halves
          const int ci = ((a * CT + ct) * 2 * 16 + xr) * 16 + cr;
          const int cv = 2 * CT * 2 * 256;
          dq[bo + (size_t)(ip + x) * C + col] =
              (comb[ci] + comb[ci + 256]) + (comb[cv + ci] + comb[cv + ci + 256]);
        }
      }
    }
    for (int e = threadIdx.x; e < T; e += NTH) {
      // band row 0: dS' of query i0 - 1 (the first chunk of a split: zero, or recomputed
      // by the prologue when that row belongs to the previous split)
      if (c > c0) R[e] = R[32 * T + e];
      // X row 32 (query i0 + 32), saved by the forward (bitwise the MFMA row)
      xim[kFQ * (T + 1) + 1 + e] = i0 + kFQ < T ? anchors[((size_t)bh * nch + c) * T + e] : 0.0f;
    }
    {
      constexpr int nq = kFQ * DQ;  // float4s of 32 rows
      for (int e = threadIdx.x; e < 2 * nq; e += NTH) {
        // [0, nq): q rows (+u and +v); [nq, 2nq): dO rows, and dO.ctx over the float4
        const int kind = e < nq ? 0 : 1;
        const int rem = e - kind * nq;
        const int x = rem / DQ, c4i = rem - x * DQ, c4 = 4 * c4i;
        const int qi = i0 + x;
        f32x4 v4 = f32x4{0.f, 0.f, 0.f, 0.f}, c4v = f32x4{0.f, 0.f, 0.f, 0.f};
        if (qi < T) {
          v4 = *(const f32x4u*)((kind == 1 ? dob : qb) + (size_t)qi * C + c4);
          if (kind == 1) c4v = *(const f32x4u*)(cob + (size_t)qi * C + c4);
        }
        if (kind == 1) {
#pragma unroll
          for (int j = 0; j < 4; ++j) do_a[x * AP + c4 + j] = v4[j];
          float a = 0.0f;
#pragma unroll
          for (int j = 0; j < 4; ++j) a = fmaf(v4[j], c4v[j], a);
          dpart[x * DQ + c4i] = a;
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            qu_a[x * AP + c4 + j] = qi < T ? v4[j] + ub[c4 + j] : 0.0f;
            qv_a[x * AP + c4 + j] = qi < T ? v4[j] + vbb[c4 + j] : 0.0f;
          }
        }
      }
    }
    if (dc.on)
      for (int e = threadIdx.x; e < kFQ * W; e += NTH) {
        const int x = e / W;
        kb_s[e] = i0 + x < Tp ? kbits[((size_t)bh * Tp + i0) * W + e] : 0u;
      }
    OB_STAMP(2);
    __syncthreads();
    OB_STAMP(3);
    // ---- phase 0b: delta, B planes (split once); phase 1: X tiles
    if (threadIdx.x < kFQ) {
      float a = 0.0f;
#pragma unroll
      for (int cc = 0; cc < DQ; ++cc) a += dpart[threadIdx.x * DQ + cc];
      delta_s[threadIdx.x] = a;
    }
    for (int e = threadIdx.x; e < 3 * DP * (kFQ / 4); e += NTH) {
      const int z = e / (DP * (kFQ / 4));
      const int rem = e - z * DP * (kFQ / 4);
      const int col = rem / (kFQ / 4), x0 = 4 * (rem - col * (kFQ / 4));
      const float* src = z == 0 ? qu_a : (z == 1 ? qv_a : do_a);
      bf16x4_t hp, mp, lp;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float x = col < D ? src[(x0 + j) * AP + col] : 0.0f;
        __bf16 hh, mm, ll;
        split3(x, hh, mm, ll);
        hp[j] = hh;
        mp[j] = mm;
        lp[j] = ll;
      }
      *(bf16x4_t*)(plane(z, 0) + col * kPlanePitch + x0) = hp;
      *(bf16x4_t*)(plane(z, 1) + col * kPlanePitch + x0) = mp;
      *(bf16x4_t*)(plane(z, 2) + col * kPlanePitch + x0) = lp;
    }
    {
      // X[query][pos] = (q+v) pos^T, the KPW x 2 tiles as independent chains
      f32x4 xa[KPW][2];
#pragma unroll
      for (int i = 0; i < KPW; ++i) xa[i][0] = xa[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < DQ; ++s) {
        const float a0 = qv_a[r * AP + g * DQ + s], a1 = qv_a[(16 + r) * AP + g * DQ + s];
#pragma unroll
        for (int i = 0; i < KPW; ++i) {
          xa[i][0] = mfma4(a0, preg[i][s], xa[i][0]);
          xa[i][1] = mfma4(a1, preg[i][s], xa[i][1]);
        }
      }
#pragma unroll
      for (int i = 0; i < KPW; ++i) {
        const int m = 16 * (w * KPW + i) + r;
        if (m < T)
#pragma unroll
          for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int e = 0; e < 4; ++e) xim[(16 * a + 4 * g + e) * (T + 1) + 1 + m] = xa[i][a][e];
      }
    }
    if (threadIdx.x <= kFQ) xim[threadIdx.x * (T + 1)] = 0.0f;
    OB_STAMP(4);
    __syncthreads();
    OB_STAMP(5);
    // ---- phase 2: S, P, dP, dS' for this wave's key tiles; key-side products
    float dsv[KPW][8];
    {
      f32x4 sa[KPW][2], sd[KPW][2];
#pragma unroll
      for (int i = 0; i < KPW; ++i)
        sa[i][0] = sa[i][1] = sd[i][0] = sd[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < DQ; ++s) {
        const float u0 = qu_a[r * AP + g * DQ + s], u1 = qu_a[(16 + r) * AP + g * DQ + s];
        const float o0 = do_a[r * AP + g * DQ + s], o1 = do_a[(16 + r) * AP + g * DQ + s];
#pragma unroll
        for (int i = 0; i < KPW; ++i) {
          const float kv = kimg[(16 * (w * KPW + i) + r) * DP + g * DQ + s];
          sa[i][0] = mfma4(u0, kv, sa[i][0]);
          sa[i][1] = mfma4(u1, kv, sa[i][1]);
          sd[i][0] = mfma4(o0, vreg[i][s], sd[i][0]);
          sd[i][1] = mfma4(o1, vreg[i][s], sd[i][1]);
        }
      }
#pragma unroll
      for (int i = 0; i < KPW; ++i) {
        const int kt = w * KPW + i;
        const int key = 16 * kt + r;
        const float tile_live = kt < nt ? 1.0f : 0.0f;
        float pdv[8];
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) {
          const int a = jj >> 2, e = jj & 3;
          const int x = 16 * a + 4 * g + e, qi = i0 + x;
          const int Lq = qi < L ? L : 0;
          // bd[qi][key] = X.flat[T + qi*T + key] of the padded image (rel_shift, :97-103)
          float sc = (sa[i][a][e] + xim[T + x * T + key - i0]) * inv_sqrt_d;
          sc = key < Lq ? sc : -INFINITY;
          const float p = __expf(sc - st_s[2 * (i0 + x)]) * st_s[2 * (i0 + x) + 1];
          // (keep words are unstaged and unused without dropout)
          const uint32_t kw = kb_s[x * W + (key >> 5)];
          const float ks = dc.on ? ((kw >> (key & 31)) & 1u ? dc.scale : 0.0f) : 1.0f;
          dsv[i][jj] = tile_live * ((p * (sd[i][a][e] * ks - delta_s[x])) * inv_sqrt_d);
          pdv[jj] = tile_live * (dc.on ? p * ks : p);
        }
        // dK += dS'^T (q+u), dV += Pd^T dO: A = this lane's 8 queries of key r (k order
        // 4g..4g+3, 16+4g..16+4g+3), B = the planes read in the same order
        if (kt < nt) {
          key_side<CT>(dsv[i], plane(0, 0), g, r, acc_k[i]);
          key_side<CT>(pdv, plane(2, 0), g, r, acc_v[i]);
        }
      }
    }
    OB_STAMP(6);
    __syncthreads();  // every X-image read is done: the band may overwrite it
    OB_STAMP(7);
#pragma unroll
    for (int i = 0; i < KPW; ++i) {
      const int key = 16 * (w * KPW + i) + r;
      if (key < T)
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) {
          const int x = 16 * (jj >> 2) + 4 * g + (jj & 3);
          R[(x + 1) * T + key] = dsv[i][jj];
        }
    }
    OB_STAMP(8);
    __syncthreads();
    OB_STAMP(9);
    // ---- phase 3: dpos (bf16x6, own position tiles) and the dq jobs (fp32)
#pragma unroll
    for (int i = 0; i < KPW; ++i) {
      const int pt = w * KPW + i;
      if (pt >= nt) continue;
      const int m = 16 * pt + r;
      float xv[8];
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        const int x = 8 * g + jj;  // dX[i0 + x][m] = dS'.flat[(i0+x)(T+1) + m + 1 - T]
        xv[jj] = i0 + x < T ? R[x * (T + 1) + i0 + m + 1] : 0.0f;
      }
      bf16x8_t ax[3];
      split8(xv, ax);
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        bf16x8_t bq[3];
#pragma unroll
        for (int pp = 0; pp < 3; ++pp)
          bq[pp] = *(const bf16x8_t*)(plane(1, pp) + (16 * ct + r) * kPlanePitch + 8 * g);
        acc_p[i][ct] = mfma_x6(ax, bq, acc_p[i][ct]);
      }
    }
    const int nk = 4 * nt;            // k steps of 4 keys / positions
    const int nk_h = 4 * ((nk + 7) / 8);  // first half: a multiple of 4 steps
#pragma unroll 1
    for (int jj = 0; jj < JPW; ++jj) {
      const int j = w + NW * jj;
      if (j >= NJ) continue;
      const int which = j / (4 * CT), a = (j / (2 * CT)) & 1, ct = (j >> 1) % CT, half = j & 1;
      const int x = 16 * a + r;
      const int sb = half ? nk_h : 0, se = half ? nk : nk_h;
      f32x4 ac4[4];
      if (which == 0)  // dS' k: A = band row x, B = k rows of the image (zero past T)
        dq_job<0, DP>(R + (x + 1) * T + g, 1.0f, kimg + g * DP + 16 * ct + r, rs_p, 0, C, sb, se,
                      ac4);
      else  // dX pos: A = the band read flat (0 for rows past T), B = pos rows (range check)
        dq_job<1, DP>(R + x * (T + 1) + i0 + 1 + g, i0 + x < T ? 1.0f : 0.0f, nullptr, rs_p,
                      (g * C + 16 * ct + r) * 4, C, sb, se, ac4);
      float cs = 0.0f;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float vsum = (ac4[0][e] + ac4[1][e]) + (ac4[2][e] + ac4[3][e]);
        comb[((((which * 2 + a) * CT + ct) * 2 + half) * 16 + 4 * g + e) * 16 + r] = vsum;
        cs += vsum;
      }
      // the job's column sums (du / dvb), accumulated over the chunks in its own LDS slot
      cs = xsum_1632(cs);
      if (g == 0) sums[((which * 2 + a) * 2 + half) * DP + 16 * ct + r] += cs;
    }
  }
  __syncthreads();
  // ---- the last chunk's dq; dk, dv, the per-row dpos partial; du / dvb column sums
  {
    const int ip = kFQ * (c1 - 1);
    for (int e = threadIdx.x; e < kFQ * D; e += NTH) {
      const int x = e / D, col = e - x * D;
      const int a = x >> 4, xr = x & 15, ct = col >> 4, cr = col & 15;
      if (ip + x < T) {
        // dq = (dS' k) + (dX pos), each the sum of its two k-range halves
        const int ci = ((a * CT + ct) * 2 * 16 + xr) * 16 + cr;
        const int cv = 2 * CT * 2 * 256;
        dq[bo + (size_t)(ip + x) * C + col] =
            (comb[ci] + comb[ci + 256]) + (comb[cv + ci] + comb[cv + ci + 256]);
      }
    }
  }
  float* dkb = dk + sp * kv_split_stride + bo;
  float* dvbp = dv + sp * kv_split_stride + bo;
  float* dpb = dp_part + ((size_t)bh * ns + sp) * T * D;
#pragma unroll
  for (int i = 0; i < KPW; ++i) {
    const int t16 = 16 * (w * KPW + i);
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      const int col = 16 * ct + r;
      if (col >= D) continue;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = t16 + 4 * g + e;
        if (row >= T) continue;
        dkb[(size_t)row * C + col] = acc_k[i][ct][e];
        dvbp[(size_t)row * C + col] = acc_v[i][ct][e];
        dpb[(size_t)row * D + col] = acc_p[i][ct][e];
      }
    }
  }
  __syncthreads();
  if (threadIdx.x < D) {
    const int col = threadIdx.x;
    const float* su = sums + col;
    du_part[((size_t)bh * ns + sp) * D + col] = (su[0] + su[DP]) + (su[2 * DP] + su[3 * DP]);
    dvb_part[((size_t)bh * ns + sp) * D + col] = (su[4 * DP] + su[5 * DP]) + (su[6 * DP] + su[7 * DP]);
  }
  OB_STAMP_WRITE(NW)
}

// du, dvb [H][D]: sum over (batch row, query tile) of the per-tile partials. Block = one
// (which, head) x 4 columns x 64 slices (slice s: pairs s, s+64, ..., four accumulators),
// the slices added in order through LDS (fixed order). 2*H*ceil(D/4) blocks: each thread
// has a few independent loads in flight (one block per (which, head) with a serial chain of
// 24 partials per thread measured 15 us at Conformer-S).
constexpr int kBiasCols = 4, kBiasSlices = kThreads / kBiasCols;

__device__ __forceinline__ void relattn_bias_reduce_block(
    int bid, const float* __restrict__ du_part, const float* __restrict__ dvb_part, int Bt, int H,
    int D, int nqt, float* __restrict__ du, float* __restrict__ dvb) {
  __shared__ float red[kBiasSlices][kBiasCols];
  const int ncg = (D + kBiasCols - 1) / kBiasCols;
  const int cg = bid % ncg, wh = bid / ncg;
  const int which = wh / H, h = wh - which * H;
  const int cl = threadIdx.x % kBiasCols, sl = threadIdx.x / kBiasCols;
  const int c = cg * kBiasCols + cl;
  const float* src = which == 0 ? du_part : dvb_part;
  const int pairs = Bt * nqt;
  float a[4] = {0.f, 0.f, 0.f, 0.f};
  if (c < D) {
    int uu = 0;
    for (int qq = sl; qq < pairs; qq += kBiasSlices, ++uu) {
      const int b = qq / nqt, qt = qq - b * nqt;
      a[uu & 3] += src[(((size_t)b * H + h) * nqt + qt) * D + c];
    }
  }
  red[sl][cl] = (a[0] + a[1]) + (a[2] + a[3]);
  __syncthreads();
  if (sl == 0 && c < D) {
    float t = 0.0f;
#pragma unroll 8
    for (int qq = 0; qq < kBiasSlices; ++qq) t += red[qq][cl];
    (which == 0 ? du : dvb)[h * D + c] = t;
  }
}

// dpos [P][T][H*D]: sum over the pass's Bp batch rows. Block = 64 consecutive output
// elements x 4 batch slices (slice s: rows s, s+4, ... of the pass); the slices are added
// in slice order through LDS (fixed order: deterministic).
__device__ __forceinline__ void relattn_dpos_reduce_block(
    int bid, const float* __restrict__ dp_part, int Bt, int P, int T, int H, int D, int ns,
    float* __restrict__ dpos) {
  __shared__ float red[4][64];
  const int C = H * D;
  const int64_t n_p = (int64_t)P * T * C;
  const int el = threadIdx.x & 63, sl = threadIdx.x >> 6;
  const int64_t f = (int64_t)bid * 64 + el;
  const int Bp = Bt / P;
  float s = 0.0f;
  if (f < n_p) {
    const int p = (int)(f / ((int64_t)T * C));
    const int rem = (int)(f - (int64_t)p * T * C);
    const int t = rem / C, hc = rem - t * C, h = hc / D, c = hc - h * D;
    float a[4] = {0.f, 0.f, 0.f, 0.f};
    int uu = 0;
    for (int b = p * Bp + sl; b < (p + 1) * Bp; b += 4)
      for (int sp = 0; sp < ns; ++sp, ++uu)  // (ns query splits per batch row)
        a[uu & 3] += dp_part[((((size_t)b * H + h) * ns + sp) * T + t) * D + c];
    s = (a[0] + a[1]) + (a[2] + a[3]);
  }
  red[sl][el] = s;
  __syncthreads();
  if (sl == 0 && f < n_p) dpos[f] = ((red[0][el] + red[1][el]) + red[2][el]) + red[3][el];
}

// Both reductions of the backward in one launch (they read different partials and write
// different outputs): blocks [0, n_dpos) reduce dpos, the rest du / dvb -- one launch per
// attention layer fewer at the per-launch floor, the same arithmetic per output.
// (and, for the flash-style backward with ns > 1 query splits, dk / dv as the fixed-order
// sum of the splits' partials: [ns][n] each, 4 elements per thread)
__global__ __launch_bounds__(kThreads) void relattn_reduce_kernel(
    const float* __restrict__ dp_part, const float* __restrict__ du_part,
    const float* __restrict__ dvb_part, int Bt, int P, int T, int H, int D, int nqt, int n_dpos,
    float* __restrict__ dpos, float* __restrict__ du, float* __restrict__ dvb, int ns_dpos,
    int n_bias, const float* __restrict__ kv_part, int64_t n_kv, float* __restrict__ dk,
    float* __restrict__ dv) {
  const int bid = (int)blockIdx.x;
  if (bid < n_dpos) {
    relattn_dpos_reduce_block(bid, dp_part, Bt, P, T, H, D, ns_dpos, dpos);
  } else if (bid < n_dpos + n_bias) {
    relattn_bias_reduce_block(bid - n_dpos, du_part, dvb_part, Bt, H, D, nqt, du, dvb);
  } else {
    const int64_t e = 4 * ((int64_t)(bid - n_dpos - n_bias) * kThreads + threadIdx.x);
    if (e >= 2 * n_kv) return;
    const bool isv = e >= n_kv;
    const int64_t i = isv ? e - n_kv : e;  // n_kv % 4 == 0
    const float* src = kv_part + (isv ? (int64_t)nqt * n_kv : 0) + i;
    f32x4 acc = *(const f32x4*)src;
    for (int sp = 1; sp < nqt; ++sp) acc += *(const f32x4*)(src + sp * n_kv);
    *(f32x4*)((isv ? dv : dk) + i) = acc;
  }
}

// keep mask of n elements in rows of T (element e = row * T + j): the attention kernels'
// index (row * Te + j); with T = n it is the flat index of the BitLinear / LayerNorm sites
__global__ __launch_bounds__(kThreads) void relattn_mask_kernel(int64_t n, int64_t T, DropCfg dc,
                                                                const uint64_t* __restrict__ rng,
                                                                uint64_t rng_off,
                                                                uint8_t* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (e >= n) return;
  const int64_t row = e / T, j = e - row * T;
  const uint64_t idx = (uint64_t)row * (uint64_t)(T + (T & 1)) + (uint64_t)j;
  out[e] = (!dc.on || drop_keep(drop_key(rng[0], rng[1] + rng_off), idx, dc.thresh)) ? 1 : 0;
}

size_t fwd_lds_bytes(int T, int D) {
  const size_t img = sizeof(float) * (size_t)(kTile + 1) * (T + 1);
  // v^T parts: 3 x [16 CT cols][min(32 ceil(nt/2), kFwdKeyChunk) keys + 8] bf16
  const size_t nt = (T + 15) / 16;
  const size_t kp = std::min<size_t>(32 * ((nt + 1) / 2), kFwdKeyChunk);
  const size_t vst = sizeof(uint16_t) * 3 * (size_t)(16 * ((D + 15) / 16)) * (kp + 8);
  return img > vst ? img : vst;
}
size_t bwd_lds_bytes(int T) { return sizeof(float) * ((size_t)(kTile + 1) * T + 128); }

}  // namespace

bool relattn_supported(int64_t T, int64_t d) {
  return T >= 1 && T <= 512 && (d == 16 || d == 32 || d == 36 || d == 64);
}

// the flash-style backward (relattn_bwd_fused_kernel): T <= 256 (16 key tiles), d <= 36, when
// selected (OB_ATTN_BWD=flash). It keeps every [T][T] quantity on chip but is slower than the
// probability path at Conformer-S (measured 400 vs 253 us per call: one fat block per (b, h)
// split in two, latency-bound chunk phases at 2 waves per SIMD; DESIGN.md "Attention"), so the
// probability path stays the default. The mode is process-wide: OB_ATTN_BWD read once (the
// first query), then only ob_relattn_set_bwd_mode changes it. The saved buffer's layout, the
// backward's work space and the backward kernel all follow it; ob_relattn_bwd checks the
// caller's saved size against the layout of the current mode, so a backward never reads a
// buffer the forward laid out under the other mode.
static std::atomic<int> g_flash{-1};
static bool flash_selected() {
  int m = g_flash.load(std::memory_order_relaxed);
  if (m < 0) {
    const char* e = getenv("OB_ATTN_BWD");
    int want = (e != nullptr && e[0] == 'f') ? 1 : 0;
    g_flash.compare_exchange_strong(m, want);
    m = g_flash.load(std::memory_order_relaxed);
  }
  return m == 1;
}
int relattn_set_flash(int on) {
  const int prev = flash_selected() ? 1 : 0;
  if (on == 0 || on == 1) g_flash.store(on, std::memory_order_relaxed);
  return prev;
}
bool relattn_fused(int64_t T, int64_t d) { return T <= 256 && d <= 36 && flash_selected(); }

// saved state of the forward for the backward (fp32 elements): row statistics
// [Bt*H][Tp][2] (max, 1/sum) | keep bits [Bt*H][Tp][W] | then either (flash-style backward)
// the X rows below each 32-query chunk [Bt*H][nch][T] or (T > 256 or d = 64) probability tiles
struct SavedLayout {
  int64_t stats, kbits, tail, total;
  SavedLayout(int64_t Bt, int64_t T, int64_t H, int64_t d) {
    const int64_t nt = (T + 15) / 16, Tp = 16 * nt, W = (nt + 1) / 2, nch = (Tp + 31) / 32;
    stats = 0;
    kbits = Bt * H * Tp * 2;
    tail = kbits + Bt * H * Tp * W;
    tail = (tail + 3) & ~(int64_t)3;  // 16-B aligned
    total = tail + (relattn_fused(T, d) ? Bt * H * nch * T : relattn_probs_elems(Bt, T, H));
  }
};

int64_t relattn_saved_elems(int64_t Bt, int64_t T, int64_t H, int64_t d) {
  return SavedLayout(Bt, T, H, d).total;
}

int64_t relattn_probs_elems(int64_t Bt, int64_t T, int64_t H) {
  const int64_t nt = (T + 15) / 16;
  return Bt * H * nt * nt * 256;
}

// query splits of the flash-style backward: two blocks per (batch row, head) once there are
// two chunks, so Bt*H*2 blocks fill whole rounds of one block per CU (Conformer-S: 768 = 3 x
// 256) instead of 1.5 rounds; the key-side partials are summed by the reduce launch
int fused_splits(int64_t T) { return ((16 * ((T + 15) / 16) + 31) / 32) >= 2 ? 2 : 1; }

// ws: [probability path: dS' [Bt][H][T][T]] | dpos per batch row [Bt][H][ns][T][d] | du, dvb
// partials per (batch row, head, query tile / split) | (ns > 1) dk, dv split partials.
size_t relattn_bwd_workspace(int64_t Bt, int64_t T, int64_t H, int64_t d) {
  if (relattn_fused(T, d)) {
    const int64_t ns = fused_splits(T);
    const int64_t kv = ns > 1 ? 2 * ns * Bt * T * H * d + 4 : 0;
    return sizeof(float) * (size_t)(Bt * H * ns * T * d + 2 * Bt * H * ns * d + kv + 64);
  }
  const int64_t nqt = (T + kTile - 1) / kTile;
  return sizeof(float) * (size_t)(Bt * H * T * T + Bt * H * T * d + 2 * Bt * H * nqt * d + 64);
}

#define OB_RA_DISPATCH(KERNEL)                 \
  do {                                         \
    const bool big = T > 256;                  \
    if (d == 16) {                             \
      if (big) KERNEL(4, 32); else KERNEL(4, 16);   \
    } else if (d == 32) {                      \
      if (big) KERNEL(8, 32); else KERNEL(8, 16);   \
    } else if (d == 36) {                      \
      if (big) KERNEL(9, 32); else KERNEL(9, 16);   \
    } else {                                   \
      if (big) KERNEL(16, 32); else KERNEL(16, 16); \
    }                                          \
  } while (0)

void launch_relattn_fwd(const float* q, const float* k, const float* v, const float* pos,
                        const float* u, const float* vb, const int* lens, int64_t Bt, int64_t P,
                        int64_t T, int64_t H, int64_t d, float p_drop, const uint64_t* rng,
                        uint64_t rng_off, float* saved, float* probs, float* ctx, hipStream_t s) {
  const dim3 grid((unsigned)(((T + kTile - 1) / kTile) * H * Bt));
  const DropCfg dc = make_drop(p_drop);
  const float inv_sqrt_d = 1.0f / (float)sqrt((double)d);  // torch: tensor / scalar = * (1/scalar)
  const size_t lds = fwd_lds_bytes((int)T, (int)d);
  const SavedLayout sl(Bt, T, H, d);
  const bool flash = saved && relattn_fused(T, d);  // else the probabilities are saved
  float* stats = flash ? saved : nullptr;
  uint32_t* kbits = flash ? reinterpret_cast<uint32_t*>(saved + sl.kbits) : nullptr;
  float* anchors = flash ? saved + sl.tail : nullptr;
  // the probability path's backward reads the tiles from the saved state
  if (saved && !relattn_fused(T, d)) probs = saved + sl.tail;
#define OB_RA_FWD(DQ, NTT)                                                                 \
  hipLaunchKernelGGL((relattn_fwd_kernel<DQ, NTT>), grid, dim3(kThreads), lds, s, q, k, v, pos, \
                     u, vb, lens, (int)(Bt / P), (int)T, (int)H, inv_sqrt_d, dc, rng, rng_off, probs, \
                     stats, kbits, anchors, ctx)
  OB_RA_DISPATCH(OB_RA_FWD);
#undef OB_RA_FWD
}

constexpr int kFusedWaves = 8;

void launch_relattn_bwd(const float* dctx, const float* ctx, const float* q, const float* k,
                        const float* v, const float* pos, const float* u, const float* vb,
                        const int* lens, int64_t Bt, int64_t P, int64_t T, int64_t H, int64_t d,
                        float p_drop, const float* saved, float* dq, float* dk, float* dv,
                        float* dpos, float* du, float* dvb, void* ws, hipStream_t s) {
  const int64_t nt = (T + 15) / 16, Tp = 16 * nt, W = (nt + 1) / 2;
  if (relattn_fused(T, d)) {
    const DropCfg dc = make_drop(p_drop);
    const float inv_sqrt_d = 1.0f / (float)sqrt((double)d);
    const int ns = fused_splits(T);
    const int64_t C = H * d;
    const int64_t n_kv = Bt * T * C;
    float* dp_part = (float*)ws;
    float* du_part = dp_part + (size_t)Bt * H * ns * T * d;
    float* dvb_part = du_part + (size_t)Bt * H * ns * d;
    float* kv_part = dvb_part + (size_t)Bt * H * ns * d;
    kv_part += (16 - ((uintptr_t)kv_part & 15)) / 4 % 4;  // 16-B aligned
    const SavedLayout sl(Bt, T, H, d);
    const float* stats = saved;
    const uint32_t* kbits = reinterpret_cast<const uint32_t*>(saved + sl.kbits);
    const float* anchors = saved + sl.tail;
    const int CT = (int)((d + 15) / 16);
    const size_t lds = sizeof(float) * FusedLds((int)T, (int)d, CT, (int)((Tp + kFQ - 1) / kFQ), (int)W).total;
    // ns == 1: the key-side results go straight to dk / dv
    float* dk_out = ns > 1 ? kv_part : dk;
    float* dv_out = ns > 1 ? kv_part + ns * n_kv : dv;
#define OB_RA_FUSED(DQ)                                                                           \
  hipLaunchKernelGGL((relattn_bwd_fused_kernel<DQ, kFusedWaves>), dim3((unsigned)(Bt * H * ns)),   \
                     dim3(64 * kFusedWaves), lds, s, dctx, ctx, q, k, v, pos, u, vb, lens, stats,   \
                     kbits, anchors, (int)(Bt / P), (int)T, (int)H, ns, inv_sqrt_d, dc, dq, dk_out, \
                     dv_out, (size_t)n_kv, dp_part, du_part, dvb_part)
    if (d == 16) OB_RA_FUSED(4);
    else if (d == 32) OB_RA_FUSED(8);
    else OB_RA_FUSED(9);
#undef OB_RA_FUSED
    const int n_dpos = (int)ceil_div(P * T * C, 64);
    const int n_bias = (int)(2 * H * ((d + kBiasCols - 1) / kBiasCols));
    const int n_kvb = ns > 1 ? (int)ceil_div(2 * n_kv, 4 * kThreads) : 0;
    hipLaunchKernelGGL(relattn_reduce_kernel, dim3((unsigned)(n_dpos + n_bias + n_kvb)),
                       dim3(kThreads), 0, s, (const float*)dp_part, (const float*)du_part,
                       (const float*)dvb_part, (int)Bt, (int)P, (int)T, (int)H, (int)d, ns, n_dpos,
                       dpos, du, dvb, ns, n_bias, (const float*)kv_part, n_kv, dk, dv);
    return;
  }
  const float* probs = saved + SavedLayout(Bt, T, H, d).tail;
  const int nqt = (int)((T + kTile - 1) / kTile);
  const dim3 grid((unsigned)(nqt * H * Bt));
  const DropCfg dc = make_drop(p_drop);
  const float inv_sqrt_d = 1.0f / (float)sqrt((double)d);  // torch: tensor / scalar = * (1/scalar)
  const size_t lds = bwd_lds_bytes((int)T);
  float* dsg = (float*)ws;
  float* dp_part = dsg + (size_t)Bt * H * T * T;
  float* du_part = dp_part + (size_t)Bt * H * T * d;
  float* dvb_part = du_part + (size_t)Bt * H * nqt * d;
#define OB_RA_BWD(DQ, NTT)                                                                     \
  hipLaunchKernelGGL((relattn_bwd_kernel<DQ, NTT>), grid, dim3(kThreads), lds, s, dctx, ctx, k,    \
                     v, pos, (int)(Bt / P), (int)T, (int)H, inv_sqrt_d, dc, probs, dq, dsg,        \
                     du_part, dvb_part)
  OB_RA_DISPATCH(OB_RA_BWD);
#undef OB_RA_BWD
#define OB_RA_KV(DQ, NTT)                                                                          \
  hipLaunchKernelGGL((relattn_bwd_kv_kernel<DQ>), grid, dim3(kThreads), 0, s, (const float*)dsg,    \
                     probs, q, dctx, u, vb, (int)T, (int)H, dc, dk, dv, dp_part)
  OB_RA_DISPATCH(OB_RA_KV);
#undef OB_RA_KV
  const int64_t C = H * d;
  const int n_dpos = (int)ceil_div(P * T * C, 64);
  const int n_bias = (int)(2 * H * ((d + kBiasCols - 1) / kBiasCols));
  hipLaunchKernelGGL(relattn_reduce_kernel, dim3((unsigned)(n_dpos + n_bias)), dim3(kThreads), 0, s,
                     (const float*)dp_part, (const float*)du_part, (const float*)dvb_part, (int)Bt,
                     (int)P, (int)T, (int)H, (int)d, nqt, n_dpos, dpos, du, dvb, 1, n_bias,
                     (const float*)nullptr, (int64_t)0, (float*)nullptr, (float*)nullptr);
}

#ifdef OB_ATTN_STAMPS
extern "C" int ob_attn_stamps(void* host_dst) {  // diagnostic build only
  return hipMemcpyFromSymbol(host_dst, HIP_SYMBOL(g_attn_stamps), sizeof(g_attn_stamps)) == hipSuccess ? 0 : -6;
}
extern "C" int ob_attn_rt(void* host_dst) {  // diagnostic build only
  return hipMemcpyFromSymbol(host_dst, HIP_SYMBOL(g_attn_rt), sizeof(g_attn_rt)) == hipSuccess ? 0 : -6;
}
#endif

void launch_relattn_dropout_mask(int64_t n, int64_t T, float p_drop, const uint64_t* rng,
                                 uint64_t rng_off, uint8_t* out, hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL(relattn_mask_kernel, dim3((unsigned)((n + kThreads - 1) / kThreads)),
                     dim3(kThreads), 0, s, n, T, make_drop(p_drop), rng, rng_off, out);
}

}  // namespace ob
