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
// per-query-tile partials), plus two small fixed-order reductions (du/dvb over tiles,
// dpos over the pass's batch rows).
//
// rel_shift as a gather: with X = (q + v) p^T,
//   bd[i][j] = X[i][T-1-i+j]   (j <= i);   0   (j == i+1);   X[i+1][j-i-2]   (j >= i+2)
// and its adjoint: dX[i][m] = dbd[i][m-T+1+i] (m >= T-1-i), else dbd[i-1][m+i+1] (i >= 1).
//
// Layout: q, k, v, ctx, dq, dk, dv [Bt][T][H*d]; pos, dpos [P][T][H*d] (batch row b uses
// pass b / (Bt/P)); u, vb, du, dvb [H][d]; probs [Bt][H][T][T]; lens int32 [Bt].
// Products on v_mfma_f32_16x16x4_f32 (exact fp32 fma chain, like torch's fp32 matmul).
// Dropout keeps (i, j) when hash(key(seed, counter + offset), index) >= p * 2^32 (a
// counter hash; torch's own RNG stream is not reproduced). The forward stores each kept
// probability as P and each dropped one as -P (P >= 0, so the sign bit is free): both
// backward kernels read the keep bit back with the probability instead of hashing the
// T x T matrix again (16 us per key-side call at Conformer-S).
#include <math.h>

#include "ob_drop.h"
#include "ob_launch.h"

// Profiling switches (tools/variant.sh builds; all 0 in the product): drop one phase of
// the forward to price it. Results are wrong with any of them set.
#ifndef RA_EXP_NOX
#define RA_EXP_NOX 0
#endif
#ifndef RA_EXP_NOAC
#define RA_EXP_NOAC 0
#endif
#ifndef RA_EXP_NOCTX
#define RA_EXP_NOCTX 0
#endif
#ifndef RA_EXP_NOPROBS
#define RA_EXP_NOPROBS 0
#endif
#ifndef RA_EXP_NODROP
#define RA_EXP_NODROP 0
#endif
#ifndef RB_EXP_NODP
#define RB_EXP_NODP 0
#endif
#ifndef RB_EXP_NODQU
#define RB_EXP_NODQU 0
#endif
#ifndef RB_EXP_NODQV
#define RB_EXP_NODQV 0
#endif
#ifndef RB_EXP_NODSG
#define RB_EXP_NODSG 0
#endif
#ifndef RB_EXP_NOPROBS
#define RB_EXP_NOPROBS 0
#endif
#ifndef RA_EXP_NOROW64
#define RA_EXP_NOROW64 0
#endif
#ifndef RB_EXP_NOROW
#define RB_EXP_NOROW 0
#endif
#ifndef RK_EXP_NOMFMA
#define RK_EXP_NOMFMA 0
#endif
#ifndef RK_EXP_NOFETCH
#define RK_EXP_NOFETCH 0
#endif
#ifndef RK_EXP_NOHASH
#define RK_EXP_NOHASH 0
#endif
#ifndef RK_EXP_NODX
#define RK_EXP_NODX 0
#endif

namespace ob {

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kThreads = 256;
constexpr int kTile = 64;  // query rows per block (16 per wave)

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
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


// ------------------------------------------------------------------------------------
// Forward: block = (query tile of 64, head, batch row). X rows i0 .. i0+64 live in LDS
// (row 64 = the next tile's first query, needed by the j >= i+2 branch of rel_shift).
// ------------------------------------------------------------------------------------
template <int DQ, int NTT>
__global__ __launch_bounds__(kThreads) void relattn_fwd_kernel(
    const float* __restrict__ q, const float* __restrict__ k, const float* __restrict__ v,
    const float* __restrict__ pos, const float* __restrict__ u, const float* __restrict__ vbias,
    const int* __restrict__ lens, int Bp, int T, int H, float inv_sqrt_d, DropCfg dc,
    const uint64_t* __restrict__ rng, uint64_t rng_off, float* __restrict__ probs,
    float* __restrict__ ctx) {
  constexpr int D = 4 * DQ;
  constexpr int CT = (D + 15) / 16;
  extern __shared__ float xs[];
  const int nt = (T + 15) >> 4;
  // pitch = 2 mod 32: the rel_shift gather below reads lanes r at stride ldx - 1 (bank
  // r + 4g, 2-way) -- a pitch of 16nt+1 put all 16 rows of a lane group on one bank
  const int ldx = 16 * nt + 2;
  const BlockId bid = block_id((T + kTile - 1) / kTile, H);
  const int b = bid.b, h = bid.h, i0 = bid.qt * kTile;
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

  const int qi = i0 + 16 * w + r;  // this lane's query row (scores phase)
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

  // X = (q + v) p^T for the wave's 16 rows: D[m][query] with A = p rows, B = (q+v)
  // four key tiles at a time, s-major: consecutive MFMAs feed different accumulators
  // (per-accumulator order unchanged). The next group's p rows are loaded (unaligned
  // dwordx4 runs) while the current group's MFMAs issue.
  float opa[4][DQ];
  load_group<DQ>(pb, C, 0, r, g, T, opa);
#pragma unroll
  for (int t0 = 0; t0 < NTT; t0 += 4) {
    if (t0 >= nt) continue;
    float opn[4][DQ];
    if (t0 + 4 < NTT && t0 + 4 < nt) load_group<DQ>(pb, C, t0 + 4, r, g, T, opn);
    f32x4 acc[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[u] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < DQ; ++s)
#pragma unroll
      for (int u = 0; u < 4; ++u) if (!RA_EXP_NOX) acc[u] = mfma4(opa[u][s], qv[s], acc[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (t0 + u >= nt) continue;
      float* dst = xs + (16 * w + r) * ldx + 16 * (t0 + u) + 4 * g;
#pragma unroll
      for (int j = 0; j < 4; ++j) dst[j] = acc[u][j];
    }
    if (t0 + 4 < NTT) {
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int s2 = 0; s2 < DQ; ++s2) opa[u][s2] = opn[u][s2];
    }
  }
  // the first key group of the scores phase, in flight over the row-64 work and barrier
  load_group<DQ>(kb, C, 0, r, g, T, opa);
  // row 64: the next tile's first query (fp32 fma chain on the VALU)
  if (!RA_EXP_NOROW64 && i0 + kTile < T) {
    const float* qe = qb + (size_t)(i0 + kTile) * C;
    for (int m = threadIdx.x; m < T; m += kThreads) {
      float pr[D];
      load_run<D>(pb + (size_t)m * C, pr);
      float a = 0.0f;
#pragma unroll
      for (int c = 0; c < D; ++c) a = fmaf(qe[c] + vbb[c], pr[c], a);
      xs[kTile * ldx + m] = a;
    }
  }
  __syncthreads();

  // scores for (query r, keys 16t+4g+j): ac by MFMA (A = k rows, B = q+u), bd gathered
  float sreg[NTT][4];
  float mx = -INFINITY;
  const float* xrow = xs + (16 * w + r) * ldx;
#pragma unroll
  for (int t0 = 0; t0 < NTT; t0 += 4) {
    if (t0 >= nt) continue;
    float opn[4][DQ];
    if (t0 + 4 < NTT && t0 + 4 < nt) load_group<DQ>(kb, C, t0 + 4, r, g, T, opn);
    f32x4 acc4[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) acc4[u] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < DQ; ++s)
#pragma unroll
      for (int u = 0; u < 4; ++u) if (!RA_EXP_NOAC) acc4[u] = mfma4(opa[u][s], qu[s], acc4[u]);
    if (t0 + 4 < NTT) {
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int s2 = 0; s2 < DQ; ++s2) opa[u][s2] = opn[u][s2];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
    const int t = t0 + u;
    if (t >= nt) continue;
    const f32x4 acc = acc4[u];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int jj = 16 * t + 4 * g + j;
      // bd = X[qi][T-1-qi+jj] (jj <= qi), 0 (jj == qi+1), X[qi+1][jj-qi-2] (jj >= qi+2):
      // one LDS read at a select-computed offset (always inside the 65-row image)
      const float xv = xrow[jj - qi + (jj <= qi ? T - 1 : ldx - 2)];
      const float bd = jj == qi + 1 ? 0.0f : xv;
      const float sc = (acc[j] + bd) * inv_sqrt_d;
      const bool valid = qi < L && jj < L;
      sreg[t][j] = valid ? sc : -INFINITY;
      mx = fmaxf(mx, sreg[t][j]);
    }
    }
  }
  mx = fmaxf(mx, __shfl_xor(mx, 16));
  mx = fmaxf(mx, __shfl_xor(mx, 32));
  float sum = 0.0f;
  const bool row_live = mx != -INFINITY;  // all -inf -> softmax NaN -> nan_to_num 0
#pragma unroll
  for (int t = 0; t < NTT; ++t) {
    if (t >= nt) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float e = row_live ? __expf(sreg[t][j] - mx) : 0.0f;
      sreg[t][j] = e;
      sum += e;
    }
  }
  sum += __shfl_xor(sum, 16);
  sum += __shfl_xor(sum, 32);
  const float rsum = 1.0f / sum;
  const uint32_t dkey = dc.on ? drop_key(rng[0], rng[1] + rng_off) : 0u;
  const size_t prow_off = (((size_t)b * H + h) * T + qic) * T;
#pragma unroll
  for (int t = 0; t < NTT; ++t) {
    if (t >= nt) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int jj = 16 * t + 4 * g + j;
      const float pr = row_live ? sreg[t][j] * rsum : 0.0f;
      float pd = pr;
      bool keep = true;
      if (dc.on && !RA_EXP_NODROP) {
        keep = drop_keep(dkey, prow_off + jj, dc.thresh);
        pd = keep ? pr * dc.scale : 0.0f;
      }
      // the keep decision rides in the sign bit (P >= 0): the backward kernels read it
      // back instead of re-hashing every element
      if (!RA_EXP_NOPROBS && probs && qi < T && jj < T) probs[prow_off + jj] = keep ? pr : -pr;
      sreg[t][j] = pd;
    }
  }

  // ctx = A v: A = the lane's probabilities (row r, k = 4g+j of tile t), B = v rows.
  // v [16 nt keys][D] of (b, h) is staged once per block into the X image (free once every
  // wave has passed the scores phase) with coalesced dwordx4 loads; the MFMA operands then
  // come from LDS (row pitch D: the 4 key rows a B fragment touches sit 16 banks apart)
  // instead of 12 scalar L2 loads per lane and key tile in each of the 4 waves.
  __syncthreads();
  float* vs = xs;
  for (int e = threadIdx.x; e < 16 * nt * DQ; e += kThreads) {
    const int key = e / DQ, c4 = 4 * (e - key * DQ);
    const f32x4 v4 = key < T ? *(const f32x4u*)(vbp + (size_t)key * C + c4) : f32x4{0.f, 0.f, 0.f, 0.f};
    *(f32x4*)(vs + key * D + c4) = v4;
  }
  __syncthreads();
  f32x4 o[CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) o[ct] = f32x4{0.f, 0.f, 0.f, 0.f};
  // (columns 16ct + r >= D read the next row: they only feed output columns never stored)
#pragma unroll
  for (int t = 0; t < NTT; ++t) {
    if (t >= nt) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float* vrow = vs + (16 * t + 4 * g + j) * D + r;
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) if (!RA_EXP_NOCTX) o[ct] = mfma4(sreg[t][j], vrow[16 * ct], o[ct]);
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
}

// ------------------------------------------------------------------------------------
// Backward, query side: block = (query tile, head, batch row). Writes dq (final), the
// tile's du / dvb partials (summed by relattn_bias_reduce_kernel) and dS' = dS / sqrt(d)
// to global for the key-side kernel. LDS holds dS' for query rows i0-1 .. i0+63 (row 0 =
// i0-1, recomputed here on the VALU) -- the rows the rel_shift adjoint of the tile needs.
// ------------------------------------------------------------------------------------
template <int DQ, int NTT>
__global__ __launch_bounds__(kThreads) void relattn_bwd_kernel(
    const float* __restrict__ dctx, const float* __restrict__ q, const float* __restrict__ k,
    const float* __restrict__ v, const float* __restrict__ pos, const float* __restrict__ u,
    const float* __restrict__ vbias, const int* __restrict__ lens, int Bp, int T, int H,
    float inv_sqrt_d, DropCfg dc, const uint64_t* __restrict__ rng, uint64_t rng_off,
    const float* __restrict__ probs, float* __restrict__ dq, float* __restrict__ dsg,
    float* __restrict__ du_part,
    float* __restrict__ dvb_part) {
  constexpr int D = 4 * DQ;
  constexpr int CT = (D + 15) / 16;
  extern __shared__ float ds[];
  __shared__ float red[kThreads / 64][2][64];
  __shared__ float rsum[kThreads / 64];
  const int nt = (T + 15) >> 4;
  const int ldx = 16 * nt + 1;
  const int nqt = (T + kTile - 1) / kTile;
  const BlockId bid = block_id(nqt, H);
  const int b = bid.b, h = bid.h, qt = bid.qt, i0 = qt * kTile;
  const int pass = b / Bp;
  const int C = H * D;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 15, g = lane >> 4;
  const size_t bo = (size_t)b * T * C + h * D;
  const float* kb = k + bo;
  const float* vbp = v + bo;
  const float* dob = dctx + bo;
  const float* pb = pos + (size_t)pass * T * C + h * D;
  const float* prb = probs + ((size_t)b * H + h) * T * T;
  (void)rng;
  (void)rng_off;
  // dropout backward factor from a stored probability's sign bit (the forward's keep bit)
  auto keep_scale = [&](float pv) -> float {
    if (!dc.on) return 1.0f;
    return __builtin_signbit(pv) ? 0.0f : dc.scale;
  };

  const int qi = i0 + 16 * w + r;
  const int qic = min(qi, T - 1);
  float dor[DQ];
  load_run<DQ>(dob + (size_t)qic * C + g * DQ, dor);

  // dPd[query r][key] = dO . v (A = v rows, B = dO row), P from the forward
  float dsr[NTT][4];
  float rowdot = 0.0f;
  // (v rows of the next four key tiles load while the current tiles' MFMAs issue)
  float opa[4][DQ];
  load_group<DQ>(vbp, C, 0, r, g, T, opa);
#pragma unroll
  for (int t0 = 0; t0 < NTT; t0 += 4) {
    if (t0 >= nt) continue;
    float opn[4][DQ];
    if (t0 + 4 < NTT && t0 + 4 < nt) load_group<DQ>(vbp, C, t0 + 4, r, g, T, opn);
    f32x4 acc4[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) acc4[u] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < DQ; ++s)
#pragma unroll
      for (int u = 0; u < 4; ++u) if (!RB_EXP_NODP) acc4[u] = mfma4(opa[u][s], dor[s], acc4[u]);
    if (t0 + 4 < NTT) {
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int s2 = 0; s2 < DQ; ++s2) opa[u][s2] = opn[u][s2];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
    const int t = t0 + u;
    if (t >= nt) continue;
    f32x4 acc = acc4[u];
    // the lane's four probabilities P[qi][16t+4g .. +3]: one unaligned dwordx4 when in range
    float pp[4];
    const int jb = 16 * t + 4 * g;
    if (qi < T && jb + 3 < T) {
      const f32x4 v4 = *(const f32x4u*)(prb + (size_t)qi * T + jb);
#pragma unroll
      for (int j = 0; j < 4; ++j) pp[j] = v4[j];
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) pp[j] = (qi < T && jb + j < T) ? prb[(size_t)qi * T + jb + j] : 0.0f;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float p = RB_EXP_NOPROBS ? 0.5f : fabsf(pp[j]);
      const float dp = acc[j] * keep_scale(pp[j]);  // dropout backward
      dsr[t][j] = p;
      acc[j] = dp;
      rowdot += p * dp;
    }
    // dS needs the row sum first: park dP in this lane's own LDS cells meanwhile
    float* dst = ds + (1 + 16 * w + r) * ldx + 16 * t + 4 * g;
#pragma unroll
    for (int j = 0; j < 4; ++j) dst[j] = acc[j];
    }
  }
  rowdot += __shfl_xor(rowdot, 16);
  rowdot += __shfl_xor(rowdot, 32);
  // dS' = P (dP - rowdot) / sqrt(d)  (softmax backward, then the 1/sqrt(d) of :120)
  const float* dprow = ds + (1 + 16 * w + r) * ldx;
#pragma unroll
  for (int t = 0; t < NTT; ++t) {
    if (t >= nt) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int jj = 16 * t + 4 * g + j;
      const float dp = dprow[jj];
      dsr[t][j] = (dsr[t][j] * (dp - rowdot)) * inv_sqrt_d;
    }
  }
  // (each lane rewrites exactly the LDS cells it wrote: no barrier needed in between)
#pragma unroll
  for (int t = 0; t < NTT; ++t) {
    if (t >= nt) continue;
    float* dst = ds + (1 + 16 * w + r) * ldx + 16 * t + 4 * g;
#pragma unroll
    for (int j = 0; j < 4; ++j) dst[j] = dsr[t][j];
  }

  // row i0-1 (LDS row 0) on the VALU, the same formula
  if (!RB_EXP_NOROW && i0 > 0) {
    const int ip = i0 - 1;
    float part = 0.0f;
    for (int jj = threadIdx.x; jj < T; jj += kThreads) {
      const float* vrow = vbp + (size_t)jj * C;
      const float* drow = dob + (size_t)ip * C;
      float a = 0.0f;
      for (int c = 0; c < D; ++c) a = fmaf(vrow[c], drow[c], a);
      const float pv = prb[(size_t)ip * T + jj];
      const float dp = a * keep_scale(pv);
      const float p = fabsf(pv);
      ds[jj] = dp;
      part += p * dp;
    }
    for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o);
    if (lane == 0) rsum[w] = part;
    __syncthreads();
    const float rd = ((rsum[0] + rsum[1]) + rsum[2]) + rsum[3];
    for (int jj = threadIdx.x; jj < T; jj += kThreads) {
      const float p = fabsf(prb[(size_t)ip * T + jj]);
      ds[jj] = (p * (ds[jj] - rd)) * inv_sqrt_d;
    }
  }
  __syncthreads();

  // dQu = dS' k (A = dS' row r, k = 4g+j of tile t; B = k rows)
  f32x4 oq[CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) oq[ct] = f32x4{0.f, 0.f, 0.f, 0.f};
  // (B operands k[16t+4g+j][16ct+r] of tile t+1 load while tile t's MFMAs issue)
  auto load_b = [&](const float* base, int t, float (&dst)[4][CT]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float* row = base + (size_t)min(16 * t + 4 * g + j, T - 1) * C;
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) dst[j][ct] = row[min(16 * ct + r, D - 1)];
    }
  };
  {
    float kb_cur[4][CT];
    load_b(kb, 0, kb_cur);
#pragma unroll
    for (int t = 0; t < NTT; ++t) {
      if (t >= nt) continue;
      float kb_nxt[4][CT];
      if (t + 1 < NTT && t + 1 < nt) load_b(kb, t + 1, kb_nxt);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) if (!RB_EXP_NODQU) oq[ct] = mfma4(dsr[t][j], kb_cur[j][ct], oq[ct]);
      if (t + 1 < NTT) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int ct = 0; ct < CT; ++ct) kb_cur[j][ct] = kb_nxt[j][ct];
      }
    }
  }
  // dQv = dX p, dX gathered from LDS by the rel_shift adjoint
  f32x4 ov[CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) ov[ct] = f32x4{0.f, 0.f, 0.f, 0.f};
  // dX[qi][m] = dS'[qi][m-T+1+qi] (m >= T-1-qi), else dS'[qi-1][m+qi+1] (qi >= 1): one LDS
  // read at a select-computed offset (LDS row 1+16w+r holds dS' row qi, the row above it
  // qi-1). Positions m = 4mk+g go four MFMA steps at a time, the next four's p operands
  // loading meanwhile; steps past the end multiply zeros.
  const float* row_i = ds + (1 + 16 * w + r) * ldx;
  const int nk = (T + 3) >> 2;
  constexpr int kMK = 4;
  auto load_p = [&](int mk0, float (&dst)[kMK][CT]) {
#pragma unroll
    for (int q = 0; q < kMK; ++q) {
      const float* prow = pb + (size_t)min(4 * (mk0 + q) + g, T - 1) * C;
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) dst[q][ct] = prow[min(16 * ct + r, D - 1)];
    }
  };
  float pv_cur[kMK][CT];
  load_p(0, pv_cur);
  for (int mk0 = 0; mk0 < nk; mk0 += kMK) {
    float pv_nxt[kMK][CT];
    if (mk0 + kMK < nk) load_p(mk0 + kMK, pv_nxt);
    float av[kMK];
#pragma unroll
    for (int q = 0; q < kMK; ++q) {
      const int m = 4 * (mk0 + q) + g;
      const int mm = min(m, T - 1);  // (clamped address; the value is masked below)
      const bool upper = mm >= T - 1 - qic;
      const float x = row_i[mm + qic + 1 - (upper ? T : ldx)];
      av[q] = (qi < T && m < T && (upper || qi >= 1)) ? x : 0.0f;
    }
#pragma unroll
    for (int q = 0; q < kMK; ++q)
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) if (!RB_EXP_NODQV) ov[ct] = mfma4(av[q], pv_cur[q][ct], ov[ct]);
#pragma unroll
    for (int q = 0; q < kMK; ++q)
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) pv_cur[q][ct] = pv_nxt[q][ct];
  }
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
    su[ct] += __shfl_xor(su[ct], 16);
    su[ct] += __shfl_xor(su[ct], 32);
    sv[ct] += __shfl_xor(sv[ct], 16);
    sv[ct] += __shfl_xor(sv[ct], 32);
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
  __syncthreads();
  if (threadIdx.x < D) {
    const int c = threadIdx.x;
    du_part[tile_id * D + c] = ((red[0][0][c] + red[1][0][c]) + red[2][0][c]) + red[3][0][c];
    dvb_part[tile_id * D + c] = ((red[0][1][c] + red[1][1][c]) + red[2][1][c]) + red[3][1][c];
  }

  // dS' rows of this tile to global for the key-side kernel (row-contiguous copy of the
  // LDS image: wave w copies rows 16w .. 16w+15, 64 consecutive columns per instruction)
  float* dsb = dsg + ((size_t)b * H + h) * T * T;
  // (4 consecutive floats per lane: one unaligned dwordx4 store, 16 per wave and row
  // quarter instead of 64 dword stores)
  for (int rr = 0; rr < 16; ++rr) {
    const int qrow = i0 + 16 * w + rr;
    if (qrow >= T) break;
    const float* src = ds + (1 + 16 * w + rr) * ldx;
    float* dst = dsb + (size_t)qrow * T;
    for (int j4 = 4 * lane; j4 < T; j4 += 256) {
      if (RB_EXP_NODSG) break;
      if (j4 + 3 < T) {
        const f32x4 v4 = {src[j4], src[j4 + 1], src[j4 + 2], src[j4 + 3]};
        *(f32x4u*)(dst + j4) = v4;
      } else {
        for (int e = j4; e < T; ++e) dst[e] = src[e];
      }
    }
  }
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
    int T, int H, DropCfg dc, const uint64_t* __restrict__ rng, uint64_t rng_off,
    float* __restrict__ dk,
    float* __restrict__ dv, float* __restrict__ dp_part) {
  constexpr int D = 4 * DQ;
  constexpr int CT = (D + 15) / 16;
  using St = KvStage<D>;
  constexpr int kQ = St::kQ;
  __shared__ St st;
  const int nkt = (T + kTile - 1) / kTile;
  const BlockId bid = block_id(nkt, H);
  const int b = bid.b, h = bid.h, k0 = bid.qt * kTile;
  const int C = H * D;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 15, g = lane >> 4;
  const size_t bo = (size_t)b * T * C + h * D;
  const float* qb = q + bo;
  const float* dob = dctx + bo;
  const float* ub = u + h * D;
  const float* vbb = vbias + h * D;
  const float* dsb = dsg + ((size_t)b * H + h) * T * T;
  const float* prb = probs + ((size_t)b * H + h) * T * T;
  (void)rng;
  (void)rng_off;

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
  f32x4 ra_k[kAH], ra_v[kAH], ra_p[kAH], rb[St::kBSlots];
  auto fetch = [&](int i0) {
#pragma unroll
    for (int hf = 0; hf < kAH; ++hf) {
    const int i = i0 + ai + 16 * hf;
    const int key0 = k0 + ax;
    if (i < T && key0 + 3 < T) {
      ra_k[hf] = *(const f32x4u*)(dsb + (size_t)i * T + key0);
      ra_v[hf] = *(const f32x4u*)(prb + (size_t)i * T + key0);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bool ok = i < T && key0 + j < T;
        ra_k[hf][j] = ok ? dsb[(size_t)i * T + key0 + j] : 0.0f;
        ra_v[hf][j] = ok ? prb[(size_t)i * T + key0 + j] : 0.0f;
      }
    }
    // dX[i][m0..m0+3]: one unaligned dwordx4 when the four positions sit in one branch of
    // the adjoint (upper: dS' row i from column m0-T+1+i; lower: row i-1 from m0+i+1)
    const int up0 = T - 1 - i;  // first upper position of row i
    if (i < T && key0 + 3 < T && (key0 >= up0 || (key0 + 3 < up0 && i >= 1))) {
      const float* src = key0 >= up0 ? dsb + (size_t)i * T + (key0 - up0)
                                     : dsb + (size_t)(i - 1) * T + (key0 + i + 1);
      ra_p[hf] = RK_EXP_NODX ? f32x4{0.5f, 0.5f, 0.5f, 0.5f} : *(const f32x4u*)src;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = key0 + j;
        const bool ok = i < T && m < T;
        const int ic = min(i, T - 1), mc = min(m, T - 1);
        const bool upper = mc >= T - 1 - ic;
        const size_t off = upper ? (size_t)ic * T + (mc - T + 1 + ic)
                                 : (size_t)max(ic - 1, 0) * T + min(mc + ic + 1, T - 1);
        const float x = RK_EXP_NODX ? 0.5f : dsb[off];
        ra_p[hf][j] = (ok && (upper || ic >= 1)) ? x : 0.0f;
      }
    }
    // Pd = P * keep * scale, the keep bit from the stored probability's sign
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (!RK_EXP_NOHASH && dc.on)
        ra_v[hf][j] = __builtin_signbit(ra_v[hf][j]) ? 0.0f : ra_v[hf][j] * dc.scale;
    }
    }
#pragma unroll
    for (int sl = 0; sl < St::kBSlots; ++sl) {
      const int e = threadIdx.x + kThreads * sl;
      const int e2 = e < St::kBVec ? e : e - St::kBVec;
      const int row = i0 + e2 / DQ, c4 = 4 * (e2 % DQ);
      if (e < 2 * St::kBVec && row < T) {
        const float* src = (e < St::kBVec ? qb : dob) + (size_t)row * C + c4;
        rb[sl] = *(const f32x4u*)src;
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
  fetch(0);
  for (int i0 = 0; i0 < T; i0 += kQ) {
    __syncthreads();  // the previous chunk's LDS reads are done
    stage();
    __syncthreads();
    if (!RK_EXP_NOFETCH && i0 + kQ < T) fetch(i0 + kQ);
#pragma unroll
    for (int s4 = 0; s4 < kQ / 4; ++s4) {
      const int qq = 4 * s4 + g;
      const float a_k = st.ak[qq][kl], a_v = st.av[qq][kl], a_p = st.ap[qq][kl];
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        const int col = 16 * ct + r;
        if (RK_EXP_NOMFMA) {
          ak[ct][0] += a_k * st.qu[qq][col];
          av[ct][0] += a_v * st.dob[qq][col];
          ap[ct][0] += a_p * st.qv[qq][col];
          continue;
        }
        ak[ct] = mfma4(a_k, st.qu[qq][col], ak[ct]);
        av[ct] = mfma4(a_v, st.dob[qq][col], av[ct]);
        ap[ct] = mfma4(a_p, st.qv[qq][col], ap[ct]);
      }
    }
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
}

// du, dvb [H][D]: sum over (batch row, query tile) of the per-tile partials. Block = one
// (which, head) x 4 columns x 64 slices (slice s: pairs s, s+64, ..., four accumulators),
// the slices added in order through LDS (fixed order). 2*H*ceil(D/4) blocks: each thread
// has a few independent loads in flight (one block per (which, head) with a serial chain of
// 24 partials per thread measured 15 us at Conformer-S).
constexpr int kBiasCols = 4, kBiasSlices = kThreads / kBiasCols;

__global__ __launch_bounds__(kThreads) void relattn_bias_reduce_kernel(
    const float* __restrict__ du_part, const float* __restrict__ dvb_part, int Bt, int H, int D,
    int nqt, float* __restrict__ du, float* __restrict__ dvb) {
  __shared__ float red[kBiasSlices][kBiasCols];
  const int ncg = (D + kBiasCols - 1) / kBiasCols;
  const int cg = blockIdx.x % ncg, wh = blockIdx.x / ncg;
  const int which = wh / H, h = wh - which * H;
  const int cl = threadIdx.x % kBiasCols, sl = threadIdx.x / kBiasCols;
  const int c = cg * kBiasCols + cl;
  const float* src = which == 0 ? du_part : dvb_part;
  const int pairs = Bt * nqt;
  float a[4] = {0.f, 0.f, 0.f, 0.f};
  if (c < D) {
    int u = 0;
    for (int q = sl; q < pairs; q += kBiasSlices, ++u) {
      const int b = q / nqt, qt = q - b * nqt;
      a[u & 3] += src[(((size_t)b * H + h) * nqt + qt) * D + c];
    }
  }
  red[sl][cl] = (a[0] + a[1]) + (a[2] + a[3]);
  __syncthreads();
  if (sl == 0 && c < D) {
    float t = 0.0f;
#pragma unroll 8
    for (int q = 0; q < kBiasSlices; ++q) t += red[q][cl];
    (which == 0 ? du : dvb)[h * D + c] = t;
  }
}

// dpos [P][T][H*D]: sum over the pass's Bp batch rows and the query tiles. Block = 64
// consecutive output elements x 4 batch slices (slice s: rows s, s+4, ... of the pass);
// the slices are added in slice order through LDS (fixed order: deterministic).
__global__ __launch_bounds__(kThreads) void relattn_dpos_reduce_kernel(
    const float* __restrict__ dp_part, int Bt, int P, int T, int H, int D, int nqt,
    float* __restrict__ dpos) {
  __shared__ float red[4][64];
  const int C = H * D;
  const int64_t n_p = (int64_t)P * T * C;
  const int el = threadIdx.x & 63, sl = threadIdx.x >> 6;
  const int64_t f = (int64_t)blockIdx.x * 64 + el;
  const int Bp = Bt / P;
  float s = 0.0f;
  if (f < n_p) {
    const int p = (int)(f / ((int64_t)T * C));
    const int rem = (int)(f - (int64_t)p * T * C);
    const int t = rem / C, hc = rem - t * C, h = hc / D, c = hc - h * D;
    float a[4] = {0.f, 0.f, 0.f, 0.f};
    int u = 0;
    for (int b = p * Bp + sl; b < (p + 1) * Bp; b += 4, ++u)
      for (int qt = 0; qt < nqt; ++qt)
        a[u & 3] += dp_part[(((((size_t)qt * Bt + b) * H + h) * T) + t) * D + c];
    s = (a[0] + a[1]) + (a[2] + a[3]);
  }
  red[sl][el] = s;
  __syncthreads();
  if (sl == 0 && f < n_p) dpos[f] = ((red[0][el] + red[1][el]) + red[2][el]) + red[3][el];
}

__global__ __launch_bounds__(kThreads) void relattn_mask_kernel(int64_t n, DropCfg dc,
                                                                const uint64_t* __restrict__ rng,
                                                                uint64_t rng_off,
                                                                uint8_t* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (e >= n) return;
  out[e] = (!dc.on || drop_keep(drop_key(rng[0], rng[1] + rng_off), (uint64_t)e, dc.thresh)) ? 1 : 0;
}


// (the forward's pitch, 16nt+2; the backward uses 16nt+1)
size_t lds_bytes(int T) { return sizeof(float) * (size_t)(kTile + 1) * (16 * ((T + 15) / 16) + 2); }

}  // namespace

bool relattn_supported(int64_t T, int64_t d) {
  return T >= 1 && T <= 512 && (d == 16 || d == 32 || d == 36 || d == 64);
}

// ws: dS' [Bt][H][T][T] | dpos per batch row [Bt][H][T][d] | du, dvb tile partials.
size_t relattn_bwd_workspace(int64_t Bt, int64_t T, int64_t H, int64_t d) {
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
                        uint64_t rng_off, float* probs, float* ctx, hipStream_t s) {
  const dim3 grid((unsigned)(((T + kTile - 1) / kTile) * H * Bt));
  const DropCfg dc = make_drop(p_drop);
  const float inv_sqrt_d = 1.0f / (float)sqrt((double)d);  // torch: tensor / scalar = * (1/scalar)
  const size_t lds = lds_bytes((int)T);
#define OB_RA_FWD(DQ, NTT)                                                                 \
  hipLaunchKernelGGL((relattn_fwd_kernel<DQ, NTT>), grid, dim3(kThreads), lds, s, q, k, v, pos, \
                     u, vb, lens, (int)(Bt / P), (int)T, (int)H, inv_sqrt_d, dc, rng, rng_off, probs, ctx)
  OB_RA_DISPATCH(OB_RA_FWD);
#undef OB_RA_FWD
}

void launch_relattn_bwd(const float* dctx, const float* q, const float* k, const float* v,
                        const float* pos, const float* u, const float* vb, const int* lens,
                        int64_t Bt, int64_t P, int64_t T, int64_t H, int64_t d, float p_drop,
                        const uint64_t* rng, uint64_t rng_off, const float* probs, float* dq,
                        float* dk, float* dv, float* dpos, float* du, float* dvb, void* ws,
                        hipStream_t s) {
  const int nqt = (int)((T + kTile - 1) / kTile);
  const dim3 grid((unsigned)(nqt * H * Bt));
  const DropCfg dc = make_drop(p_drop);
  const float inv_sqrt_d = 1.0f / (float)sqrt((double)d);  // torch: tensor / scalar = * (1/scalar)
  const size_t lds = lds_bytes((int)T);
  float* dsg = (float*)ws;
  float* dp_part = dsg + (size_t)Bt * H * T * T;
  float* du_part = dp_part + (size_t)Bt * H * T * d;
  float* dvb_part = du_part + (size_t)Bt * H * nqt * d;
#define OB_RA_BWD(DQ, NTT)                                                                     \
  hipLaunchKernelGGL((relattn_bwd_kernel<DQ, NTT>), grid, dim3(kThreads), lds, s, dctx, q, k, v,  \
                     pos, u, vb, lens, (int)(Bt / P), (int)T, (int)H, inv_sqrt_d, dc, rng, rng_off, probs, dq, \
                     dsg, du_part, dvb_part)
  OB_RA_DISPATCH(OB_RA_BWD);
#undef OB_RA_BWD
#define OB_RA_KV(DQ, NTT)                                                                       \
  hipLaunchKernelGGL((relattn_bwd_kv_kernel<DQ>), grid, dim3(kThreads), 0, s, (const float*)dsg, \
                     probs, q, dctx, u, vb, (int)T, (int)H, dc, rng, rng_off, dk, dv, dp_part)
  OB_RA_DISPATCH(OB_RA_KV);
#undef OB_RA_KV
  const int64_t C = H * d;
  hipLaunchKernelGGL(relattn_bias_reduce_kernel,
                     dim3((unsigned)(2 * H * ((d + kBiasCols - 1) / kBiasCols))), dim3(kThreads),
                     0, s, (const float*)du_part, (const float*)dvb_part, (int)Bt, (int)H, (int)d,
                     nqt, du, dvb);
  hipLaunchKernelGGL(relattn_dpos_reduce_kernel, dim3((unsigned)ceil_div(P * T * C, 64)),
                     dim3(kThreads), 0, s, (const float*)dp_part, (int)Bt, (int)P, (int)T, (int)H,
                     (int)d, 1, dpos);
}

void launch_relattn_dropout_mask(int64_t n, float p_drop, const uint64_t* rng, uint64_t rng_off,
                                 uint8_t* out, hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL(relattn_mask_kernel, dim3((unsigned)((n + kThreads - 1) / kThreads)),
                     dim3(kThreads), 0, s, n, make_drop(p_drop), rng, rng_off, out);
}

}  // namespace ob
