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
// Dropout keeps (i, j) when hash(key(seed, counter), index) >= p * 2^32 (a counter hash:
// the backward regenerates the same mask; torch's own RNG stream is not reproduced).
#include <math.h>

#include "ob_drop.h"
#include "ob_launch.h"

namespace ob {

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kThreads = 256;
constexpr int kTile = 64;  // query rows per block (16 per wave)

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
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
    const int* __restrict__ lens, int Bp, int T, int H, float sqrt_d, DropCfg dc,
    const uint64_t* __restrict__ rng, float* __restrict__ probs, float* __restrict__ ctx) {
  constexpr int D = 4 * DQ;
  constexpr int CT = (D + 15) / 16;
  extern __shared__ float xs[];
  const int nt = (T + 15) >> 4;
  const int ldx = 16 * nt + 1;
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
#pragma unroll
  for (int s = 0; s < DQ; ++s) {
    const int c = g * DQ + s;
    const float x = qb[(size_t)qic * C + c];
    qu[s] = x + ub[c];
    qv[s] = x + vbb[c];
  }

  // X = (q + v) p^T for the wave's 16 rows: D[m][query] with A = p rows, B = (q+v)
  // four key tiles at a time, s-major: consecutive MFMAs feed different accumulators
  // (per-accumulator order unchanged)
#pragma unroll
  for (int t0 = 0; t0 < NTT; t0 += 4) {
    if (t0 >= nt) continue;
    f32x4 acc[4];
    const float* prow[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      acc[u] = f32x4{0.f, 0.f, 0.f, 0.f};
      prow[u] = pb + (size_t)min(16 * (t0 + u) + r, T - 1) * C + g * DQ;
    }
#pragma unroll
    for (int s = 0; s < DQ; ++s)
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[u] = mfma4(prow[u][s], qv[s], acc[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (t0 + u >= nt) continue;
      float* dst = xs + (16 * w + r) * ldx + 16 * (t0 + u) + 4 * g;
#pragma unroll
      for (int j = 0; j < 4; ++j) dst[j] = acc[u][j];
    }
  }
  // row 64: the next tile's first query (fp32 fma chain on the VALU)
  if (i0 + kTile < T) {
    const float* qe = qb + (size_t)(i0 + kTile) * C;
    for (int m = threadIdx.x; m < T; m += kThreads) {
      const float* prow = pb + (size_t)m * C;
      float a = 0.0f;
      for (int c = 0; c < D; ++c) a = fmaf(qe[c] + vbb[c], prow[c], a);
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
    f32x4 acc4[4];
    const float* krow[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      acc4[u] = f32x4{0.f, 0.f, 0.f, 0.f};
      krow[u] = kb + (size_t)min(16 * (t0 + u) + r, T - 1) * C + g * DQ;
    }
#pragma unroll
    for (int s = 0; s < DQ; ++s)
#pragma unroll
      for (int u = 0; u < 4; ++u) acc4[u] = mfma4(krow[u][s], qu[s], acc4[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
    const int t = t0 + u;
    if (t >= nt) continue;
    const f32x4 acc = acc4[u];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int jj = 16 * t + 4 * g + j;
      float bd;
      if (jj <= qi) bd = xrow[max(T - 1 - qi + jj, 0)];
      else if (jj == qi + 1) bd = 0.0f;
      else bd = xrow[ldx + (jj - qi - 2)];
      const float sc = (acc[j] + bd) / sqrt_d;
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
      const float e = row_live ? expf(sreg[t][j] - mx) : 0.0f;
      sreg[t][j] = e;
      sum += e;
    }
  }
  sum += __shfl_xor(sum, 16);
  sum += __shfl_xor(sum, 32);
  const uint32_t dkey = dc.on ? drop_key(rng[0], rng[1]) : 0u;
  const size_t prow_off = (((size_t)b * H + h) * T + qic) * T;
#pragma unroll
  for (int t = 0; t < NTT; ++t) {
    if (t >= nt) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int jj = 16 * t + 4 * g + j;
      const float pr = row_live ? sreg[t][j] / sum : 0.0f;
      if (probs && qi < T && jj < T) probs[prow_off + jj] = pr;
      float pd = pr;
      if (dc.on) {
        const bool keep = drop_hash(dkey, prow_off + jj) >= dc.thresh;
        pd = keep ? pr * dc.scale : 0.0f;
      }
      sreg[t][j] = pd;
    }
  }

  // ctx = A v: A = the lane's probabilities (row r, k = 4g+j of tile t), B = v rows
  f32x4 o[CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) o[ct] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < NTT; ++t) {
    if (t >= nt) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int key = min(16 * t + 4 * g + j, T - 1);
      const float* vrow = vbp + (size_t)key * C;
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) o[ct] = mfma4(sreg[t][j], vrow[min(16 * ct + r, D - 1)], o[ct]);
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
    float sqrt_d, DropCfg dc, const uint64_t* __restrict__ rng, const float* __restrict__ probs,
    float* __restrict__ dq, float* __restrict__ dsg, float* __restrict__ du_part,
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
  const uint32_t dkey = dc.on ? drop_key(rng[0], rng[1]) : 0u;
  const size_t pbase = ((size_t)b * H + h) * T * T;
  auto keep_scale = [&](int i, int j) -> float {
    if (!dc.on) return 1.0f;
    return drop_hash(dkey, pbase + (size_t)i * T + j) >= dc.thresh ? dc.scale : 0.0f;
  };

  const int qi = i0 + 16 * w + r;
  const int qic = min(qi, T - 1);
  float dor[DQ];
#pragma unroll
  for (int s = 0; s < DQ; ++s) dor[s] = dob[(size_t)qic * C + g * DQ + s];

  // dPd[query r][key] = dO . v (A = v rows, B = dO row), P from the forward
  float dsr[NTT][4];
  float rowdot = 0.0f;
#pragma unroll
  for (int t0 = 0; t0 < NTT; t0 += 4) {
    if (t0 >= nt) continue;
    f32x4 acc4[4];
    const float* vrow[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      acc4[u] = f32x4{0.f, 0.f, 0.f, 0.f};
      vrow[u] = vbp + (size_t)min(16 * (t0 + u) + r, T - 1) * C + g * DQ;
    }
#pragma unroll
    for (int s = 0; s < DQ; ++s)
#pragma unroll
      for (int u = 0; u < 4; ++u) acc4[u] = mfma4(vrow[u][s], dor[s], acc4[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
    const int t = t0 + u;
    if (t >= nt) continue;
    f32x4 acc = acc4[u];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int jj = 16 * t + 4 * g + j;
      const float p = (qi < T && jj < T) ? prb[(size_t)qi * T + jj] : 0.0f;
      const float dp = acc[j] * keep_scale(qic, jj);  // dropout backward
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
      dsr[t][j] = (dsr[t][j] * (dp - rowdot)) / sqrt_d;
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
  if (i0 > 0) {
    const int ip = i0 - 1;
    float part = 0.0f;
    for (int jj = threadIdx.x; jj < T; jj += kThreads) {
      const float* vrow = vbp + (size_t)jj * C;
      const float* drow = dob + (size_t)ip * C;
      float a = 0.0f;
      for (int c = 0; c < D; ++c) a = fmaf(vrow[c], drow[c], a);
      const float dp = a * keep_scale(ip, jj);
      const float p = prb[(size_t)ip * T + jj];
      ds[jj] = dp;
      part += p * dp;
    }
    for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o);
    if (lane == 0) rsum[w] = part;
    __syncthreads();
    const float rd = ((rsum[0] + rsum[1]) + rsum[2]) + rsum[3];
    for (int jj = threadIdx.x; jj < T; jj += kThreads) {
      const float p = prb[(size_t)ip * T + jj];
      ds[jj] = (p * (ds[jj] - rd)) / sqrt_d;
    }
  }
  __syncthreads();

  // dQu = dS' k (A = dS' row r, k = 4g+j of tile t; B = k rows)
  f32x4 oq[CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) oq[ct] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < NTT; ++t) {
    if (t >= nt) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int key = min(16 * t + 4 * g + j, T - 1);
      const float* krow = kb + (size_t)key * C;
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) oq[ct] = mfma4(dsr[t][j], krow[min(16 * ct + r, D - 1)], oq[ct]);
    }
  }
  // dQv = dX p, dX gathered from LDS by the rel_shift adjoint
  f32x4 ov[CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) ov[ct] = f32x4{0.f, 0.f, 0.f, 0.f};
  const float* row_i = ds + (1 + 16 * w + r) * ldx;  // dS' row qi
  const float* row_im1 = row_i - ldx;                 // dS' row qi-1
  auto dX = [&](int i, const float* ri, const float* rim1, int m) -> float {
    if (m >= T - 1 - i) return ri[m - T + 1 + i];
    return i >= 1 ? rim1[m + i + 1] : 0.0f;
  };
  const int nk = (T + 3) >> 2;
  for (int mk = 0; mk < nk; ++mk) {
    const int m = 4 * mk + g;
    const float a = (qi < T && m < T) ? dX(qi, row_i, row_im1, m) : 0.0f;
    const float* prow = pb + (size_t)min(m, T - 1) * C;
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) ov[ct] = mfma4(a, prow[min(16 * ct + r, D - 1)], ov[ct]);
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
  for (int rr = 0; rr < 16; ++rr) {
    const int qrow = i0 + 16 * w + rr;
    if (qrow >= T) break;
    const float* src = ds + (1 + 16 * w + rr) * ldx;
    for (int jj = lane; jj < T; jj += 64) dsb[(size_t)qrow * T + jj] = src[jj];
  }
}

// ------------------------------------------------------------------------------------
// Backward, key side: block = (key tile of 64, head, batch row), wave w = keys 16w..16w+15
// of the tile; every query row is visited (no per-query-tile partials):
//   dK[key]  = sum_i dS'[i][key] (q+u)[i]       dV[key] = sum_i Pd[i][key] dO[i]
//   dpos[m]  = sum_i dX[i][m] (q+v)[i]          (per batch row; summed over the pass later)
// MFMA 16x16x4: A[key r][query g] from dS' / probs (global, coalesced over keys), B[query
// g][column] from q / dO rows; four query steps are issued per iteration.
// ------------------------------------------------------------------------------------
template <int DQ>
__global__ __launch_bounds__(kThreads) void relattn_bwd_kv_kernel(
    const float* __restrict__ dsg, const float* __restrict__ probs, const float* __restrict__ q,
    const float* __restrict__ dctx, const float* __restrict__ u, const float* __restrict__ vbias,
    int T, int H, DropCfg dc, const uint64_t* __restrict__ rng, float* __restrict__ dk,
    float* __restrict__ dv, float* __restrict__ dp_part) {
  constexpr int D = 4 * DQ;
  constexpr int CT = (D + 15) / 16;
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
  const uint32_t dkey = dc.on ? drop_key(rng[0], rng[1]) : 0u;
  const size_t pbase = ((size_t)b * H + h) * T * T;
  const int key = k0 + 16 * w + r;  // A row: key / position m
  const bool kok = key < T;
  const int kc = min(key, T - 1);
  float bu[CT], bv[CT];
  int cc[CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    cc[ct] = min(16 * ct + r, D - 1);
    bu[ct] = ub[cc[ct]];
    bv[ct] = vbb[cc[ct]];
  }
  f32x4 ak[CT], av[CT], ap[CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    ak[ct] = f32x4{0.f, 0.f, 0.f, 0.f};
    av[ct] = f32x4{0.f, 0.f, 0.f, 0.f};
    ap[ct] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  // dX[i][m] = dS'[i][m-T+1+i] (m >= T-1-i), else dS'[i-1][m+i+1] (i >= 1)
  auto dx_at = [&](int i) -> float {
    if (kc >= T - 1 - i) return dsb[(size_t)i * T + (kc - T + 1 + i)];
    return i >= 1 ? dsb[(size_t)(i - 1) * T + (kc + i + 1)] : 0.0f;
  };
  constexpr int kU = 4;  // query steps (of 4 rows) in flight
  for (int i0 = 0; i0 < T; i0 += 4 * kU) {
    float a_k[kU], a_v[kU], a_p[kU], qx[kU][CT], dx[kU][CT];
#pragma unroll
    for (int uu = 0; uu < kU; ++uu) {
      const int i = i0 + 4 * uu + g;
      const bool ok = kok && i < T;
      const int ic = min(i, T - 1);
      a_k[uu] = ok ? dsb[(size_t)ic * T + kc] : 0.0f;
      const float pv = ok ? prb[(size_t)ic * T + kc] : 0.0f;
      a_v[uu] = dc.on ? (drop_hash(dkey, pbase + (size_t)ic * T + kc) >= dc.thresh ? pv * dc.scale : 0.0f) : pv;
      a_p[uu] = ok ? dx_at(ic) : 0.0f;
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        qx[uu][ct] = qb[(size_t)ic * C + cc[ct]];
        dx[uu][ct] = dob[(size_t)ic * C + cc[ct]];
      }
    }
#pragma unroll
    for (int uu = 0; uu < kU; ++uu) {
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        ak[ct] = mfma4(a_k[uu], qx[uu][ct] + bu[ct], ak[ct]);
        av[ct] = mfma4(a_v[uu], dx[uu][ct], av[ct]);
        ap[ct] = mfma4(a_p[uu], qx[uu][ct] + bv[ct], ap[ct]);
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
// (which, head) x 64 columns x 16 slices (slice s: pairs s, s+16, ...), slices added in
// order through LDS (fixed order). A thread per output with a serial loop over the
// Bt*nqt partials measured 170 us at Conformer-S (one dependent load chain per thread).
constexpr int kBiasSlices = 16;

__global__ __launch_bounds__(64 * kBiasSlices) void relattn_bias_reduce_kernel(
    const float* __restrict__ du_part, const float* __restrict__ dvb_part, int Bt, int H, int D,
    int nqt, float* __restrict__ du, float* __restrict__ dvb) {
  __shared__ float red[kBiasSlices][64];
  const int which = blockIdx.x / H, h = blockIdx.x - which * H;
  const int c = threadIdx.x & 63, sl = threadIdx.x >> 6;
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
  red[sl][c] = (a[0] + a[1]) + (a[2] + a[3]);
  __syncthreads();
  if (sl == 0 && c < D) {
    float t = 0.0f;
#pragma unroll
    for (int q = 0; q < kBiasSlices; ++q) t += red[q][c];
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
                                                                uint8_t* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (e >= n) return;
  out[e] = (!dc.on || drop_hash(drop_key(rng[0], rng[1]), (uint64_t)e) >= dc.thresh) ? 1 : 0;
}


size_t lds_bytes(int T) { return sizeof(float) * (size_t)(kTile + 1) * (16 * ((T + 15) / 16) + 1); }

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
                        float* probs, float* ctx, hipStream_t s) {
  const dim3 grid((unsigned)(((T + kTile - 1) / kTile) * H * Bt));
  const DropCfg dc = make_drop(p_drop);
  const float sqrt_d = (float)sqrt((double)d);
  const size_t lds = lds_bytes((int)T);
#define OB_RA_FWD(DQ, NTT)                                                                 \
  hipLaunchKernelGGL((relattn_fwd_kernel<DQ, NTT>), grid, dim3(kThreads), lds, s, q, k, v, pos, \
                     u, vb, lens, (int)(Bt / P), (int)T, (int)H, sqrt_d, dc, rng, probs, ctx)
  OB_RA_DISPATCH(OB_RA_FWD);
#undef OB_RA_FWD
}

void launch_relattn_bwd(const float* dctx, const float* q, const float* k, const float* v,
                        const float* pos, const float* u, const float* vb, const int* lens,
                        int64_t Bt, int64_t P, int64_t T, int64_t H, int64_t d, float p_drop,
                        const uint64_t* rng, const float* probs, float* dq, float* dk, float* dv,
                        float* dpos, float* du, float* dvb, void* ws, hipStream_t s) {
  const int nqt = (int)((T + kTile - 1) / kTile);
  const dim3 grid((unsigned)(nqt * H * Bt));
  const DropCfg dc = make_drop(p_drop);
  const float sqrt_d = (float)sqrt((double)d);
  const size_t lds = lds_bytes((int)T);
  float* dsg = (float*)ws;
  float* dp_part = dsg + (size_t)Bt * H * T * T;
  float* du_part = dp_part + (size_t)Bt * H * T * d;
  float* dvb_part = du_part + (size_t)Bt * H * nqt * d;
#define OB_RA_BWD(DQ, NTT)                                                                     \
  hipLaunchKernelGGL((relattn_bwd_kernel<DQ, NTT>), grid, dim3(kThreads), lds, s, dctx, q, k, v,  \
                     pos, u, vb, lens, (int)(Bt / P), (int)T, (int)H, sqrt_d, dc, rng, probs, dq, \
                     dsg, du_part, dvb_part)
  OB_RA_DISPATCH(OB_RA_BWD);
#undef OB_RA_BWD
#define OB_RA_KV(DQ, NTT)                                                                       \
  hipLaunchKernelGGL((relattn_bwd_kv_kernel<DQ>), grid, dim3(kThreads), 0, s, (const float*)dsg, \
                     probs, q, dctx, u, vb, (int)T, (int)H, dc, rng, dk, dv, dp_part)
  OB_RA_DISPATCH(OB_RA_KV);
#undef OB_RA_KV
  const int64_t C = H * d;
  hipLaunchKernelGGL(relattn_bias_reduce_kernel, dim3((unsigned)(2 * H)), dim3(64 * kBiasSlices),
                     0, s, (const float*)du_part, (const float*)dvb_part, (int)Bt, (int)H, (int)d,
                     nqt, du, dvb);
  hipLaunchKernelGGL(relattn_dpos_reduce_kernel, dim3((unsigned)ceil_div(P * T * C, 64)),
                     dim3(kThreads), 0, s, (const float*)dp_part, (int)Bt, (int)P, (int)T, (int)H,
                     (int)d, 1, dpos);
}

void launch_relattn_dropout_mask(int64_t n, float p_drop, const uint64_t* rng, uint8_t* out,
                                 hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL(relattn_mask_kernel, dim3((unsigned)((n + kThreads - 1) / kThreads)),
                     dim3(kThreads), 0, s, n, make_drop(p_drop), rng, out);
}

}  // namespace ob
