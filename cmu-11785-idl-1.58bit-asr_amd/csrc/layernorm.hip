// layernorm.hip — LayerNorm over the last dim for the Conformer's LN wrappers
// (reference onebit_asr/conformer.py:19-24 ``LayerNorm`` = nn.LayerNorm(d), eps 1e-5, used
// before every BitLinear call site: ff1/ff2 (:36), mhsa (:109), conv (:145), block out (:228)).
//
// At Conformer-S the three stacked passes normalise 23,904 rows of d = 144 per call, ~90
// calls per step. torch's kernels reach ~1 TB/s on these short rows (one block per row
// forward; three kernels backward). Here:
//   forward : 16 lanes per row (lane j holds columns j, j+16, ...: 64-byte coalesced
//             segments), the row's values stay in registers for a two-pass mean/variance;
//             writes y and the per-row (mean, rstd) the backward needs;
//   backward: the same row mapping; dx in one pass over (dy, x); dgamma/dbeta are
//             accumulated per lane over the block's rows and written as per-block
//             partials, summed over blocks in fixed order by a second launch
//             (deterministic, no atomics); optionally a second output dy2 = the
//             consumer's dropout/pad/scale backward of dx (GScale below), so the
//             residual-dropout backward of the module feeding this LN needs no pass
//             of its own.
// Numerics: var = mean((x - mean)^2) (biased, as torch), rstd = 1/sqrt(var + eps).
#include <cstdlib>

#include "ob_drop.h"
#include "ob_fp.h"
#include "ob_launch.h"
#include "ob_ln.h"

namespace ob {

namespace {

constexpr int kThreads = 256;
constexpr int kLanesPerRow = lnrow::kLanesPerRow;
constexpr int kRowsPerBlock = kThreads / kLanesPerRow;  // 16

using lnrow::load_cols;
using lnrow::ln_row_v;
using lnrow::row_sum16;
using lnrow::store_cols;

// One row (16 lanes): y = LN(x) and the row's (mean, rstd); returns this lane's max|y|.
// y == nullptr: no fp32 store; yq != nullptr: also the int8 image of y at scale sx.
// this lane's columns of one row (the loads of ln_row, separable so that a thread can have
// several rows in flight before it reduces the first)
template <int NPL, int VW>
__device__ __forceinline__ void ln_load(const float* __restrict__ x, int64_t row, int d,
                                        float (&v)[NPL][VW]) {
  const int j = threadIdx.x & (kLanesPerRow - 1);
  const float* xr = x + row * d;
#pragma unroll
  for (int i = 0; i < NPL; ++i) load_cols<VW>(xr, VW * (j + kLanesPerRow * i), d, v[i]);
}


template <int NPL, int VW = 1>
__device__ __forceinline__ float ln_row(const float* __restrict__ x,
                                        const float* __restrict__ gamma,
                                        const float* __restrict__ beta, int64_t row, int d,
                                        float eps, float* __restrict__ y,
                                        float* __restrict__ mean_out,
                                        float* __restrict__ rstd_out,
                                        int8_t* __restrict__ yq = nullptr, float sx = 0.0f) {
  float v[NPL][VW];
  ln_load<NPL, VW>(x, row, d, v);
  return ln_row_v<NPL, VW>(v, gamma, beta, row, d, eps, y, mean_out, rstd_out, yq, sx);
}

// RPT rows per 16-lane group (rows sub, sub + 16, ... of the block's 16 * RPT): every row's
// loads are issued before the first row is reduced (RPT x the bytes in flight per wave).
// Measured at d = 144 (tools/ln_bench.py): RPT 2 / 4 are slower (7.1 / 9.5 us vs 6.3 us), so
// the default stays 1; OB_LN_RPT keeps the others for other widths.
template <int NPL, int VW, int RPT>  // columns per lane: d <= 16 * NPL * VW
__global__ __launch_bounds__(kThreads) void ln_fwd_kernel(
    const float* __restrict__ x, const float* __restrict__ gamma, const float* __restrict__ beta,
    int64_t rows, int d, float eps, float* __restrict__ y, float* __restrict__ mean_out,
    float* __restrict__ rstd_out) {
  const int64_t row0 = (int64_t)blockIdx.x * (kRowsPerBlock * RPT) + (threadIdx.x / kLanesPerRow);
  if constexpr (RPT == 1) {
    if (row0 < rows) (void)ln_row<NPL, VW>(x, gamma, beta, row0, d, eps, y, mean_out, rstd_out);
    return;
  }
  float v[RPT][NPL][VW];
#pragma unroll
  for (int q = 0; q < RPT; ++q) {
    const int64_t row = row0 + kRowsPerBlock * q;
    ln_load<NPL, VW>(x, row < rows ? row : rows - 1, d, v[q]);
  }
#pragma unroll
  for (int q = 0; q < RPT; ++q) {
    const int64_t row = row0 + kRowsPerBlock * q;
    if (row < rows) (void)ln_row_v<NPL, VW>(v[q], gamma, beta, row, d, eps, y, mean_out, rstd_out);
  }
}

// Two LayerNorms back to back, y1 = LN1(x), y2 = LN2(y1) (a block's final LN and the next
// module's input LN, conformer.py:228 then :28): one pass over x, y1 never re-read; the
// per-row arithmetic is ln_row's (y1 is normalised from the registers it is stored from), so
// y1 / y2 / the statistics equal two ln_fwd launches bit for bit.
template <int NPL, int VW>
__global__ __launch_bounds__(kThreads) void ln_fwd_pair_kernel(
    const float* __restrict__ x, const float* __restrict__ g1, const float* __restrict__ b1,
    const float* __restrict__ g2, const float* __restrict__ b2, int64_t rows, int d, float eps1,
    float eps2, float* __restrict__ y1, float* __restrict__ mean1, float* __restrict__ rstd1,
    float* __restrict__ y2, float* __restrict__ mean2, float* __restrict__ rstd2) {
  const int64_t row = (int64_t)blockIdx.x * kRowsPerBlock + (threadIdx.x / kLanesPerRow);
  if (row >= rows) return;
  float v[NPL][VW];
  ln_load<NPL, VW>(x, row, d, v);
  (void)ln_row_v<NPL, VW>(v, g1, b1, row, d, eps1, y1, mean1, rstd1, nullptr, 0.0f, &v);
  (void)ln_row_v<NPL, VW>(v, g2, b2, row, d, eps2, y2, mean2, rstd2);
}

// The same rows plus the per-pass max|y| (the int8 activation scale of the BitLinear that
// consumes y; passes = consecutive blocks of rows_per_pass rows). Blocks stride over the
// rows; each keeps per-pass maxima in LDS (ds_max on the fp32 bit patterns: |y| >= 0 so
// the unsigned order is the float order) and writes them as partials part[p][block]; a
// one-wave launch reduces them (no same-address atomics: 1024 of those cost 10 us here).
// Max is order-independent: deterministic.
constexpr int kAmaxMaxPasses = 8;
template <int NPL, int VW>
__global__ __launch_bounds__(kThreads) void ln_fwd_amax_kernel(
    const float* __restrict__ x, const float* __restrict__ gamma, const float* __restrict__ beta,
    int64_t rows, int d, float eps, float* __restrict__ y, float* __restrict__ mean_out,
    float* __restrict__ rstd_out, int64_t rows_per_pass, int P, uint32_t* __restrict__ part) {
  __shared__ uint32_t smax[kAmaxMaxPasses];
  if (threadIdx.x < kAmaxMaxPasses) smax[threadIdx.x] = 0u;
  __syncthreads();
  for (int64_t r0 = (int64_t)blockIdx.x * kRowsPerBlock; r0 < rows;
       r0 += (int64_t)gridDim.x * kRowsPerBlock) {
    const int64_t row = r0 + (threadIdx.x / kLanesPerRow);
    if (row < rows) {
      float m = ln_row<NPL, VW>(x, gamma, beta, row, d, eps, y, mean_out, rstd_out);
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
      if ((threadIdx.x & (kLanesPerRow - 1)) == 0)
        atomicMax(&smax[(int)(row / rows_per_pass)], __float_as_uint(m));
    }
  }
  __syncthreads();
  if ((int)threadIdx.x < P) part[(int64_t)threadIdx.x * gridDim.x + blockIdx.x] = smax[threadIdx.x];
}

__global__ __launch_bounds__(kThreads) void ln_amax_final_kernel(
    const uint32_t* __restrict__ part, int nparts, uint32_t* __restrict__ amax) {
  __shared__ uint32_t red[kThreads / 64];
  const int p = blockIdx.x;
  const uint32_t* src = part + (int64_t)p * nparts;
  uint32_t m[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // 8 independent loads in flight per thread
  for (int i0 = 0; i0 < nparts; i0 += 8 * kThreads) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = i0 + u * kThreads + threadIdx.x;
      if (i < nparts) m[u] = max(m[u], src[i]);
    }
  }
  uint32_t v = max(max(max(m[0], m[1]), max(m[2], m[3])), max(max(m[4], m[5]), max(m[6], m[7])));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) amax[p] = max(max(red[0], red[1]), max(red[2], red[3]));
}

constexpr int kAmaxBlocks = 2048;

// The int8 image of LN(x) for an int8 consumer: the rows are normalised again (the same
// ln_row arithmetic as the absmax pass, so the same y) and quantised at the pass's scale
// sx = 127 / max(amax[p], 1e-5) -- exactly the quantisation tgemm_i8 applies in registers
// to an fp32 operand, so the int8-operand GEMM is bit-identical to that path.
template <int NPL, int VW>
__global__ __launch_bounds__(kThreads) void ln_fwd_q8_kernel(
    const float* __restrict__ x, const float* __restrict__ gamma, const float* __restrict__ beta,
    int64_t rows, int d, float eps, int64_t rows_per_pass, const float* __restrict__ amax,
    int8_t* __restrict__ yq) {
  const int64_t row = (int64_t)blockIdx.x * kRowsPerBlock + (threadIdx.x / kLanesPerRow);
  if (row >= rows) return;
  const float sx = 127.0f / fmaxf(amax[(int)(row / rows_per_pass)], 1e-5f);
  (void)ln_row<NPL, VW>(x, gamma, beta, row, d, eps, nullptr, nullptr, nullptr, yq, sx);
}

// The backward of a residual junction's "R + rscale * rowvalid * drop(y)" applied to this
// LN's dx (the junction's output gradient): dy2 = rscale * rowvalid * keep * scale * dx,
// element for element what drop_scale_bwd_kernel (fused.hip) computes from dx.
struct GScale {
  float* dy2;  // nullptr: off
  float rscale;
  DropCfg dc;
  const uint64_t* rng;
  uint64_t rng_off;
  const int* lens;
  int T;
};

// dx = rstd * (g - mean(g) - xhat * mean(g * xhat)),  g = dy * gamma
template <int NPL, int VW>
__global__ __launch_bounds__(kThreads) void ln_bwd_kernel(
    const float* __restrict__ dy, const float* __restrict__ x, const float* __restrict__ gamma,
    const float* __restrict__ mean_in, const float* __restrict__ rstd_in, int64_t rows, int d,
    int rows_per_block, const float* __restrict__ dres, float* __restrict__ dx,
    float* __restrict__ part_g, float* __restrict__ part_b, GScale gs, LnDefer df,
    LnParamEntry ent) {
  __shared__ float red_g[kRowsPerBlock][kLanesPerRow * NPL * VW];
  __shared__ float red_b[kRowsPerBlock][kLanesPerRow * NPL * VW];
  if (df.table && blockIdx.x == 0 && threadIdx.x == 0) df.table[df.slot] = ent;
  const int j = threadIdx.x & (kLanesPerRow - 1);
  const int sub = threadIdx.x / kLanesPerRow;
  const float inv_d = 1.0f / (float)d;
  float gam[NPL][VW], acc_g[NPL][VW], acc_b[NPL][VW];
#pragma unroll
  for (int i = 0; i < NPL; ++i) {
    const int c0 = VW * (j + kLanesPerRow * i);
    if (gamma) load_cols<VW>(gamma, c0, d, gam[i]);
#pragma unroll
    for (int e = 0; e < VW; ++e) {
      if (!gamma) gam[i][e] = c0 + e < d ? 1.0f : 0.0f;
      acc_g[i][e] = 0.0f;
      acc_b[i][e] = 0.0f;
    }
  }
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(rows, r0 + rows_per_block);
  const uint32_t dkey = (gs.dy2 && gs.dc.on) ? drop_key(gs.rng[0], gs.rng[1] + gs.rng_off) : 0u;
  // The next row's operands (mean, rstd, x, dy, dres) are loaded before this row is
  // reduced: two rows in flight per 16-lane group (the kernel is latency-bound otherwise).
  struct RowIn {
    float mu, rs;
    float xv[NPL][VW], dv[NPL][VW], res[NPL][VW];
  };
  auto fetch = [&](int64_t row, RowIn& in) {
    in.mu = mean_in[row];
    in.rs = rstd_in[row];
    if (dres) {
#pragma unroll
      for (int i = 0; i < NPL; ++i) load_cols<VW>(dres + row * d, VW * (j + kLanesPerRow * i), d, in.res[i]);
    }
#pragma unroll
    for (int i = 0; i < NPL; ++i) {
      const int c0 = VW * (j + kLanesPerRow * i);
      load_cols<VW>(x + row * d, c0, d, in.xv[i]);
      load_cols<VW>(dy + row * d, c0, d, in.dv[i]);
    }
  };
  RowIn cur, nxt;
  if (r0 + sub < r1) fetch(r0 + sub, cur);
  for (int64_t row = r0 + sub; row < r1; row += kRowsPerBlock) {
    if (row + kRowsPerBlock < r1) fetch(row + kRowsPerBlock, nxt);
    const float mu = cur.mu, rs = cur.rs;
    float xh[NPL][VW], g[NPL][VW];
    const float (&res)[NPL][VW] = cur.res;
    float s1 = 0.0f, s2 = 0.0f;
    const bool rr = dres != nullptr;
#pragma unroll
    for (int i = 0; i < NPL; ++i) {
      const float (&xv)[VW] = cur.xv[i];
      const float (&dv)[VW] = cur.dv[i];
#pragma unroll
      for (int e = 0; e < VW; ++e) {
        xh[i][e] = (xv[e] - mu) * rs;
        acc_g[i][e] = fmaf(dv[e], xh[i][e], acc_g[i][e]);
        acc_b[i][e] += dv[e];
        g[i][e] = dv[e] * gam[i][e];
        s1 += g[i][e];
        s2 = fmaf(g[i][e], xh[i][e], s2);
      }
    }
    const float m1 = row_sum16(s1) * inv_d;
    const float m2 = row_sum16(s2) * inv_d;
    float* dr = dx + row * d;
    bool rvalid = true;
    if (gs.dy2 && gs.lens) {
      const int64_t b = row / gs.T;
      rvalid = row - b * gs.T < gs.lens[b];
    }
#pragma unroll
    for (int i = 0; i < NPL; ++i) {
      const int c0 = VW * (j + kLanesPerRow * i);
      if (c0 < d) {
        float o[VW], w2[VW];
#pragma unroll
        for (int e = 0; e < VW; ++e) {
          // explicit roundings: identical with and without dres (hipcc may contract the
          // two loop versions differently otherwise)
          const float v = nc_mul(rs, nc_sub(nc_sub(g[i][e], m1), nc_mul(xh[i][e], m2)));
          // + the residual branch's gradient (the add autograd would do), not contracted
          o[e] = rr ? nc_add(v, res[i][e]) : v;
          // the same operation sequence as drop_scale_bwd_kernel
          float w = o[e];
          if (gs.dc.on)
            w = nc_mul(w, drop_keep(dkey, (uint64_t)(row * d + c0 + e), gs.dc.thresh) ? gs.dc.scale : 0.0f);
          if (!rvalid) w = nc_mul(w, 0.0f);
          w2[e] = gs.rscale == 1.0f ? w : nc_mul(gs.rscale, w);
        }
        store_cols<VW>(dr, c0, o);
        if (gs.dy2) store_cols<VW>(gs.dy2 + row * d, c0, w2);
      }
    }
    cur = nxt;
  }
  if (!part_g) return;
#pragma unroll
  for (int i = 0; i < NPL; ++i)
#pragma unroll
    for (int e = 0; e < VW; ++e) {
      red_g[sub][VW * (j + kLanesPerRow * i) + e] = acc_g[i][e];
      red_b[sub][VW * (j + kLanesPerRow * i) + e] = acc_b[i][e];
    }
  __syncthreads();
  for (int c = threadIdx.x; c < d; c += kThreads) {
    float sg = 0.0f, sb = 0.0f;
#pragma unroll
    for (int r = 0; r < kRowsPerBlock; ++r) {
      sg += red_g[r][c];
      sb += red_b[r][c];
    }
    part_g[(int64_t)blockIdx.x * d + c] = sg;
    part_b[(int64_t)blockIdx.x * d + c] = sb;
  }
}

// One LayerNorm backward row stage (ln_bwd_kernel's arithmetic): dx = rstd * (g - mean(g) -
// xhat * mean(g * xhat)) (+ res), g = dy * gamma, and the dgamma / dbeta accumulators;
// columns >= d give 0.
template <int NPL, int VW>
__device__ __forceinline__ void ln_bwd_stage(const float (&xv)[NPL][VW], const float (&dv)[NPL][VW],
                                             const float (*res)[NPL][VW], float mu, float rs,
                                             const float (&gam)[NPL][VW], float inv_d, int d,
                                             float (&acc_g)[NPL][VW], float (&acc_b)[NPL][VW],
                                             float (&o)[NPL][VW]) {
  const int j = threadIdx.x & (kLanesPerRow - 1);
  float xh[NPL][VW], g[NPL][VW];
  float s1 = 0.0f, s2 = 0.0f;
#pragma unroll
  for (int i = 0; i < NPL; ++i)
#pragma unroll
    for (int e = 0; e < VW; ++e) {
      xh[i][e] = (xv[i][e] - mu) * rs;
      acc_g[i][e] = fmaf(dv[i][e], xh[i][e], acc_g[i][e]);
      acc_b[i][e] += dv[i][e];
      g[i][e] = dv[i][e] * gam[i][e];
      s1 += g[i][e];
      s2 = fmaf(g[i][e], xh[i][e], s2);
    }
  const float m1 = row_sum16(s1) * inv_d;
  const float m2 = row_sum16(s2) * inv_d;
#pragma unroll
  for (int i = 0; i < NPL; ++i)
#pragma unroll
    for (int e = 0; e < VW; ++e) {
      const float v = nc_mul(rs, nc_sub(nc_sub(g[i][e], m1), nc_mul(xh[i][e], m2)));
      const bool live = VW * (j + kLanesPerRow * i) + e < d;
      o[i][e] = live ? (res ? nc_add(v, (*res)[i][e]) : v) : 0.0f;
    }
}

// The backward of a LayerNorm pair (y1 = LN1(x), y2 = LN2(y1), y1 also taken by a residual
// branch whose gradient is gres): g = LN2_backward(dy) + gres and dx = LN1_backward(g) (with
// the dy2 of the residual tail feeding x, as ln_bwd_kernel), in one pass per row -- g never
// goes to memory; both layers' dgamma / dbeta partials (part_*2 for LN2, part_*1 for LN1,
// the same row blocks as ln_bwd_kernel).
template <int NPL, int VW>
__global__ __launch_bounds__(kThreads) void ln_bwd_pair_kernel(
    const float* __restrict__ dy, const float* __restrict__ y1, const float* __restrict__ g2,
    const float* __restrict__ mean2, const float* __restrict__ rstd2,
    const float* __restrict__ gres, const float* __restrict__ x, const float* __restrict__ g1,
    const float* __restrict__ mean1, const float* __restrict__ rstd1, int64_t rows, int d,
    int rows_per_block, float* __restrict__ dx, float* __restrict__ pg2, float* __restrict__ pb2,
    float* __restrict__ pg1, float* __restrict__ pb1, GScale gs, LnDefer df2, LnParamEntry ent2,
    LnDefer df1, LnParamEntry ent1) {
  __shared__ float red[2][kRowsPerBlock][kLanesPerRow * NPL * VW];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (df2.table) df2.table[df2.slot] = ent2;
    if (df1.table) df1.table[df1.slot] = ent1;
  }
  const int j = threadIdx.x & (kLanesPerRow - 1);
  const int sub = threadIdx.x / kLanesPerRow;
  const float inv_d = 1.0f / (float)d;
  float gm2[NPL][VW], gm1[NPL][VW], ag2[NPL][VW], ab2[NPL][VW], ag1[NPL][VW], ab1[NPL][VW];
#pragma unroll
  for (int i = 0; i < NPL; ++i) {
    const int c0 = VW * (j + kLanesPerRow * i);
    if (g2) load_cols<VW>(g2, c0, d, gm2[i]);
    if (g1) load_cols<VW>(g1, c0, d, gm1[i]);
#pragma unroll
    for (int e = 0; e < VW; ++e) {
      if (!g2) gm2[i][e] = c0 + e < d ? 1.0f : 0.0f;
      if (!g1) gm1[i][e] = c0 + e < d ? 1.0f : 0.0f;
      ag2[i][e] = ab2[i][e] = ag1[i][e] = ab1[i][e] = 0.0f;
    }
  }
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(rows, r0 + rows_per_block);
  const uint32_t dkey = (gs.dy2 && gs.dc.on) ? drop_key(gs.rng[0], gs.rng[1] + gs.rng_off) : 0u;
  // the next row's operands load while this row is reduced (as ln_bwd_kernel)
  struct RowIn {
    float mu2, rs2, mu1, rs1;
    float yv[NPL][VW], dv[NPL][VW], rv[NPL][VW], xv[NPL][VW];
  };
  auto fetch = [&](int64_t row, RowIn& in) {
    in.mu2 = mean2[row];
    in.rs2 = rstd2[row];
    in.mu1 = mean1[row];
    in.rs1 = rstd1[row];
#pragma unroll
    for (int i = 0; i < NPL; ++i) {
      const int c0 = VW * (j + kLanesPerRow * i);
      load_cols<VW>(y1 + row * d, c0, d, in.yv[i]);
      load_cols<VW>(dy + row * d, c0, d, in.dv[i]);
      if (gres) load_cols<VW>(gres + row * d, c0, d, in.rv[i]);
      load_cols<VW>(x + row * d, c0, d, in.xv[i]);
    }
  };
  RowIn cur, nxt;
  if (r0 + sub < r1) fetch(r0 + sub, cur);
  for (int64_t row = r0 + sub; row < r1; row += kRowsPerBlock) {
    if (row + kRowsPerBlock < r1) fetch(row + kRowsPerBlock, nxt);
    float gv[NPL][VW], o[NPL][VW];
    ln_bwd_stage<NPL, VW>(cur.yv, cur.dv, gres ? &cur.rv : nullptr, cur.mu2, cur.rs2, gm2, inv_d,
                          d, ag2, ab2, gv);
    ln_bwd_stage<NPL, VW>(cur.xv, gv, nullptr, cur.mu1, cur.rs1, gm1, inv_d, d, ag1, ab1, o);
    bool rvalid = true;
    if (gs.dy2 && gs.lens) {
      const int64_t b = row / gs.T;
      rvalid = row - b * gs.T < gs.lens[b];
    }
#pragma unroll
    for (int i = 0; i < NPL; ++i) {
      const int c0 = VW * (j + kLanesPerRow * i);
      if (c0 < d) {
        float w2[VW];
#pragma unroll
        for (int e = 0; e < VW; ++e) {
          float w = o[i][e];
          if (gs.dc.on)
            w = nc_mul(w, drop_keep(dkey, (uint64_t)(row * d + c0 + e), gs.dc.thresh) ? gs.dc.scale : 0.0f);
          if (!rvalid) w = nc_mul(w, 0.0f);
          w2[e] = gs.rscale == 1.0f ? w : nc_mul(gs.rscale, w);
        }
        store_cols<VW>(dx + row * d, c0, o[i]);
        if (gs.dy2) store_cols<VW>(gs.dy2 + row * d, c0, w2);
      }
    }
    cur = nxt;
  }
  // the two layers' partials in turn through one [2][16][cols] LDS buffer
#pragma unroll
  for (int layer = 0; layer < 2; ++layer) {
    float* og = layer == 0 ? pg2 : pg1;
    float* ob = layer == 0 ? pb2 : pb1;
    if (layer == 1) __syncthreads();  // layer 0's reads are done
#pragma unroll
    for (int i = 0; i < NPL; ++i)
#pragma unroll
      for (int e = 0; e < VW; ++e) {
        const int c = VW * (j + kLanesPerRow * i) + e;
        red[0][sub][c] = layer == 0 ? ag2[i][e] : ag1[i][e];
        red[1][sub][c] = layer == 0 ? ab2[i][e] : ab1[i][e];
      }
    __syncthreads();
    if (og)
      for (int c = threadIdx.x; c < d; c += kThreads) {
        float sg = 0.0f, sb = 0.0f;
#pragma unroll
        for (int r = 0; r < kRowsPerBlock; ++r) {
          sg += red[0][r][c];
          sb += red[1][r][c];
        }
        og[(int64_t)blockIdx.x * d + c] = sg;
        ob[(int64_t)blockIdx.x * d + c] = sb;
      }
  }
}

// dgamma[c] = sum over blocks of part_g[blk][c], same for dbeta. Block = 4 columns x 64
// block-slices; slice s sums blocks s, s+64, ... (4 independent accumulators in flight),
// then the 64 slices are added in slice order through LDS (fixed order: deterministic).
// (16 columns x 16 slices: 9 blocks at d = 144, each thread a 32-load chain, 5.8 us.)
constexpr int kRedCols = 4, kRedSlices = kThreads / kRedCols;

__global__ __launch_bounds__(kThreads) void ln_param_reduce_kernel(
    const float* __restrict__ part_g, const float* __restrict__ part_b, int nblk, int d,
    float* __restrict__ dgamma, float* __restrict__ dbeta) {
  __shared__ float sg[kRedSlices][kRedCols], sb[kRedSlices][kRedCols];
  const int cl = threadIdx.x % kRedCols, sl = threadIdx.x / kRedCols;
  const int c = blockIdx.x * kRedCols + cl;
  float ag = 0.0f, ab = 0.0f;
  if (c < d) {
    float g4[4] = {0.f, 0.f, 0.f, 0.f}, b4[4] = {0.f, 0.f, 0.f, 0.f};
    int b = sl;
    for (; b + 3 * kRedSlices < nblk; b += 4 * kRedSlices) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        g4[u] += part_g[(int64_t)(b + u * kRedSlices) * d + c];
        b4[u] += part_b[(int64_t)(b + u * kRedSlices) * d + c];
      }
    }
    for (int u = 0; b < nblk; b += kRedSlices, ++u) {
      g4[u & 3] += part_g[(int64_t)b * d + c];
      b4[u & 3] += part_b[(int64_t)b * d + c];
    }
    ag = (g4[0] + g4[1]) + (g4[2] + g4[3]);
    ab = (b4[0] + b4[1]) + (b4[2] + b4[3]);
  }
  sg[sl][cl] = ag;
  sb[sl][cl] = ab;
  __syncthreads();
  if (sl == 0 && c < d) {
    float tg = 0.0f, tb = 0.0f;
#pragma unroll
    for (int q = 0; q < kRedSlices; ++q) {
      tg += sg[q][cl];
      tb += sb[q][cl];
    }
    if (dgamma) dgamma[c] = tg;
    if (dbeta) dbeta[c] = tb;
  }
}

// Every deferred LN parameter reduction of a backward in one launch: grid (column groups of
// 4, entries); the same fixed-order arithmetic as ln_param_reduce_kernel per entry.
__global__ __launch_bounds__(kThreads) void ln_param_table_kernel(
    const LnParamEntry* __restrict__ tab) {
  const LnParamEntry e = tab[blockIdx.y];
  if ((int)blockIdx.x * kRedCols >= e.d) return;
  __shared__ float sg[kRedSlices][kRedCols], sb[kRedSlices][kRedCols];
  const int cl = threadIdx.x % kRedCols, sl = threadIdx.x / kRedCols;
  const int c = blockIdx.x * kRedCols + cl;
  const int d = e.d, nblk = e.nblk;
  float ag = 0.0f, ab = 0.0f;
  if (c < d) {
    float g4[4] = {0.f, 0.f, 0.f, 0.f}, b4[4] = {0.f, 0.f, 0.f, 0.f};
    int b = sl;
    for (; b + 3 * kRedSlices < nblk; b += 4 * kRedSlices) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        g4[u] += e.part_g[(int64_t)(b + u * kRedSlices) * d + c];
        b4[u] += e.part_b[(int64_t)(b + u * kRedSlices) * d + c];
      }
    }
    for (int u = 0; b < nblk; b += kRedSlices, ++u) {
      g4[u & 3] += e.part_g[(int64_t)b * d + c];
      b4[u & 3] += e.part_b[(int64_t)b * d + c];
    }
    ag = (g4[0] + g4[1]) + (g4[2] + g4[3]);
    ab = (b4[0] + b4[1]) + (b4[2] + b4[3]);
  }
  sg[sl][cl] = ag;
  sb[sl][cl] = ab;
  __syncthreads();
  if (sl == 0 && c < d) {
    float tg = 0.0f, tb = 0.0f;
#pragma unroll
    for (int q = 0; q < kRedSlices; ++q) {
      tg += sg[q][cl];
      tb += sb[q][cl];
    }
    if (e.dgamma) e.dgamma[c] = tg;
    if (e.dbeta) e.dbeta[c] = tb;
  }
}

// launch shapes measured in round 3 (profiles/r3/ln/): 512 backward blocks, one row per
// 16-lane group in the forward
int max_bwd_blocks() { return 512; }
int fwd_rows_per_group() { return 1; }

int bwd_blocks(int64_t rows, int* rows_per_block) {
  int64_t nb = ceil_div(rows, kRowsPerBlock);
  if (nb > max_bwd_blocks()) nb = max_bwd_blocks();
  if (nb < 1) nb = 1;
  int64_t rpb = ceil_div(rows, nb);
  rpb = ceil_div(rpb, kRowsPerBlock) * kRowsPerBlock;
  *rows_per_block = (int)rpb;
  return (int)ceil_div(rows, rpb);
}

}  // namespace

bool layernorm_supported(int64_t d) { return d >= 1 && d <= 16 * 32; }

size_t layernorm_bwd_workspace(int64_t rows, int64_t d) {
  int rpb;
  const int nb = rows > 0 ? bwd_blocks(rows, &rpb) : 1;
  return sizeof(float) * (size_t)(2 * nb * d) + 256;
}

#define OB_LN_NPL(MACRO) \
  if (npl <= 4) MACRO(4) else if (npl <= 9) MACRO(9) else if (npl <= 16) MACRO(16) \
  else MACRO(32)
// 4-column slots (d % 4 == 0, 16-byte aligned operands): d <= 64 * NPL
#define OB_LN_NPL4(MACRO) \
  if (npl4 <= 1) MACRO(1) else if (npl4 <= 2) MACRO(2) else if (npl4 <= 3) MACRO(3) \
  else if (npl4 <= 4) MACRO(4) else MACRO(8)

inline bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

void launch_layernorm_fwd(const float* x, const float* gamma, const float* beta, int64_t rows,
                          int64_t d, float eps, float* y, float* mean, float* rstd,
                          hipStream_t s) {
  if (rows == 0) return;
  const int npl = (int)ceil_div(d, kLanesPerRow);
  const int npl4 = (int)ceil_div(d, 4 * kLanesPerRow);
  const dim3 grid((unsigned)ceil_div(rows, kRowsPerBlock));
  const bool vec = d % 4 == 0 && al16(x) && al16(y) && al16(gamma) && al16(beta);
  const int rpt = fwd_rows_per_group();
  const dim3 grid_r((unsigned)ceil_div(rows, kRowsPerBlock * rpt));
#define OB_LNF(N)                                                                                \
  hipLaunchKernelGGL((ln_fwd_kernel<N, 1, 1>), grid, dim3(kThreads), 0, s, x, gamma, beta, rows, \
                     (int)d, eps, y, mean, rstd);
#define OB_LNF4R(N, R)                                                                           \
  hipLaunchKernelGGL((ln_fwd_kernel<N, 4, R>), grid_r, dim3(kThreads), 0, s, x, gamma, beta,     \
                     rows, (int)d, eps, y, mean, rstd);
#define OB_LNF4(N)                                                   \
  if (rpt == 4) { OB_LNF4R(N, 4) } else if (rpt == 2) { OB_LNF4R(N, 2) } \
  else { OB_LNF4R(N, 1) }
  if (vec) {
    OB_LN_NPL4(OB_LNF4)
  } else {
    OB_LN_NPL(OB_LNF)
  }
#undef OB_LNF
#undef OB_LNF4
#undef OB_LNF4R
}

void launch_layernorm_fwd_pair(const float* x, const float* g1, const float* b1, const float* g2,
                               const float* b2, int64_t rows, int64_t d, float eps1, float eps2,
                               float* y1, float* mean1, float* rstd1, float* y2, float* mean2,
                               float* rstd2, hipStream_t s) {
  if (rows == 0) return;
  const int npl = (int)ceil_div(d, kLanesPerRow);
  const int npl4 = (int)ceil_div(d, 4 * kLanesPerRow);
  const dim3 grid((unsigned)ceil_div(rows, kRowsPerBlock));
  const bool vec = d % 4 == 0 && al16(x) && al16(y1) && al16(y2) && al16(g1) && al16(b1) &&
                   al16(g2) && al16(b2);
#define OB_LNP(N)                                                                                \
  hipLaunchKernelGGL((ln_fwd_pair_kernel<N, 1>), grid, dim3(kThreads), 0, s, x, g1, b1, g2, b2,  \
                     rows, (int)d, eps1, eps2, y1, mean1, rstd1, y2, mean2, rstd2);
#define OB_LNP4(N)                                                                               \
  hipLaunchKernelGGL((ln_fwd_pair_kernel<N, 4>), grid, dim3(kThreads), 0, s, x, g1, b1, g2, b2,  \
                     rows, (int)d, eps1, eps2, y1, mean1, rstd1, y2, mean2, rstd2);
  if (vec) {
    OB_LN_NPL4(OB_LNP4)
  } else {
    OB_LN_NPL(OB_LNP)
  }
#undef OB_LNP
#undef OB_LNP4
}

size_t layernorm_fwd_amax_workspace(int64_t P) {
  return sizeof(uint32_t) * (size_t)P * kAmaxBlocks;
}

void launch_layernorm_fwd_amax(const float* x, const float* gamma, const float* beta,
                               int64_t rows, int64_t d, float eps, float* y, float* mean,
                               float* rstd, int P, float* amax, void* ws, hipStream_t s) {
  if (rows == 0) {
    launch_zero_words(amax, P, s);
    return;
  }
  const int npl = (int)ceil_div(d, kLanesPerRow);
  int64_t nb = ceil_div(rows, kRowsPerBlock);
  if (nb > kAmaxBlocks) nb = kAmaxBlocks;
  const int64_t rpp = rows / P;
  uint32_t* part = static_cast<uint32_t*>(ws);
  // (the same column slots as launch_layernorm_fwd: y bit-identical to the plain forward)
  const int npl4 = (int)ceil_div(d, 4 * kLanesPerRow);
  const bool vec = d % 4 == 0 && al16(x) && al16(y) && al16(gamma) && al16(beta);
#define OB_LNFA(N)                                                                              \
  hipLaunchKernelGGL((ln_fwd_amax_kernel<N, 1>), dim3((unsigned)nb), dim3(kThreads), 0, s, x,    \
                     gamma, beta, rows, (int)d, eps, y, mean, rstd, rpp, P, part);
#define OB_LNFA4(N)                                                                             \
  hipLaunchKernelGGL((ln_fwd_amax_kernel<N, 4>), dim3((unsigned)nb), dim3(kThreads), 0, s, x,    \
                     gamma, beta, rows, (int)d, eps, y, mean, rstd, rpp, P, part);
  if (vec) {
    OB_LN_NPL4(OB_LNFA4)
  } else {
    OB_LN_NPL(OB_LNFA)
  }
#undef OB_LNFA
#undef OB_LNFA4
  hipLaunchKernelGGL(ln_amax_final_kernel, dim3((unsigned)P), dim3(kThreads), 0, s,
                     (const uint32_t*)part, (int)nb, reinterpret_cast<uint32_t*>(amax));
}

void launch_layernorm_fwd_i8(const float* x, const float* gamma, const float* beta, int64_t rows,
                             int64_t d, float eps, int P, float* amax, int8_t* yq, void* ws,
                             hipStream_t s) {
  // pass 1: per-pass max|LN(x)| (no y store); pass 2: LN(x) again, quantised
  launch_layernorm_fwd_amax(x, gamma, beta, rows, d, eps, nullptr, nullptr, nullptr, P, amax, ws,
                            s);
  if (rows == 0) return;
  const int npl = (int)ceil_div(d, kLanesPerRow);
  const int npl4 = (int)ceil_div(d, 4 * kLanesPerRow);
  const int64_t rpp = rows / P;
  const dim3 grid((unsigned)ceil_div(rows, kRowsPerBlock));
  // the same column slots (hence the same summation order) as the absmax pass, whose y is
  // nullptr; yq is 4-byte aligned (checked by the C ABI), so a 4-column slot is one dword
  const bool vec = d % 4 == 0 && al16(x) && al16(gamma) && al16(beta);
#define OB_LNQ(N)                                                                                \
  hipLaunchKernelGGL((ln_fwd_q8_kernel<N, 1>), grid, dim3(kThreads), 0, s, x, gamma, beta, rows, \
                     (int)d, eps, rpp, (const float*)amax, yq);
#define OB_LNQ4(N)                                                                               \
  hipLaunchKernelGGL((ln_fwd_q8_kernel<N, 4>), grid, dim3(kThreads), 0, s, x, gamma, beta, rows, \
                     (int)d, eps, rpp, (const float*)amax, yq);
  if (vec) {
    OB_LN_NPL4(OB_LNQ4)
  } else {
    OB_LN_NPL(OB_LNQ)
  }
#undef OB_LNQ
#undef OB_LNQ4
}

void launch_ln_param_table(const LnParamEntry* table, int n, int dmax, hipStream_t s) {
  if (n <= 0 || dmax <= 0) return;
  hipLaunchKernelGGL(ln_param_table_kernel, dim3((unsigned)ceil_div(dmax, kRedCols), (unsigned)n),
                     dim3(kThreads), 0, s, table);
}

void launch_layernorm_bwd_pair(const float* dy, const float* y1, const float* g2,
                               const float* mean2, const float* rstd2, const float* gres,
                               const float* x, const float* g1, const float* mean1,
                               const float* rstd1, int64_t rows, int64_t d, float* dx,
                               float* dg2, float* db2, float* dg1, float* db1, void* ws,
                               hipStream_t s, const LnGradScale* gsc, const LnDefer* defer2,
                               const LnDefer* defer1) {
  GScale gs{};
  if (gsc && gsc->dy2) {
    gs.dy2 = gsc->dy2;
    gs.rscale = gsc->rscale;
    gs.dc = make_drop(gsc->p_drop);
    gs.rng = gsc->rng;
    gs.rng_off = gsc->rng_off;
    gs.lens = gsc->lens;
    gs.T = gsc->T > 0 ? gsc->T : 1;
  }
  int rpb = kRowsPerBlock;
  const int nb = rows > 0 ? bwd_blocks(rows, &rpb) : 0;
  // ws: LN2's partials then LN1's, each layernorm_bwd_workspace's layout
  float* pg2 = static_cast<float*>(ws);
  float* pb2 = pg2 + (size_t)nb * d;
  float* pg1 = reinterpret_cast<float*>(static_cast<char*>(ws) + layernorm_bwd_workspace(rows, d));
  float* pb1 = pg1 + (size_t)nb * d;
  const bool p2 = dg2 || db2, p1 = dg1 || db1;
  LnDefer f2{nullptr, 0}, f1{nullptr, 0};
  if (defer2 && defer2->table && p2 && rows > 0) f2 = *defer2;
  if (defer1 && defer1->table && p1 && rows > 0) f1 = *defer1;
  const LnParamEntry e2{pg2, pb2, dg2, db2, nb, (int)d}, e1{pg1, pb1, dg1, db1, nb, (int)d};
  const int npl = (int)ceil_div(d, kLanesPerRow);
  const int npl4 = (int)ceil_div(d, 4 * kLanesPerRow);
  const bool vec = d % 4 == 0 && al16(dy) && al16(y1) && al16(g2) && al16(gres) && al16(x) &&
                   al16(g1) && al16(dx) && al16(gs.dy2);
  if (rows > 0) {
#define OB_LNBP(N, V)                                                                            \
  hipLaunchKernelGGL((ln_bwd_pair_kernel<N, V>), dim3((unsigned)nb), dim3(kThreads), 0, s, dy,   \
                     y1, g2, mean2, rstd2, gres, x, g1, mean1, rstd1, rows, (int)d, rpb, dx,     \
                     p2 ? pg2 : nullptr, p2 ? pb2 : nullptr, p1 ? pg1 : nullptr,                 \
                     p1 ? pb1 : nullptr, gs, f2, e2, f1, e1);
#define OB_LNBP1(N) OB_LNBP(N, 1)
#define OB_LNBP4(N) OB_LNBP(N, 4)
    if (vec) {
      OB_LN_NPL4(OB_LNBP4)
    } else {
      OB_LN_NPL(OB_LNBP1)
    }
#undef OB_LNBP1
#undef OB_LNBP4
#undef OB_LNBP
  }
  if (p2 && !f2.table)
    hipLaunchKernelGGL(ln_param_reduce_kernel, dim3((unsigned)ceil_div(d, kRedCols)), dim3(kThreads), 0,
                       s, pg2, pb2, nb, (int)d, dg2, db2);
  if (p1 && !f1.table)
    hipLaunchKernelGGL(ln_param_reduce_kernel, dim3((unsigned)ceil_div(d, kRedCols)), dim3(kThreads), 0,
                       s, pg1, pb1, nb, (int)d, dg1, db1);
}

void launch_layernorm_bwd(const float* dy, const float* x, const float* gamma, const float* mean,
                          const float* rstd, int64_t rows, int64_t d, const float* dres,
                          float* dx, float* dgamma, float* dbeta, void* ws, hipStream_t s,
                          const LnGradScale* gsc, const LnDefer* defer) {
  GScale gs{};
  if (gsc && gsc->dy2) {
    gs.dy2 = gsc->dy2;
    gs.rscale = gsc->rscale;
    gs.dc = make_drop(gsc->p_drop);
    gs.rng = gsc->rng;
    gs.rng_off = gsc->rng_off;
    gs.lens = gsc->lens;
    gs.T = gsc->T > 0 ? gsc->T : 1;
  }
  const int npl = (int)ceil_div(d, kLanesPerRow);
  float* part_g = static_cast<float*>(ws);
  int rpb = kRowsPerBlock;
  const int nb = rows > 0 ? bwd_blocks(rows, &rpb) : 0;
  float* part_b = part_g + (size_t)nb * d;
  const bool params = dgamma || dbeta;
  LnDefer df{nullptr, 0};
  if (defer && defer->table && params && rows > 0) df = *defer;
  const LnParamEntry ent{part_g, part_b, dgamma, dbeta, nb, (int)d};
  const int npl4 = (int)ceil_div(d, 4 * kLanesPerRow);
  const bool vec = d % 4 == 0 && al16(dy) && al16(x) && al16(gamma) && al16(dres) && al16(dx) &&
                   al16(gs.dy2);
  if (rows > 0) {
#define OB_LNB(N)                                                                              \
  hipLaunchKernelGGL((ln_bwd_kernel<N, 1>), dim3((unsigned)nb), dim3(kThreads), 0, s, dy, x, \
                     gamma, mean, rstd, rows, (int)d, rpb, dres, dx,                           \
                     params ? part_g : nullptr, part_b, gs, df, ent);
#define OB_LNB4(N)                                                                             \
  hipLaunchKernelGGL((ln_bwd_kernel<N, 4>), dim3((unsigned)nb), dim3(kThreads), 0, s, dy, x, \
                     gamma, mean, rstd, rows, (int)d, rpb, dres, dx,                           \
                     params ? part_g : nullptr, part_b, gs, df, ent);
    if (vec) {
      OB_LN_NPL4(OB_LNB4)
    } else {
      OB_LN_NPL(OB_LNB)
    }
#undef OB_LNB
#undef OB_LNB4
  }
  if (params && !df.table)
    hipLaunchKernelGGL(ln_param_reduce_kernel, dim3((unsigned)ceil_div(d, kRedCols)), dim3(kThreads), 0,
                       s, part_g, part_b, nb, (int)d, dgamma, dbeta);
}

}  // namespace ob
