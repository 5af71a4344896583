// convmod.hip — the Conformer conv module's elementwise/depthwise core, channels-last.
//
// Reference: onebit_asr/conformer.py:139-167 (full precision):
//   y = LN(x) -> [B,C,T] -> pw1 (1x1, C -> 2C) -> GLU(dim=C) -> depthwise k (pad k/2)
//     -> BatchNorm1d (batch statistics over B and T, padded frames included,
//        track_running_stats=False) -> swish -> pw2 (1x1) -> dropout -> [B,T,C];  x + y
// The reference transposes to [B,C,T] for nn.Conv1d. Here everything stays [rows, C]
// (rows = Bt*T, channel fastest): pw1 / pw2 are plain GEMMs on that layout (hipBLASLt,
// bias in its epilogue) and this file covers what lies between them:
//   forward   u [rows][2C] -> g = u[:, :C] * sigmoid(u[:, C:]) -> z = dw(g) + b_dw
//             -> per-(pass, channel) mean / rstd of z -> v = swish(BN(z))        (4 launches)
//   backward  dv -> dz (BN + swish backward, per-pass batch statistics) -> dg = dw^T(dz)
//             -> du (GLU backward); dw_dw, db_dw, dgamma, dbeta                   (6 launches)
// The forward keeps g (GLU output) and z for the backward.
// Stacked passes (P > 1, Bt = P*B): pass p's utterances are rows [p*B*T, (p+1)*B*T) and
// BatchNorm uses that pass's own statistics (each reference pass normalises its own batch);
// gamma / beta / the depthwise weights are shared, so their gradients sum over passes.
// Reductions are fixed-order (deterministic); statistics accumulate in fp64.
#include <math.h>

#include <cstdlib>

#include "ob_fp.h"
#include "ob_launch.h"

namespace ob {

namespace {

constexpr int kThreads = 256;
constexpr size_t kMaxLds = 160 * 1024;

// sigmoid through v_exp_f32 and v_rcp_f32 (a few ulp from torch's expf-based sigmoid, far
// inside the fused-vs-unfused bars of tests/test_convmod_gpu.py; the accurate expf and IEEE
// division were ~35 VALU ops per element, most of the depthwise tiles' arithmetic)
__device__ __forceinline__ float sigm(float x) { return fast_sigmoid(x); }  // ob_fp.h
// swish y * sigmoid(y)
__device__ __forceinline__ float swish(float y) { return y * sigm(y); }

// out[r] = sum_j wt[j] * tile[(tl0 + r + j) * C + c], r < R: one channel, R consecutive
// frames, the R + KT - 1 tile values held in registers (KT compile-time) -- 1 + (KT-1)/R LDS
// reads per output instead of 2 KT.
template <int KT, int R>
__device__ __forceinline__ void conv_window(const float* __restrict__ tile, int C, int c, int tl0,
                                            const float (&wt)[KT], float (&out)[R]) {
  float win[R + KT - 1];
#pragma unroll
  for (int i = 0; i < R + KT - 1; ++i) win[i] = tile[(tl0 + i) * C + c];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    float acc = 0.0f;
#pragma unroll
    for (int j = 0; j < KT; ++j) acc = fmaf(wt[j], win[r + j], acc);
    out[r] = acc;
  }
}

constexpr int kR = 8;  // frames per register window
constexpr int kLB = 16;  // window elements loaded per thread and batch (all in flight)
constexpr int kSB = 16;  // rows per batch of the per-channel statistics loops

// ------------------------------------------------------------------ forward
// Block = (time tile of TT frames, utterance). LDS holds g over [t0-P, t0+TT+P) x C and
// the depthwise weights; outputs z for the tile (consecutive threads = consecutive
// channels: coalesced global access, conflict-free LDS).
// KT > 0: the kernel width as a compile-time constant (register windows); KT == 0: generic.
template <int KT>
__global__ __launch_bounds__(1024) void cm_glu_dw_fwd_kernel(
    const float* __restrict__ u, const float* __restrict__ wdw, const float* __restrict__ bdw,
    int T, int C, int K, int TT, float* __restrict__ z, float* __restrict__ gout) {
  extern __shared__ float sm[];
  const int nth = blockDim.x;
  const int P = K / 2;
  const int W = TT + K - 1;
  float* gs = sm;                 // [W][C]
  float* ws = sm + (size_t)W * C;  // [C][K]
  const int b = blockIdx.y;
  const int t0 = blockIdx.x * TT;
  const size_t rb = (size_t)b * T;
  for (int i = threadIdx.x; i < C * K; i += nth) ws[i] = wdw[i];
  // the tile's window in batches of kLB elements per thread: all kLB value / gate loads are
  // issued (clamped addresses, no branches) before any is used -- one HBM latency per batch
  // (the 94 x 144 window is 24 elements per thread at 576 threads: one batch), instead of
  // a latency per 4 elements
  for (int i0 = 0; i0 < W * C; i0 += kLB * nth) {
    float va[kLB], vb[kLB];
#pragma unroll
    for (int q = 0; q < kLB; ++q) {
      const int i = i0 + threadIdx.x + q * nth;
      const int tl = i / C, c = i - tl * C;
      const int t = t0 - P + tl;
      const int tc = t < 0 ? 0 : (t >= T ? T - 1 : t);
      const float* ur = u + (rb + tc) * (size_t)(2 * C);
      const int cc = i < W * C ? c : 0;
      va[q] = ur[cc];
      vb[q] = ur[C + cc];
    }
#pragma unroll
    for (int q = 0; q < kLB; ++q) {
      const int i = i0 + threadIdx.x + q * nth;
      if (i >= W * C) break;
      const int tl = i / C;
      const int t = t0 - P + tl;
      gs[i] = (t >= 0 && t < T) ? va[q] * sigm(vb[q]) : 0.0f;
    }
  }
  __syncthreads();
  if constexpr (KT > 0) {
    const int nrb = (TT + kR - 1) / kR;
    for (int it = threadIdx.x; it < C * nrb; it += nth) {
      const int c = it % C, tl0 = kR * (it / C);
      if (t0 + tl0 >= T) break;
      float wt[KT], out[kR];
#pragma unroll
      for (int j = 0; j < KT; ++j) wt[j] = ws[c * KT + j];
      conv_window<KT, kR>(gs, C, c, tl0, wt, out);
      const float bc = bdw ? bdw[c] : 0.0f;
#pragma unroll
      for (int r = 0; r < kR; ++r) {
        const int t = t0 + tl0 + r;
        if (tl0 + r < TT && t < T) {
          z[(rb + t) * C + c] = out[r] + bc;
          gout[(rb + t) * C + c] = gs[(tl0 + r + P) * C + c];  // kept for the weight gradient
        }
      }
    }
  } else {
    for (int i = threadIdx.x; i < TT * C; i += nth) {
      const int tl = i / C, c = i - tl * C;
      const int t = t0 + tl;
      if (t >= T) break;  // i increases monotonically: later i are later frames
      float acc = 0.0f;
      const float* wc = ws + c * K;
      for (int j = 0; j < K; ++j) acc = fmaf(wc[j], gs[(tl + j) * C + c], acc);
      z[(rb + t) * C + c] = acc + (bdw ? bdw[c] : 0.0f);
      gout[(rb + t) * C + c] = gs[(tl + P) * C + c];  // kept for the weight gradient
    }
  }
}

// Per-(pass, chunk) partial sums of x and x^2 (fp64) per channel: block = (chunk, pass),
// thread c < C walks the chunk's rows.
__global__ __launch_bounds__(kThreads) void cm_stats_part_kernel(const float* __restrict__ x,
                                                                 int64_t rows_pp, int C, int S,
                                                                 double* __restrict__ part) {
  const int s = blockIdx.x, p = blockIdx.y;
  const int64_t r0 = rows_pp * s / S, r1 = rows_pp * (s + 1) / S;
  const float* xp = x + (size_t)p * rows_pp * C;
  for (int c = threadIdx.x; c < C; c += kThreads) {
    double s1 = 0.0, s2 = 0.0;
    // rows in batches of kSB loads in flight (clamped addresses, masked use)
    for (int64_t rb = r0; rb < r1; rb += kSB) {
      float v[kSB];
#pragma unroll
      for (int q = 0; q < kSB; ++q) v[q] = xp[min(rb + q, r1 - 1) * C + c];
#pragma unroll
      for (int q = 0; q < kSB; ++q)
        if (rb + q < r1) {
          s1 += (double)v[q];
          s2 += (double)v[q] * v[q];
        }
    }
    double* o = part + (((size_t)p * C + c) * S + s) * 2;
    o[0] = s1;
    o[1] = s2;
  }
}

// Fixed-order wave sum of a per-lane fp64 value (deterministic).
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// stats[p][c] = {mean, rstd} (biased variance, as BatchNorm's normalisation uses).
// One wave per (p, c): lanes take chunks s = lane, lane + 64, ...
__global__ __launch_bounds__(64) void cm_stats_final_kernel(const double* __restrict__ part,
                                                            int P, int C, int S, int64_t n,
                                                            float eps, float* __restrict__ stats) {
  const int i = blockIdx.x;  // p * C + c
  const int p = i / C, c = i - p * C;
  double s1 = 0.0, s2 = 0.0;
  for (int s = threadIdx.x; s < S; s += 64) {
    const double* o = part + (((size_t)p * C + c) * S + s) * 2;
    s1 += o[0];
    s2 += o[1];
  }
  s1 = wave_sum(s1);
  s2 = wave_sum(s2);
  if (threadIdx.x == 0) {
    const double mean = s1 / (double)n;
    double var = s2 / (double)n - mean * mean;
    var = var > 0.0 ? var : 0.0;
    stats[2 * i] = (float)mean;
    stats[2 * i + 1] = (float)(1.0 / sqrt(var + (double)eps));
  }
}

// v = swish(gamma * (z - mean) * rstd + beta), pass-wise statistics.
__global__ __launch_bounds__(kThreads) void cm_bn_swish_fwd_kernel(
    const float* __restrict__ z, const float* __restrict__ stats, const float* __restrict__ gamma,
    const float* __restrict__ beta, int64_t rows_pp, int C, int64_t total,
    float* __restrict__ v) {
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  for (int64_t i = blockIdx.x * (int64_t)kThreads + threadIdx.x; i < total; i += stride) {
    const int64_t row = i / C;
    const int c = (int)(i - row * C);
    const int p = (int)(row / rows_pp);
    const float* st = stats + 2 * ((size_t)p * C + c);
    const float y = (z[i] - st[0]) * st[1] * gamma[c] + beta[c];
    v[i] = swish(y);
  }
}

// ------------------------------------------------------------------ backward
// dy_bn = dv * swish'(y) at element (row, c), y recomputed from z and the statistics.
__device__ __forceinline__ float bn_dy(float dv, float zz, const float* st, float gm, float bt,
                                       float& xhat) {
  xhat = (zz - st[0]) * st[1];
  const float y = xhat * gm + bt;
  const float s = sigm(y);
  return dv * s * (1.0f + y * (1.0f - s));
}

// Per-(pass, chunk) partials of sum(dy_bn) and sum(dy_bn * xhat) (fp64).
__global__ __launch_bounds__(kThreads) void cm_bn_bwd_part_kernel(
    const float* __restrict__ dv, const float* __restrict__ z, const float* __restrict__ stats,
    const float* __restrict__ gamma, const float* __restrict__ beta, int64_t rows_pp, int C,
    int S, double* __restrict__ part) {
  const int s = blockIdx.x, p = blockIdx.y;
  const int64_t r0 = rows_pp * s / S, r1 = rows_pp * (s + 1) / S;
  const size_t base = (size_t)p * rows_pp * C;
  for (int c = threadIdx.x; c < C; c += kThreads) {
    const float* st = stats + 2 * ((size_t)p * C + c);
    const float gm = gamma[c], bt = beta[c];
    double s1 = 0.0, s2 = 0.0;
    for (int64_t rb = r0; rb < r1; rb += kSB) {
      float a[kSB], zz[kSB];
#pragma unroll
      for (int q = 0; q < kSB; ++q) {
        const size_t e = base + min(rb + q, r1 - 1) * C + c;
        a[q] = dv[e];
        zz[q] = z[e];
      }
#pragma unroll
      for (int q = 0; q < kSB; ++q)
        if (rb + q < r1) {
          float xh;
          const float d = bn_dy(a[q], zz[q], st, gm, bt, xh);
          s1 += d;
          s2 += (double)d * xh;
        }
    }
    double* o = part + (((size_t)p * C + c) * S + s) * 2;
    o[0] = s1;
    o[1] = s2;
  }
}

// coef[p][c] = {mean(dy_bn), mean(dy_bn * xhat)}; dgamma / dbeta summed over passes.
// One wave per channel.
__global__ __launch_bounds__(64) void cm_bn_bwd_final_kernel(
    const double* __restrict__ part, int P, int C, int S, int64_t n, float* __restrict__ coef,
    float* __restrict__ dgamma, float* __restrict__ dbeta) {
  const int c = blockIdx.x;
  double tg = 0.0, tb = 0.0;
  for (int p = 0; p < P; ++p) {
    double s1 = 0.0, s2 = 0.0;
    for (int s = threadIdx.x; s < S; s += 64) {
      const double* o = part + (((size_t)p * C + c) * S + s) * 2;
      s1 += o[0];
      s2 += o[1];
    }
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
    if (threadIdx.x == 0) {
      coef[2 * ((size_t)p * C + c)] = (float)(s1 / (double)n);
      coef[2 * ((size_t)p * C + c) + 1] = (float)(s2 / (double)n);
    }
    tb += s1;
    tg += s2;
  }
  if (threadIdx.x == 0) {
    dgamma[c] = (float)tg;
    dbeta[c] = (float)tb;
  }
}

// dz = dL/dz (BatchNorm + swish backward with per-pass batch statistics), elementwise.
__global__ __launch_bounds__(kThreads) void cm_dz_kernel(
    const float* __restrict__ dv, const float* __restrict__ z, const float* __restrict__ stats,
    const float* __restrict__ coef, const float* __restrict__ gamma,
    const float* __restrict__ beta, int64_t rows_pp, int C, int64_t total,
    float* __restrict__ dz) {
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  for (int64_t i = blockIdx.x * (int64_t)kThreads + threadIdx.x; i < total; i += stride) {
    const int64_t row = i / C;
    const int c = (int)(i - row * C);
    const size_t pc = 2 * ((size_t)(row / rows_pp) * C + c);
    float xh;
    const float dy = bn_dy(dv[i], z[i], stats + pc, gamma[c], beta[c], xh);
    dz[i] = gamma[c] * stats[pc + 1] * (dy - coef[pc] - xh * coef[pc + 1]);
  }
}

// Block = (time tile, utterance). LDS: dz over [t0-P, t0+TT+P) and g over the same window
// (plain copies of the global tensors), plus the weights. Writes dg = sum_j w[j]
// dz[t-j+P] for the tile's frames, and this block's depthwise weight/bias gradient partial:
// part[blk][c][j] = sum_t dz[t] g[t+j-P] over the tile's frames, part[blk][c][K] = sum dz.
template <int KT>
__global__ __launch_bounds__(1024) void cm_dw_bwd_kernel(
    const float* __restrict__ dz, const float* __restrict__ g, const float* __restrict__ wdw,
    int T, int C, int K, int TT, float* __restrict__ dg, float* __restrict__ wpart) {
  extern __shared__ float sm[];
  const int nth = blockDim.x;
  const int P = K / 2;
  const int W = TT + K - 1;
  float* dzs = sm;                 // [W][C], frame t0-P+i
  float* gs = sm + (size_t)W * C;  // [W][C]
  float* ws = gs + (size_t)W * C;  // [C][K]
  const int b = blockIdx.y;
  const int t0 = blockIdx.x * TT;
  const size_t rb = (size_t)b * T;
  for (int i = threadIdx.x; i < C * K; i += nth) ws[i] = wdw[i];
  // (batched window loads as in the forward)
  for (int i0 = 0; i0 < W * C; i0 += kLB * nth) {
    float va[kLB], vb[kLB];
#pragma unroll
    for (int q = 0; q < kLB; ++q) {
      const int i = i0 + threadIdx.x + q * nth;
      const int tl = i / C, c = i - tl * C;
      const int t = t0 - P + tl;
      const int tc = t < 0 ? 0 : (t >= T ? T - 1 : t);
      const size_t e = (rb + tc) * C + (i < W * C ? c : 0);
      va[q] = dz[e];
      vb[q] = g[e];
    }
#pragma unroll
    for (int q = 0; q < kLB; ++q) {
      const int i = i0 + threadIdx.x + q * nth;
      if (i >= W * C) break;
      const int t = t0 - P + i / C;
      const bool in = t >= 0 && t < T;
      dzs[i] = in ? va[q] : 0.0f;
      gs[i] = in ? vb[q] : 0.0f;
    }
  }
  __syncthreads();
  // dg[t] = sum_j w[j] dz[t - j + P] = sum_j' w[K-1-j'] dz-tile[tl + j'] (flipped weights)
  if constexpr (KT > 0) {
    const int nrb = (TT + kR - 1) / kR;
    for (int it = threadIdx.x; it < C * nrb; it += nth) {
      const int c = it % C, tl0 = kR * (it / C);
      if (t0 + tl0 >= T) break;
      float wt[KT], out[kR];
#pragma unroll
      for (int j = 0; j < KT; ++j) wt[j] = ws[c * KT + (KT - 1 - j)];
      conv_window<KT, kR>(dzs, C, c, tl0, wt, out);
#pragma unroll
      for (int r = 0; r < kR; ++r) {
        const int t = t0 + tl0 + r;
        if (tl0 + r < TT && t < T) dg[(rb + t) * C + c] = out[r];
      }
    }
  } else {
    for (int i = threadIdx.x; i < TT * C; i += nth) {
      const int tl = i / C, c = i - tl * C;
      const int t = t0 + tl;
      if (t >= T) break;
      const float* wc = ws + c * K;
      float acc = 0.0f;  // dz index for tap j: frame t - j + P  ->  LDS row tl + 2P - j
      for (int j = 0; j < K; ++j) acc = fmaf(wc[j], dzs[(tl + 2 * P - j) * C + c], acc);
      dg[(rb + t) * C + c] = acc;
    }
  }
  // weight-gradient partial over this tile's frames (frame t = t0 + tl, tl < n_t):
  // item = (channel c, 8 consecutive taps j0..j0+7; tap K is the bias, g == 1)
  const int n_t = min(TT, T - t0);
  float* wp = wpart + ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * C * (K + 1);
  const int ngrp = (K + 1 + 7) / 8;
  for (int it = threadIdx.x; it < C * ngrp; it += nth) {
    const int c = it % C, j0 = 8 * (it / C);  // consecutive threads = consecutive channels
    float acc[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] = 0.0f;
    // sliding window of raw tile values gr[q] = g-tile[tl + j0 + q] (row clamped: rows past
    // the window only meet taps j >= K), one new LDS read per frame; tap K (the bias) uses 1.
    const int W = TT + K - 1;
    float gr[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) gr[q] = gs[min(j0 + q, W - 1) * C + c];
    for (int tl = 0; tl < n_t; ++tl) {
      const float d = dzs[(tl + P) * C + c];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int j = j0 + q;
        acc[q] = fmaf(d, j < K ? gr[q] : (j == K ? 1.0f : 0.0f), acc[q]);
      }
#pragma unroll
      for (int q = 0; q < 7; ++q) gr[q] = gr[q + 1];
      gr[7] = gs[min(tl + 1 + j0 + 7, W - 1) * C + c];
    }
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (j0 + q <= K) wp[(size_t)c * (K + 1) + j0 + q] = acc[q];
  }
}

// GLU backward (conformer.py:156, g = a * sigmoid(b)): du = [dg * s, dg * a * s * (1 - s)].
__global__ __launch_bounds__(kThreads) void cm_glu_bwd_kernel(const float* __restrict__ dg,
                                                              const float* __restrict__ u, int C,
                                                              int64_t total,
                                                              float* __restrict__ du) {
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  for (int64_t i = blockIdx.x * (int64_t)kThreads + threadIdx.x; i < total; i += stride) {
    const int64_t row = i / C;
    const int c = (int)(i - row * C);
    const size_t ua = row * (size_t)(2 * C) + c;
    const float a = u[ua];
    const float sb = sigm(u[ua + C]);
    const float d = dg[i];
    du[ua] = d * sb;
    du[ua + C] = d * a * sb * (1.0f - sb);
  }
}

// 32-bit offsets into one utterance slice through a buffer descriptor (no 64-bit address
// arithmetic per access; loads past the slice read 0)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const float* base, size_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, (int)bytes,
                                           0x00020000);
}
__device__ __forceinline__ float bload(__amdgpu_buffer_rsrc_t r, int off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}
__device__ __forceinline__ void bstore(__amdgpu_buffer_rsrc_t r, int off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(int, v), r, off, 0, 0);
}
typedef float cm_f32x4 __attribute__((ext_vector_type(4)));
// four consecutive channels (off 16-byte aligned: C % 4 == 0, channel groups of 4)
__device__ __forceinline__ cm_f32x4 bload4(__amdgpu_buffer_rsrc_t r, int off) {
  return __builtin_bit_cast(cm_f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
constexpr int kLBQ = 4;  // channel quads per thread and batch of the tiles' window loads

// ------------------------------------------------------------------ channel-split tiles
// The kernels above give one block a [W][C] window (all channels: 94 x 144 x 2 floats of LDS
// in the backward), so one block fits a CU and its window loads never overlap arithmetic
// (PMC: 58% of wave time waiting). These split the channels: block = (64-frame tile,
// utterance, CG-channel group), 256 threads, LDS [W][CG] per array -- several blocks per
// CU. The backward also folds what were two more passes over HBM into the tile: dz (the
// BatchNorm + swish backward) is formed while the window loads, and the GLU backward is
// applied to dg in registers (du written directly; dz and dg never reach HBM). The
// arithmetic is the kernels' above, operation for operation (bitwise identical outputs).
constexpr int kTT = 64;  // frames per tile (pick_tt's choice at every shape these serve)

template <int KT, int CG>
__global__ __launch_bounds__(kThreads) void cm_fwd_tile_kernel(
    const float* __restrict__ u, const float* __restrict__ wdw, const float* __restrict__ bdw,
    int T, int C, float* __restrict__ z, float* __restrict__ gout) {
  constexpr int P = KT / 2, W = kTT + KT - 1, NW = W * CG;
  constexpr int CQ = CG / 4, NQ = W * CQ;  // window loads in channel quads (dwordx4)
  __shared__ __attribute__((aligned(16))) float gs[NW];
  const int t0 = blockIdx.x * kTT, b = blockIdx.y, c0 = blockIdx.z * CG;
  const size_t rb = (size_t)b * T;
  const __amdgpu_buffer_rsrc_t ru = rsrc(u + rb * 2 * C, (size_t)T * 2 * C * 4);
  for (int i0 = 0; i0 < NQ; i0 += kLBQ * kThreads) {
    cm_f32x4 va[kLBQ], vb[kLBQ];
#pragma unroll
    for (int q = 0; q < kLBQ; ++q) {
      const int i = i0 + threadIdx.x + q * kThreads;
      const int tl = i / CQ, cq = i - tl * CQ;
      const int t = t0 - P + tl;
      const int tc = t < 0 ? 0 : (t >= T ? T - 1 : t);
      const int off = 4 * (tc * 2 * C + c0 + 4 * (i < NQ ? cq : 0));
      va[q] = bload4(ru, off);
      vb[q] = bload4(ru, off + 4 * C);
    }
#pragma unroll
    for (int q = 0; q < kLBQ; ++q) {
      const int i = i0 + threadIdx.x + q * kThreads;
      if (i >= NQ) break;
      const int tl = i / CQ, cq = i - tl * CQ;
      const int t = t0 - P + tl;
      const bool in = t >= 0 && t < T;
      cm_f32x4 g4;
#pragma unroll
      for (int k = 0; k < 4; ++k) g4[k] = in ? va[q][k] * sigm(vb[q][k]) : 0.0f;
      *reinterpret_cast<cm_f32x4*>(gs + tl * CG + 4 * cq) = g4;
    }
  }
  __syncthreads();
  constexpr int nrb = kTT / kR;
  for (int it = threadIdx.x; it < CG * nrb; it += kThreads) {
    const int c = it % CG, tl0 = kR * (it / CG);
    if (t0 + tl0 >= T) break;
    float wt[KT], out[kR];
#pragma unroll
    for (int j = 0; j < KT; ++j) wt[j] = wdw[(c0 + c) * KT + j];
    conv_window<KT, kR>(gs, CG, c, tl0, wt, out);
    const float bc = bdw ? bdw[c0 + c] : 0.0f;
#pragma unroll
    for (int r = 0; r < kR; ++r) {
      const int t = t0 + tl0 + r;
      if (t < T) {
        z[(rb + t) * C + c0 + c] = out[r] + bc;
        gout[(rb + t) * C + c0 + c] = gs[(tl0 + r + P) * CG + c];  // kept for the weight gradient
      }
    }
  }
}

template <int KT, int CG>
__global__ __launch_bounds__(kThreads) void cm_bwd_tile_kernel(
    const float* __restrict__ dv, const float* __restrict__ z, const float* __restrict__ g,
    const float* __restrict__ u, const float* __restrict__ stats, const float* __restrict__ coef,
    const float* __restrict__ gamma, const float* __restrict__ beta,
    const float* __restrict__ wdw, int64_t rows_pp, int T, int C, float* __restrict__ du,
    float* __restrict__ wpart, CmWgradEntry* __restrict__ tslot, CmWgradEntry ent) {
  constexpr int P = KT / 2, W = kTT + KT - 1, NW = W * CG;
  constexpr int CQ = CG / 4, NQ = W * CQ;  // window loads in channel quads (dwordx4)
  if (tslot && blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0 && threadIdx.x == 0) *tslot = ent;
  __shared__ __attribute__((aligned(16))) float dzs[NW];  // dz over frames [t0-P, t0+kTT+P)
  __shared__ __attribute__((aligned(16))) float gs[NW];   // g over the same window
  const int t0 = blockIdx.x * kTT, b = blockIdx.y, c0 = blockIdx.z * CG;
  const size_t rb = (size_t)b * T;
  const int pass = (int)(rb / rows_pp);  // every frame of utterance b is in its pass
  const size_t sl = (size_t)T * C * 4;
  const __amdgpu_buffer_rsrc_t rdv = rsrc(dv + rb * C, sl), rz = rsrc(z + rb * C, sl),
                               rg = rsrc(g + rb * C, sl);
  const __amdgpu_buffer_rsrc_t ru = rsrc(u + rb * 2 * C, 2 * sl), rdu = rsrc(du + rb * 2 * C, 2 * sl);
  // window: dz = BatchNorm + swish backward (per-pass statistics, cm_dz_kernel's formula)
  for (int i0 = 0; i0 < NQ; i0 += kLBQ * kThreads) {
    cm_f32x4 va[kLBQ], vz[kLBQ], vg[kLBQ];
#pragma unroll
    for (int q = 0; q < kLBQ; ++q) {
      const int i = i0 + threadIdx.x + q * kThreads;
      const int tl = i / CQ, cq = i - tl * CQ;
      const int t = t0 - P + tl;
      const int tc = t < 0 ? 0 : (t >= T ? T - 1 : t);
      const int e = 4 * (tc * C + c0 + 4 * (i < NQ ? cq : 0));
      va[q] = bload4(rdv, e);
      vz[q] = bload4(rz, e);
      vg[q] = bload4(rg, e);
    }
#pragma unroll
    for (int q = 0; q < kLBQ; ++q) {
      const int i = i0 + threadIdx.x + q * kThreads;
      if (i >= NQ) break;
      const int tl = i / CQ, cq = i - tl * CQ;
      const int t = t0 - P + tl;
      const bool in = t >= 0 && t < T;
      cm_f32x4 dz4, g4;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int cg = c0 + 4 * cq + k;
        const int pc = 2 * (pass * C + cg);
        float xh;
        const float dy = bn_dy(va[q][k], vz[q][k], stats + pc, gamma[cg], beta[cg], xh);
        const float dzv = gamma[cg] * stats[pc + 1] * (dy - coef[pc] - xh * coef[pc + 1]);
        dz4[k] = in ? dzv : 0.0f;
        g4[k] = in ? vg[q][k] : 0.0f;
      }
      *reinterpret_cast<cm_f32x4*>(dzs + tl * CG + 4 * cq) = dz4;
      *reinterpret_cast<cm_f32x4*>(gs + tl * CG + 4 * cq) = g4;
    }
  }
  __syncthreads();
  // dg[t] = sum_j w[j] dz[t - j + P] (flipped weights), then the GLU backward (cm_glu_bwd's
  // formula) in registers: du = [dg * s, dg * a * s * (1 - s)], (a, b) = u, s = sigmoid(b)
  constexpr int nrb = kTT / kR;
  for (int it = threadIdx.x; it < CG * nrb; it += kThreads) {
    const int c = it % CG, tl0 = kR * (it / CG);
    if (t0 + tl0 >= T) break;
    float wt[KT], out[kR];
#pragma unroll
    for (int j = 0; j < KT; ++j) wt[j] = wdw[(c0 + c) * KT + (KT - 1 - j)];
    conv_window<KT, kR>(dzs, CG, c, tl0, wt, out);
    float ua[kR], ub[kR];
    const int a0 = 4 * ((t0 + tl0) * 2 * C + c0 + c);  // frames past T read 0, never stored
#pragma unroll
    for (int r = 0; r < kR; ++r) {
      ua[r] = bload(ru, a0 + 8 * C * r);
      ub[r] = bload(ru, a0 + 8 * C * r + 4 * C);
    }
#pragma unroll
    for (int r = 0; r < kR; ++r) {
      if (t0 + tl0 + r < T) {
        const float sb = sigm(ub[r]);
        bstore(rdu, a0 + 8 * C * r, out[r] * sb);
        bstore(rdu, a0 + 8 * C * r + 4 * C, out[r] * ua[r] * sb * (1.0f - sb));
      }
    }
  }
  // weight-gradient partial over this tile's frames (cm_dw_bwd_kernel's loop): item =
  // (channel, 8 consecutive taps j0..j0+7; tap K is the bias, g == 1)
  const int n_t = min(kTT, T - t0);
  float* wp = wpart + ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * C * (KT + 1);
  constexpr int ngrp = (KT + 1 + 7) / 8;
  for (int it = threadIdx.x; it < CG * ngrp; it += kThreads) {
    const int c = it % CG, j0 = 8 * (it / CG);
    float acc[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] = 0.0f;
    if (KT > 0 && j0 + 7 < KT) {
      // all 8 taps are weights: 8 frames per round from a 16-value window of g (one move per
      // frame instead of seven, no per-tap select); the same fma order per accumulator
      float win[16];
#pragma unroll
      for (int q = 0; q < 8; ++q) win[q] = gs[(j0 + q) * CG + c];
      int tl = 0;
      for (; tl + 8 <= n_t; tl += 8) {
#pragma unroll
        for (int q = 0; q < 8; ++q) win[8 + q] = gs[(tl + 8 + j0 + q) * CG + c];
#pragma unroll
        for (int st = 0; st < 8; ++st) {
          const float d = dzs[(tl + st + P) * CG + c];
#pragma unroll
          for (int q = 0; q < 8; ++q) acc[q] = fmaf(d, win[st + q], acc[q]);
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) win[q] = win[8 + q];
      }
      for (; tl < n_t; ++tl) {  // the last tile's remaining frames
        const float d = dzs[(tl + P) * CG + c];
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[q] = fmaf(d, win[q], acc[q]);
#pragma unroll
        for (int q = 0; q < 7; ++q) win[q] = win[q + 1];
        win[7] = gs[min(tl + 1 + j0 + 7, W - 1) * CG + c];
      }
    } else {
      float gr[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) gr[q] = gs[min(j0 + q, W - 1) * CG + c];
      for (int tl = 0; tl < n_t; ++tl) {
        const float d = dzs[(tl + P) * CG + c];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int j = j0 + q;
          acc[q] = fmaf(d, j < KT ? gr[q] : (j == KT ? 1.0f : 0.0f), acc[q]);
        }
#pragma unroll
        for (int q = 0; q < 7; ++q) gr[q] = gr[q + 1];
        gr[7] = gs[min(tl + 1 + j0 + 7, W - 1) * CG + c];
      }
    }
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (j0 + q <= KT) wp[(size_t)(c0 + c) * (KT + 1) + j0 + q] = acc[q];
  }
}

// ------------------------------------------------------------------ row-vectorised passes
// The per-element kernels above index with 64-bit divisions (i / C, row / rows_pp) and one
// float per thread; these take a row's channels as float4 groups (C % 4 == 0): thread
// (row lane, group) of a 256-thread block, kRL = 256 / (C/4) rows per block iteration, one
// division per row, dwordx4 loads and stores.
typedef float f32x4 __attribute__((ext_vector_type(4)));

// v = swish(gamma * (z - mean) * rstd + beta), pass-wise statistics (cm_bn_swish_fwd's formula)
__global__ __launch_bounds__(kThreads) void cm_bn_swish_rows_kernel(
    const float* __restrict__ z, const float* __restrict__ stats, const float* __restrict__ gamma,
    const float* __restrict__ beta, int rows_pp, int rows, int C, float* __restrict__ v) {
  const int G = C / 4, rl = threadIdx.x / G, q = threadIdx.x - rl * G, RL = kThreads / G;
  if (rl >= RL) return;
  const int c = 4 * q;
  const f32x4 gm = *reinterpret_cast<const f32x4*>(gamma + c);
  const f32x4 bt = *reinterpret_cast<const f32x4*>(beta + c);
  for (int row = blockIdx.x * RL + rl; row < rows; row += gridDim.x * RL) {
    const int p = row / rows_pp;
    const float* st = stats + 2 * ((size_t)p * C + c);
    const f32x4 zz = *reinterpret_cast<const f32x4*>(z + (size_t)row * C + c);
    f32x4 out;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float y = (zz[e] - st[2 * e]) * st[2 * e + 1] * gm[e] + bt[e];
      out[e] = swish(y);
    }
    *reinterpret_cast<f32x4*>(v + (size_t)row * C + c) = out;
  }
}

// Per-(pass, chunk) partial sums (fp64) of x and x^2 (MODE 0: the statistics of z) or of
// dy_bn and dy_bn * xhat (MODE 1: the BatchNorm backward's sums), per channel: block =
// (chunk, pass); thread (row lane rl, group q) walks rows r0 + rl, r0 + rl + RL, ... of the
// chunk; the RL row lanes are added in lane order through LDS (fixed order).
template <int MODE>
__global__ __launch_bounds__(kThreads) void cm_sums_rows_kernel(
    const float* __restrict__ x, const float* __restrict__ dv, const float* __restrict__ stats,
    const float* __restrict__ gamma, const float* __restrict__ beta, int64_t rows_pp, int C,
    int S, double* __restrict__ part) {
  __shared__ double red[kThreads][2 * 4];
  const int G = C / 4, rl = threadIdx.x / G, q = threadIdx.x - rl * G, RL = kThreads / G;
  const int s = blockIdx.x, p = blockIdx.y;
  const int64_t r0 = rows_pp * s / S, r1 = rows_pp * (s + 1) / S;
  const size_t base = (size_t)p * rows_pp * C;
  const int c = 4 * q;
  double s1[4] = {0.0, 0.0, 0.0, 0.0}, s2[4] = {0.0, 0.0, 0.0, 0.0};
  if (rl < RL) {
    f32x4 gm = {0.f, 0.f, 0.f, 0.f}, bt = gm;
    const float* st = stats + 2 * ((size_t)p * C + c);
    if (MODE == 1) {
      gm = *reinterpret_cast<const f32x4*>(gamma + c);
      bt = *reinterpret_cast<const f32x4*>(beta + c);
    }
    // rows in batches of 4 per lane, all loads of a batch issued first (clamped addresses,
    // masked use)
    for (int64_t rb = r0 + rl; rb < r1; rb += 4 * RL) {
      f32x4 a[4], d[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int64_t r = min(rb + k * RL, r1 - 1);
        a[k] = *reinterpret_cast<const f32x4*>(x + base + r * C + c);
        if (MODE == 1) d[k] = *reinterpret_cast<const f32x4*>(dv + base + r * C + c);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (rb + k * RL >= r1) break;
        if (MODE == 0) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            s1[e] += (double)a[k][e];
            s2[e] += (double)a[k][e] * a[k][e];
          }
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float xh;
            const float dd = bn_dy(d[k][e], a[k][e], st + 2 * e, gm[e], bt[e], xh);
            s1[e] += dd;
            s2[e] += (double)dd * xh;
          }
        }
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    red[threadIdx.x][2 * e] = s1[e];
    red[threadIdx.x][2 * e + 1] = s2[e];
  }
  __syncthreads();
  if (rl == 0) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      double t1 = 0.0, t2 = 0.0;
      for (int l = 0; l < RL; ++l) {
        t1 += red[l * G + q][2 * e];
        t2 += red[l * G + q][2 * e + 1];
      }
      double* o = part + (((size_t)p * C + c + e) * S + s) * 2;
      o[0] = t1;
      o[1] = t2;
    }
  }
}

// channel group of the tile kernels (0: none applies -- the whole-row kernels run).
// OB_CM_TILE=0 in the environment forces the whole-row kernels (bitwise A/B test).
int tile_cg(int64_t C, int64_t K) {
  static const bool off = [] {
    const char* e = getenv("OB_CM_TILE");
    return e && e[0] == '0';
  }();
  if (off || K != 31) return 0;
  if (C % 48 == 0) return 48;
  if (C % 32 == 0) return 32;
  if (C % 16 == 0) return 16;
  return 0;
}

// dw_dw[c][j] = sum over blocks (fixed order) of the partials; db_dw[c] likewise.
// One wave per output: lanes take blocks k = lane, lane + 64, ... (fp64 lane sums).
// Block = 64 consecutive outputs (c, j) x 16 block-slices (slice q: partials q, q+16, ...,
// 8 loads in flight), fp64, the slices added in order through LDS (fixed order). Lanes read
// consecutive outputs of one partial: coalesced (one wave per output walked the partials
// 18 KB apart: a cache line per 4-byte value, 16 us per launch).
constexpr int kWfSlices = 16;
__device__ __forceinline__ void cm_wgrad_final_block(
    int bid, const float* __restrict__ wpart, int nblk, int C, int K, float* __restrict__ dw,
    float* __restrict__ db) {
  __shared__ double red[kWfSlices][64];
  const int n = C * (K + 1);
  const int lane = threadIdx.x & 63, sl = threadIdx.x >> 6;
  const int i = bid * 64 + lane;  // c * (K + 1) + j
  const int ic = i < n ? i : n - 1;
  double acc = 0.0;
  for (int k0 = sl; k0 < nblk; k0 += 8 * kWfSlices) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int k = k0 + u * kWfSlices;
      v[u] = wpart[(size_t)(k < nblk ? k : nblk - 1) * n + ic];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (k0 + u * kWfSlices < nblk) acc += (double)v[u];
  }
  red[sl][lane] = acc;
  __syncthreads();
  if (sl != 0 || i >= n) return;
  double t = 0.0;
#pragma unroll
  for (int q = 0; q < kWfSlices; ++q) t += red[q][lane];
  const int c = i / (K + 1), j = i - c * (K + 1);
  if (j < K) dw[(size_t)c * K + j] = (float)t;
  else if (db) db[c] = (float)t;
}

__global__ __launch_bounds__(64 * kWfSlices) void cm_wgrad_final_kernel(
    const float* __restrict__ wpart, int nblk, int C, int K, float* __restrict__ dw,
    float* __restrict__ db) {
  cm_wgrad_final_block((int)blockIdx.x, wpart, nblk, C, K, dw, db);
}

// every deferred finish of a backward: grid (output groups of 64, entries)
__global__ __launch_bounds__(64 * kWfSlices) void cm_wgrad_table_kernel(
    const CmWgradEntry* __restrict__ tab) {
  const CmWgradEntry e = tab[blockIdx.y];
  if ((int)blockIdx.x * 64 >= e.C * (e.K + 1)) return;
  cm_wgrad_final_block((int)blockIdx.x, e.wpart, e.nblk, e.C, e.K, e.dw, e.db);
}

// Row chunks per pass of the BatchNorm statistics / backward sums: ~16 rows per block at
// Conformer-S (one batch of kSB loads in flight per thread), at most 512 chunks. Partials
// are laid out [pass][channel][chunk][2] so the final kernels' lanes (consecutive chunks)
// read consecutive 16-byte pairs.
// chunks of the row-vectorised sums: ~8 rows per row lane (kThreads / (C/4) lanes), at most
// stats_chunks' count (the workspace is sized for that)
int rows_chunks(int64_t rows_pp, int64_t C) {
  const int64_t per = 8 * (kThreads / (C / 4));
  const int64_t s = (rows_pp + per - 1) / per;
  const int64_t cap = (rows_pp + kSB - 1) / kSB;
  const int64_t m = cap < 512 ? cap : 512;
  return (int)(s < 1 ? 1 : (s > m ? m : s));
}

int stats_chunks(int64_t rows_pp) {
  const int64_t s = (rows_pp + kSB - 1) / kSB;
  return (int)(s < 1 ? 1 : (s > 512 ? 512 : s));
}

size_t lds_fwd(int C, int K, int TT) { return sizeof(float) * ((size_t)(TT + K - 1) * C + (size_t)C * K); }
size_t lds_bwd(int C, int K, int TT) {
  return sizeof(float) * (2 * (size_t)(TT + K - 1) * C + (size_t)C * K);
}

// Frames per depthwise block: the widest tile whose backward LDS image fits (0: none).
int pick_tt(int64_t C, int64_t K) {
  for (int tt : {64, 32, 16})
    if (lds_bwd((int)C, (int)K, tt) <= kMaxLds) return tt;
  return 0;
}

}  // namespace

// Threads of the depthwise blocks: one per (channel, 8-tap group) of the weight gradient
// (576 = 9 waves at C = 144, K = 31), within [256, 1024].
int dw_threads(int64_t C, int64_t K) {
  int64_t n = C * ((K + 1 + 7) / 8);
  n = (n + 63) / 64 * 64;
  return (int)(n < 256 ? 256 : (n > 1024 ? 1024 : n));
}

bool convmod_supported(int64_t C, int64_t K) {
  return C >= 1 && K >= 1 && K % 2 == 1 && K <= 127 && pick_tt(C, K) > 0;
}

size_t convmod_workspace(int64_t P, int64_t Bt, int64_t T, int64_t C, int64_t K) {
  const int64_t rows_pp = Bt / P * T;
  const int S = stats_chunks(rows_pp);
  const int64_t ntt = ceil_div(T, pick_tt(C, K));
  size_t b = sizeof(double) * (size_t)(P * S * C * 2);         // stats / bn partials
  b += sizeof(float) * (size_t)(P * C * 2);                     // bn backward coefficients
  b += sizeof(float) * (size_t)(Bt * ntt * C * (K + 1));        // weight-gradient partials
  b += 2 * sizeof(float) * (size_t)(Bt * T * C);                 // dz, dg
  return b + 256;
}

void launch_convmod_fwd(const float* u, const float* wdw, const float* bdw, const float* gamma,
                        const float* beta, int64_t P, int64_t Bt, int64_t T, int64_t C, int64_t K,
                        float eps, float* z, float* g, float* stats, float* v, void* ws,
                        hipStream_t s) {
  const int64_t rows_pp = Bt / P * T;
  const int S = stats_chunks(rows_pp);
  double* part = reinterpret_cast<double*>(ws);
  const int TT = pick_tt(C, K);
  const dim3 gdw((unsigned)ceil_div(T, TT), (unsigned)Bt);
  const int cg = TT == kTT ? tile_cg(C, K) : 0;
  if (cg) {  // channel-split tiles (the Conformer width K = 31, C a multiple of 16)
    const dim3 gt((unsigned)ceil_div(T, kTT), (unsigned)Bt, (unsigned)(C / cg));
    if (cg == 48)
      hipLaunchKernelGGL((cm_fwd_tile_kernel<31, 48>), gt, dim3(kThreads), 0, s, u, wdw, bdw,
                         (int)T, (int)C, z, g);
    else if (cg == 32)
      hipLaunchKernelGGL((cm_fwd_tile_kernel<31, 32>), gt, dim3(kThreads), 0, s, u, wdw, bdw,
                         (int)T, (int)C, z, g);
    else
      hipLaunchKernelGGL((cm_fwd_tile_kernel<31, 16>), gt, dim3(kThreads), 0, s, u, wdw, bdw,
                         (int)T, (int)C, z, g);
  } else if (K == 31)  // the Conformer width (reference default, every config here)
    hipLaunchKernelGGL(cm_glu_dw_fwd_kernel<31>, gdw, dim3(dw_threads(C, K)), lds_fwd((int)C, (int)K, TT),
                       s, u, wdw, bdw, (int)T, (int)C, (int)K, TT, z, g);
  else
    hipLaunchKernelGGL(cm_glu_dw_fwd_kernel<0>, gdw, dim3(dw_threads(C, K)), lds_fwd((int)C, (int)K, TT),
                       s, u, wdw, bdw, (int)T, (int)C, (int)K, TT, z, g);
  const bool rowvec = C % 4 == 0 && C / 4 <= kThreads && Bt * T < (1ll << 31);
  const int Sr = rowvec ? rows_chunks(rows_pp, C) : S;
  if (rowvec)
    hipLaunchKernelGGL(cm_sums_rows_kernel<0>, dim3((unsigned)Sr, (unsigned)P), dim3(kThreads), 0, s,
                       (const float*)z, (const float*)nullptr, (const float*)nullptr,
                       (const float*)nullptr, (const float*)nullptr, rows_pp, (int)C, Sr, part);
  else
    hipLaunchKernelGGL(cm_stats_part_kernel, dim3((unsigned)S, (unsigned)P), dim3(kThreads), 0, s,
                       (const float*)z, rows_pp, (int)C, S, part);
  hipLaunchKernelGGL(cm_stats_final_kernel, dim3((unsigned)(P * C)), dim3(64), 0, s,
                     (const double*)part, (int)P, (int)C, Sr, rows_pp, eps, stats);
  const int64_t total = Bt * T * C;
  int64_t blocks = ceil_div(total, kThreads);
  if (blocks > 8192) blocks = 8192;
  if (rowvec) {
    const int rl = kThreads / (int)(C / 4);
    const int64_t rb = ceil_div(Bt * T, rl);
    hipLaunchKernelGGL(cm_bn_swish_rows_kernel, dim3((unsigned)(rb < 8192 ? rb : 8192)),
                       dim3(kThreads), 0, s, (const float*)z, (const float*)stats, gamma, beta,
                       (int)rows_pp, (int)(Bt * T), (int)C, v);
  } else {
    hipLaunchKernelGGL(cm_bn_swish_fwd_kernel, dim3((unsigned)blocks), dim3(kThreads), 0, s,
                       (const float*)z, (const float*)stats, gamma, beta, rows_pp, (int)C, total, v);
  }
}

void launch_convmod_bwd(const float* dv, const float* u, const float* z, const float* g,
                        const float* stats, const float* wdw, const float* gamma,
                        const float* beta, int64_t P, int64_t Bt, int64_t T, int64_t C, int64_t K,
                        float* du, float* dwdw, float* dbdw, float* dgamma, float* dbeta, void* ws,
                        hipStream_t s, const CmDefer* defer) {
  const int64_t rows_pp = Bt / P * T;
  const int S = stats_chunks(rows_pp);
  const int TT = pick_tt(C, K);
  const int64_t ntt = ceil_div(T, TT);
  double* part = reinterpret_cast<double*>(ws);
  float* coef = reinterpret_cast<float*>(part + (size_t)(P * S * C * 2));
  float* wpart = coef + (size_t)(P * C * 2);
  float* dz = wpart + (size_t)(Bt * ntt * C * (K + 1));
  float* dg = dz + (size_t)(Bt * T * C);
  const int64_t total = Bt * T * C;
  int64_t eblocks = ceil_div(total, kThreads);
  if (eblocks > 8192) eblocks = 8192;
  const bool rowvec = C % 4 == 0 && C / 4 <= kThreads;
  const int Sr = rowvec ? rows_chunks(rows_pp, C) : S;
  if (rowvec)
    hipLaunchKernelGGL(cm_sums_rows_kernel<1>, dim3((unsigned)Sr, (unsigned)P), dim3(kThreads), 0, s,
                       z, dv, stats, gamma, beta, rows_pp, (int)C, Sr, part);
  else
    hipLaunchKernelGGL(cm_bn_bwd_part_kernel, dim3((unsigned)S, (unsigned)P), dim3(kThreads), 0, s,
                       dv, z, stats, gamma, beta, rows_pp, (int)C, S, part);
  hipLaunchKernelGGL(cm_bn_bwd_final_kernel, dim3((unsigned)C), dim3(64), 0, s,
                     (const double*)part, (int)P, (int)C, Sr, rows_pp, coef, dgamma, dbeta);
  const int cg = TT == kTT ? tile_cg(C, K) : 0;
  if (cg) {  // dz, dg and the GLU backward inside the channel-split tiles
    const dim3 gt((unsigned)ntt, (unsigned)Bt, (unsigned)(C / cg));
    const bool dfr = defer && defer->table && Bt * ntt > 0;
    CmWgradEntry* tslot = dfr ? defer->table + defer->slot : nullptr;
    const CmWgradEntry ent{wpart, dwdw, dbdw, (int)(Bt * ntt), (int)C, (int)K};
#define OB_CM_BWD_TILE(CG)                                                                      \
  hipLaunchKernelGGL((cm_bwd_tile_kernel<31, CG>), gt, dim3(kThreads), 0, s, dv, z, g, u, stats, \
                     (const float*)coef, gamma, beta, wdw, rows_pp, (int)T, (int)C, du, wpart,   \
                     tslot, ent)
    if (cg == 48) OB_CM_BWD_TILE(48);
    else if (cg == 32) OB_CM_BWD_TILE(32);
    else OB_CM_BWD_TILE(16);
#undef OB_CM_BWD_TILE
    if (!dfr)
      hipLaunchKernelGGL(cm_wgrad_final_kernel, dim3((unsigned)ceil_div(C * (K + 1), 64)),
                         dim3(64 * kWfSlices), 0, s,
                         (const float*)wpart, (int)(Bt * ntt), (int)C, (int)K, dwdw, dbdw);
    return;
  }
  hipLaunchKernelGGL(cm_dz_kernel, dim3((unsigned)eblocks), dim3(kThreads), 0, s, dv, z, stats,
                     (const float*)coef, gamma, beta, rows_pp, (int)C, total, dz);
  const dim3 gdw((unsigned)ntt, (unsigned)Bt);
  if (K == 31)
    hipLaunchKernelGGL(cm_dw_bwd_kernel<31>, gdw, dim3(dw_threads(C, K)), lds_bwd((int)C, (int)K, TT), s,
                       (const float*)dz, g, wdw, (int)T, (int)C, (int)K, TT, dg, wpart);
  else
    hipLaunchKernelGGL(cm_dw_bwd_kernel<0>, gdw, dim3(dw_threads(C, K)), lds_bwd((int)C, (int)K, TT), s,
                       (const float*)dz, g, wdw, (int)T, (int)C, (int)K, TT, dg, wpart);
  hipLaunchKernelGGL(cm_glu_bwd_kernel, dim3((unsigned)eblocks), dim3(kThreads), 0, s,
                     (const float*)dg, u, (int)C, total, du);
  hipLaunchKernelGGL(cm_wgrad_final_kernel, dim3((unsigned)ceil_div(C * (K + 1), 64)),
                     dim3(64 * kWfSlices), 0, s,
                     (const float*)wpart, (int)(Bt * ntt), (int)C, (int)K, dwdw, dbdw);
}

bool convmod_bwd_deferrable(int64_t C, int64_t K) {
  const int TT = pick_tt(C, K);
  return TT == kTT && tile_cg(C, K) != 0;
}

void launch_cm_wgrad_table(const CmWgradEntry* table, int n, int nmax, hipStream_t s) {
  if (n <= 0 || nmax <= 0) return;
  hipLaunchKernelGGL(cm_wgrad_table_kernel, dim3((unsigned)ceil_div(nmax, 64), (unsigned)n),
                     dim3(64 * kWfSlices), 0, s, table);
}

}  // namespace ob
