// decattn.hip — the decoder's scaled-dot-product attention core, fused (forward + backward).
//
// Reference: the stock nn.TransformerDecoderLayer of onebit_asr/conformer.py:275-299, i.e.
// torch.nn.functional.multi_head_attention_forward between the in- and out-projections:
//   S = (q k^T) * (1/sqrt(dh)) + mask      mask: -inf at masked keys (key padding) and, for
//                                           self-attention, at keys after the query (causal)
//   A = softmax(S); Ad = dropout(A); ctx = Ad v   (per head, heads = column slices of e)
// torch runs that as ~7 kernels forward and ~12 backward per call (batched GEMMs, a head
// transpose copy each way, scale, mask add, softmax, dropout, their backwards) for at most
// 41 x 250 scores per head. Here one block per (batch row, head) keeps the head's q / k / v
// rows and its scores in LDS: one launch forward, one backward, no transposes (q / k / v are
// read as column slices of the packed projection outputs, their gradients written into the
// packed gradient the same way).
//
// Arithmetic: fp32 fma chains on the VALU (the products are tiny: 1.5 MFLOP per head);
// softmax = exp(s - max) / sum with IEEE exp and division; the backward's row term is
// sum_j A_ij dA_ij (torch's softmax backward), reduced across the block's waves in a fixed
// order. Dropout: the counter hash of ob_drop.h (not torch's Philox stream, like every fused
// dropout of this library) on index ((b*H + h)*Lq + i)*Lk + j; the forward stores each kept
// probability as P and each dropped one as -P (the sign bit is free, P >= 0), the backward
// reads the keep bit back. Fully masked rows give NaN, as torch's softmax does.
//
// Blocks: forward (b, h, 16-query tile), backward (b, h) -- dk / dv sum over every query.
// Layout: q rows at q + (b*Lq + i)*sq + h*dh (sq = the row stride in floats: 3e for the
// packed self-attention projection, e or 2e for the cross-attention pieces), k / v likewise
// with Lk rows; ctx, dctx [B][Lq][H*dh]; probs [B][H][Lq][Lk]; kmask uint8 [B][Lk] (1 =
// masked), may be null.
#include <math.h>

#include <algorithm>

#include "ob_drop.h"
#include "ob_launch.h"

namespace ob {

namespace {

constexpr int kDaThreads = 256;  // one key per thread in the per-key phases: Lk <= 256

struct DaArgs {
  const float* q;
  const float* k;
  const float* v;
  int64_t sq, sk, sv;
  const uint8_t* kmask;
  int causal;
  int H, Lq, Lk;
  float scale;
  DropCfg dc;
  const uint64_t* rng;
  uint64_t rng_off;
  int vec;  // q / k / v bases and strides 16-byte aligned
};

// Bijective XCD-aware remap (hardware block b runs on XCD b % 8)
__device__ __forceinline__ int xcd_logical_da(int b, int nb) {
  const int q = nb / 8, r = nb % 8, x = b % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

constexpr int kDaQT = 16;  // query rows per forward block

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

__host__ __device__ inline int lk_pitch(int Lk) { return (Lk + 3) & ~3; }

// rows [0, n) of a strided [rows][*] tensor's head slice into an LDS [n][DH] image (DH % 4
// == 0: every row 16-byte aligned, read back as float4 broadcasts). Every load of a pass is
// issued before the first store (one memory latency per pass, not per element): vec (16-byte
// aligned rows) moves float4s, 12 per thread per pass; otherwise floats, 40 per pass.
template <int DH>
__device__ __forceinline__ void stage_rows(float* __restrict__ dst, const float* __restrict__ src,
                                           int64_t stride, int n, int vec) {
  if (vec) {
    constexpr int U = 12, C4 = DH / 4;
    const int n4 = n * C4;
    for (int e0 = threadIdx.x; e0 < n4; e0 += U * kDaThreads) {
      f32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = e0 + u * kDaThreads;
        const int r = e / C4, c4 = e - r * C4;
        v[u] = e < n4 ? *reinterpret_cast<const f32x4*>(src + (int64_t)r * stride + 4 * c4)
                      : f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = e0 + u * kDaThreads;
        if (e < n4) *reinterpret_cast<f32x4*>(dst + 4 * e) = v[u];
      }
    }
    return;
  }
  constexpr int U = 40;
  for (int e0 = threadIdx.x; e0 < n * DH; e0 += U * kDaThreads) {
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = e0 + u * kDaThreads;
      const int r = e / DH, c = e - r * DH;
      v[u] = e < n * DH ? src[(int64_t)r * stride + c] : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = e0 + u * kDaThreads;
      if (e < n * DH) dst[e] = v[u];  // (r * DH + c == e)
    }
  }
}

// The fp32 chains of these helpers run two lanes of a v_pk_fma_f32 at a time: the same
// operations in the same order as their scalar forms (the same bits), half the VALU issue.

// dot of an LDS row (float4 broadcast reads) with a register row: four chains (c mod 4),
// fixed order, as the halves of two packed accumulators
template <int DH>
__device__ __forceinline__ float dot_row(const float* __restrict__ row, const float (&x)[DH]) {
  f32x2 d01 = f32x2{0.f, 0.f}, d23 = f32x2{0.f, 0.f};
#pragma unroll
  for (int c = 0; c < DH; c += 4) {
    const f32x4 r4 = *reinterpret_cast<const f32x4*>(row + c);
    d01 = __builtin_elementwise_fma(f32x2{r4[0], r4[1]}, f32x2{x[c], x[c + 1]}, d01);
    d23 = __builtin_elementwise_fma(f32x2{r4[2], r4[3]}, f32x2{x[c + 2], x[c + 3]}, d23);
  }
  return (d01[0] + d01[1]) + (d23[0] + d23[1]);
}

// out[0..3] = sum_j w[j] * M[j][c4 .. c4+3] for j < Lk: w an LDS row (pitch >= Lk, 16-byte
// aligned), M an LDS [Lk][DH] image; per column two interleaved partial sums (even / odd j)
// added in a fixed order; 4 keys per step (one float4 of w, four of M)
template <int DH>
__device__ __forceinline__ f32x4 row_times_cols4(const float* __restrict__ w,
                                                 const float* __restrict__ M, int c4, int Lk) {
  f32x2 a0l = f32x2{0.f, 0.f}, a0h = a0l, a1l = a0l, a1h = a0l;  // columns (0,1), (2,3)
  auto lo = [](const f32x4& v) { return f32x2{v[0], v[1]}; };
  auto hi = [](const f32x4& v) { return f32x2{v[2], v[3]}; };
  int jj = 0;
#pragma unroll 2
  for (; jj + 4 <= Lk; jj += 4) {
    const f32x4 w4 = *reinterpret_cast<const f32x4*>(w + jj);
    const f32x4 m0 = *reinterpret_cast<const f32x4*>(M + jj * DH + c4);
    const f32x4 m1 = *reinterpret_cast<const f32x4*>(M + (jj + 1) * DH + c4);
    const f32x4 m2 = *reinterpret_cast<const f32x4*>(M + (jj + 2) * DH + c4);
    const f32x4 m3 = *reinterpret_cast<const f32x4*>(M + (jj + 3) * DH + c4);
    const f32x2 w0 = f32x2{w4[0], w4[0]}, w1 = f32x2{w4[1], w4[1]};
    const f32x2 w2 = f32x2{w4[2], w4[2]}, w3 = f32x2{w4[3], w4[3]};
    a0l = __builtin_elementwise_fma(w0, lo(m0), a0l);
    a0h = __builtin_elementwise_fma(w0, hi(m0), a0h);
    a1l = __builtin_elementwise_fma(w1, lo(m1), a1l);
    a1h = __builtin_elementwise_fma(w1, hi(m1), a1h);
    a0l = __builtin_elementwise_fma(w2, lo(m2), a0l);
    a0h = __builtin_elementwise_fma(w2, hi(m2), a0h);
    a1l = __builtin_elementwise_fma(w3, lo(m3), a1l);
    a1h = __builtin_elementwise_fma(w3, hi(m3), a1h);
  }
  for (; jj < Lk; ++jj) {
    const f32x4 m = *reinterpret_cast<const f32x4*>(M + jj * DH + c4);
    const f32x2 ww = f32x2{w[jj], w[jj]};
    a0l = __builtin_elementwise_fma(ww, lo(m), a0l);
    a0h = __builtin_elementwise_fma(ww, hi(m), a0h);
  }
  const f32x2 sl = a0l + a1l, sh = a0h + a1h;
  return f32x4{sl[0], sl[1], sh[0], sh[1]};
}

// ------------------------------------------------------------------------------------
// Forward: block = (batch row b, head h, 16-query tile). LDS: Q [16][DH], V [Lk][DH],
// S [16][Lkp]. Thread j = key j for the scores (its k row in registers, from global).
// ------------------------------------------------------------------------------------
template <int DH>
__global__ __launch_bounds__(kDaThreads) void decattn_fwd_kernel(DaArgs a, float* __restrict__ probs,
                                                                 float* __restrict__ ctx) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int Lq = a.Lq, Lk = a.Lk, H = a.H;
  const int nqt = (Lq + kDaQT - 1) / kDaQT;
  // XCD-aware: the query tiles of one (b, h) -- which read the same k / v rows -- are dealt
  // to one XCD (consecutive logical ids share an XCD under round-robin dispatch)
  const int L = xcd_logical_da((int)blockIdx.x, (int)gridDim.x);
  const int qt = L % nqt, bhi = L / nqt;
  const int b = bhi / H, h = bhi - b * H;
  const int i0 = qt * kDaQT, nq = min(kDaQT, Lq - i0);
  const int Lkp = lk_pitch(Lk);
  float* Qs = lds;
  float* Vs = Qs + kDaQT * DH;
  float* S = Vs + Lk * DH;
  stage_rows<DH>(Qs, a.q + ((int64_t)b * Lq + i0) * a.sq + h * DH, a.sq, nq, a.vec);
  stage_rows<DH>(Vs, a.v + (int64_t)b * Lk * a.sv + h * DH, a.sv, Lk, a.vec);
  const int j = threadIdx.x;
  float kr[DH];
  if (j < Lk) {
    const float* kp = a.k + ((int64_t)b * Lk + j) * a.sk + h * DH;
    if (a.vec) {  // 16-byte aligned rows: DH/4 dwordx4 loads
#pragma unroll
      for (int c = 0; c < DH; c += 4) {
        const f32x4 k4 = *reinterpret_cast<const f32x4*>(kp + c);
        kr[c] = k4[0];
        kr[c + 1] = k4[1];
        kr[c + 2] = k4[2];
        kr[c + 3] = k4[3];
      }
    } else {
#pragma unroll
      for (int c = 0; c < DH; ++c) kr[c] = kp[c];
    }
  }
  __syncthreads();

  // scores (the key-padding bit is loaded once per thread, with the k row)
  if (j < Lk) {
    const bool kpad = a.kmask && a.kmask[(int64_t)b * Lk + j];
    for (int il = 0; il < nq; ++il) {
      const float s = dot_row<DH>(Qs + il * DH, kr) * a.scale;
      S[il * Lkp + j] = (kpad || (a.causal && j > i0 + il)) ? -INFINITY : s;
    }
  } else if (j < Lkp) {
    for (int il = 0; il < nq; ++il) S[il * Lkp + j] = 0.0f;  // pad: adds 0 below
  }
  __syncthreads();

  // softmax + dropout per row: wave w takes rows w, w+4, ...; lanes over keys
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t dkey = a.dc.on ? drop_key(a.rng[0], a.rng[1] + a.rng_off) : 0u;
  const int64_t bh = (int64_t)b * H + h;
  for (int il = w; il < nq; il += kDaThreads / 64) {
    const int i = i0 + il;
    float* row = S + il * Lkp;
    float mx = -INFINITY;
    for (int jj = lane; jj < Lk; jj += 64) mx = fmaxf(mx, row[jj]);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    float sum = 0.0f;
    for (int jj = lane; jj < Lk; jj += 64) {
      const float e = expf(row[jj] - mx);  // all -inf: exp(NaN) = NaN, as torch
      row[jj] = e;
      sum += e;
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) sum += __shfl_xor(sum, o);
    float* prow = probs + (bh * Lq + i) * Lk;
    for (int jj = lane; jj < Lk; jj += 64) {
      const float p = row[jj] / sum;
      bool keep = true;
      if (a.dc.on) keep = drop_keep(dkey, (uint64_t)((bh * Lq + i) * Lk + jj), a.dc.thresh);
      prow[jj] = keep ? p : -p;
      row[jj] = a.dc.on ? (keep ? p * a.dc.scale : 0.0f) : p;
    }
  }
  __syncthreads();

  // ctx[i][c] = sum_j Ad[i][j] v[j][c], four columns per task
  const int e = H * DH;
  constexpr int CG = DH / 4;
  for (int o = threadIdx.x; o < nq * CG; o += kDaThreads) {
    const int il = o / CG, c4 = 4 * (o - il * CG);
    const f32x4 r = row_times_cols4<DH>(S + il * Lkp, Vs, c4, Lk);
    *reinterpret_cast<f32x4*>(ctx + ((int64_t)b * Lq + i0 + il) * e + h * DH + c4) = r;
  }
}

// ------------------------------------------------------------------------------------
// Backward: block = (b, h). LDS: Q, dO [Lq][DH], delta [Lq]. The softmax
// backward's row term sum_j A_ij dA_ij equals delta_i = dO_i . ctx_i (ctx = Ad v), formed
// first, so thread j (= key j) finishes its column in one pass over the queries: dA, dS',
// its dv and dk rows (no partials: every query of the head is in the block).
// ------------------------------------------------------------------------------------
// dq is a second launch (decattn_dq_kernel): each dS'[i][j] goes from the thread of key j
// straight over P[i][j] in the probs buffer (consumed). The block's LDS is then Q, dO and
// delta (12 KB at Lq = 41, dh = 36) and P streams through registers: two blocks per CU (174
// VGPRs), every (b, h) of the training step resident at once, where the P and K images of
// the fused form (77 KB more) held it to one block -- one wave per SIMD, every LDS and
// memory latency of the per-key query walk exposed (91 us for the cross-attention).
template <int DH>
__global__ __launch_bounds__(kDaThreads) void decattn_bwd_kernel(
    DaArgs a, const float* __restrict__ dctx, const float* __restrict__ ctxo,
    float* __restrict__ probs, float* __restrict__ dq, int64_t gq, float* __restrict__ dk,
    int64_t gk, float* __restrict__ dv, int64_t gv) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int b = blockIdx.x / a.H, h = blockIdx.x - b * a.H;
  const int Lq = a.Lq, Lk = a.Lk, H = a.H;
  const int e = H * DH;
  float* Qs = lds;
  float* Os = Qs + Lq * DH;
  float* delta = Os + Lq * DH;  // [Lq]
  const int64_t bh = (int64_t)b * H + h;
  const int j = threadIdx.x;
  const bool live = j < Lk;
  // The prologue's global reads -- this thread's v row, the ctx / dO rows of delta_j (j < Lq)
  // and its share of the Q / dO images -- are all issued before the first is used: one
  // memory latency, not four.
  float vr[DH], cr[DH], orr[DH];
  const float* qsrc = a.q + (int64_t)b * Lq * a.sq + h * DH;
  const float* osrc = dctx + (int64_t)b * Lq * e + h * DH;
  constexpr int C4 = DH / 4;
  constexpr int kSt = 2;  // Q / dO image units (float4) per thread and source, vec path
  const bool fast = a.vec && Lq * C4 <= kSt * kDaThreads;
  {
    const float* vp = a.v + ((int64_t)b * Lk + (live ? j : 0)) * a.sv + h * DH;
    const int jq = j < Lq ? j : 0;
    const float* cp = ctxo + ((int64_t)b * Lq + jq) * e + h * DH;
    const float* op = osrc + (int64_t)jq * e;
    if (a.vec) {
      f32x4 qv[kSt], ov[kSt];
      if (fast) {
#pragma unroll
        for (int u = 0; u < kSt; ++u) {
          const int t = threadIdx.x + u * kDaThreads;
          const int r = t / C4, c4 = t - r * C4;
          const int rr = r < Lq ? r : 0;
          qv[u] = *reinterpret_cast<const f32x4*>(qsrc + (int64_t)rr * a.sq + 4 * c4);
          ov[u] = *reinterpret_cast<const f32x4*>(osrc + (int64_t)rr * e + 4 * c4);
        }
      }
#pragma unroll
      for (int c = 0; c < DH; c += 4) {
        const f32x4 v4 = *reinterpret_cast<const f32x4*>(vp + c);
        const f32x4 c4v = *reinterpret_cast<const f32x4*>(cp + c);
        const f32x4 o4 = *reinterpret_cast<const f32x4*>(op + c);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          vr[c + q] = live ? v4[q] : 0.0f;
          cr[c + q] = c4v[q];
          orr[c + q] = o4[q];
        }
      }
      if (fast) {
#pragma unroll
        for (int u = 0; u < kSt; ++u) {
          const int t = threadIdx.x + u * kDaThreads;
          if (t < Lq * C4) {
            *reinterpret_cast<f32x4*>(Qs + 4 * t) = qv[u];
            *reinterpret_cast<f32x4*>(Os + 4 * t) = ov[u];
          }
        }
      }
    } else {
#pragma unroll
      for (int c = 0; c < DH; ++c) {
        vr[c] = live ? vp[c] : 0.0f;
        cr[c] = cp[c];
        orr[c] = op[c];
      }
    }
  }
  if (!fast) {
    stage_rows<DH>(Qs, qsrc, a.sq, Lq, a.vec);
    stage_rows<DH>(Os, osrc, e, Lq, a.vec);
  }
  if (j < Lq) {  // delta_j = dO_j . ctx_j (row j of this head)
    float d0 = 0.0f, d1 = 0.0f, d2 = 0.0f, d3 = 0.0f;
#pragma unroll
    for (int c = 0; c < DH; c += 4) {
      d0 = fmaf(orr[c], cr[c], d0);
      d1 = fmaf(orr[c + 1], cr[c + 1], d1);
      d2 = fmaf(orr[c + 2], cr[c + 2], d2);
      d3 = fmaf(orr[c + 3], cr[c + 3], d3);
    }
    delta[j] = (d0 + d1) + (d2 + d3);
  }
  __syncthreads();

  if (live) {
    // Every fp32 chain below is the scalar form's, two lanes of a v_pk_fma_f32 at a time
    // (the kernel is VALU-bound: 108 fma per query and key): the dot product's chains
    // (c mod 4) are the two halves of two packed accumulators, the dv / dk rows pairs of
    // columns. The same operations in the same order: the same bits.
    f32x2 gv2[DH / 2], gk2[DH / 2], vr2[DH / 2];
#pragma unroll
    for (int c = 0; c < DH / 2; ++c) {
      gv2[c] = f32x2{0.f, 0.f};
      gk2[c] = f32x2{0.f, 0.f};
      vr2[c] = f32x2{vr[2 * c], vr[2 * c + 1]};
    }
    // P[i][j] straight from the probs buffer, kPRing rows ahead in a register ring (coalesced
    // across the block's threads); dS'[i][j] is written back over P[i][j] after it is read.
    // The loop is unrolled by kPRing so every ring index is static; the loads are clamped to
    // the last row (a clamped value is never used).
    constexpr int kPRing = 4;
    float* pcol = probs + bh * Lq * Lk + j;
    float pr[kPRing];
#pragma unroll
    for (int u = 0; u < kPRing; ++u) pr[u] = pcol[(int64_t)(u < Lq - 1 ? u : Lq - 1) * Lk];
    for (int i0 = 0; i0 < Lq; i0 += kPRing) {
#pragma unroll
      for (int u = 0; u < kPRing; ++u) {
        const int i = i0 + u;
        if (i >= Lq) break;
        f32x2 o2[DH / 2];
#pragma unroll
        for (int c = 0; c < DH; c += 4) {
          const f32x4 r4 = *reinterpret_cast<const f32x4*>(Os + i * DH + c);
          o2[c / 2] = f32x2{r4[0], r4[1]};
          o2[c / 2 + 1] = f32x2{r4[2], r4[3]};
        }
        f32x2 d01 = f32x2{0.f, 0.f}, d23 = f32x2{0.f, 0.f};  // dAd = dO_i . v_j
#pragma unroll
        for (int c = 0; c < DH / 2; c += 2) {
          d01 = __builtin_elementwise_fma(o2[c], vr2[c], d01);
          d23 = __builtin_elementwise_fma(o2[c + 1], vr2[c + 1], d23);
        }
        const float d = (d01[0] + d01[1]) + (d23[0] + d23[1]);
        const float pv = pr[u];
        const bool keep = !__builtin_signbit(pv);
        const float A = fabsf(pv);
        const float dA = a.dc.on ? (keep ? d * a.dc.scale : 0.0f) : d;
        const float Ad = a.dc.on ? (keep ? A * a.dc.scale : 0.0f) : A;
        const float ds = (A * (dA - delta[i])) * a.scale;
        pcol[(int64_t)i * Lk] = ds;
        pr[u] = pcol[(int64_t)(i + kPRing < Lq - 1 ? i + kPRing : Lq - 1) * Lk];
        const f32x2 ad2 = f32x2{Ad, Ad}, ds2 = f32x2{ds, ds};
#pragma unroll
        for (int c = 0; c < DH / 2; ++c) gv2[c] = __builtin_elementwise_fma(ad2, o2[c], gv2[c]);
#pragma unroll
        for (int c = 0; c < DH; c += 4) {
          const f32x4 q4 = *reinterpret_cast<const f32x4*>(Qs + i * DH + c);
          gk2[c / 2] = __builtin_elementwise_fma(ds2, f32x2{q4[0], q4[1]}, gk2[c / 2]);
          gk2[c / 2 + 1] = __builtin_elementwise_fma(ds2, f32x2{q4[2], q4[3]}, gk2[c / 2 + 1]);
        }
        __builtin_amdgcn_sched_barrier(0);  // (one query's operands live at a time)
      }
    }
#pragma unroll
    for (int c = 0; c < DH; ++c) {
      dv[((int64_t)b * Lk + j) * gv + h * DH + c] = gv2[c / 2][c % 2];
      dk[((int64_t)b * Lk + j) * gk + h * DH + c] = gk2[c / 2][c % 2];
    }
  }
}

// dq[i][c] = sum_j dS'[i][j] k[j][c]: block = (b, h, qtile-query tile; dq_tile: every query
// of the decoder's 41-token rows in one block when K is long, so K is staged once per (b, h),
// 16-query tiles when it is short); LDS: K [Lk][DH] and the tile's dS' rows
// [min(qtile, Lq)][Lkp] (from the probs buffer, zero-padded to the pitch); four columns per
// task (row_times_cols4's fixed order).
inline int dq_tile(int Lk) { return Lk > 64 ? 48 : 16; }
template <int DH>
__global__ __launch_bounds__(kDaThreads) void decattn_dq_kernel(DaArgs a,
                                                                const float* __restrict__ dsp,
                                                                float* __restrict__ dq, int64_t gq,
                                                                int qtile) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int Lq = a.Lq, Lk = a.Lk, H = a.H;
  const int nqt = (Lq + qtile - 1) / qtile;
  const int L = xcd_logical_da((int)blockIdx.x, (int)gridDim.x);  // a (b, h)'s tiles on one XCD
  const int qt = L % nqt, bhi = L / nqt;
  const int b = bhi / H, h = bhi - b * H;
  const int i0 = qt * qtile, nq = min(qtile, Lq - i0);
  const int Lkp = lk_pitch(Lk);
  float* Ks = lds;
  float* S = Ks + Lk * DH;  // [nq][Lkp]
  stage_rows<DH>(Ks, a.k + (int64_t)b * Lk * a.sk + h * DH, a.sk, Lk, a.vec);
  // dS' rows: 8 loads per thread in flight per pass, then their stores
  const float* src = dsp + ((int64_t)bhi * Lq + i0) * Lk;
  constexpr int kU = 8;
  for (int t0 = threadIdx.x; t0 < nq * Lkp; t0 += kU * kDaThreads) {
    float pv[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int t = t0 + u * kDaThreads;
      const int i = t / Lkp, jj = t - i * Lkp;
      pv[u] = (t < nq * Lkp && jj < Lk) ? src[(int64_t)i * Lk + jj] : 0.0f;  // pads: 0
    }
#pragma unroll
    for (int u = 0; u < kU; ++u)
      if (t0 + u * kDaThreads < nq * Lkp) S[t0 + u * kDaThreads] = pv[u];
  }
  __syncthreads();
  constexpr int CG = DH / 4;
  for (int o = threadIdx.x; o < nq * CG; o += kDaThreads) {
    const int il = o / CG, c4 = 4 * (o - il * CG);
    const f32x4 r = row_times_cols4<DH>(S + il * Lkp, Ks, c4, Lk);
    float* dst = dq + ((int64_t)b * Lq + i0 + il) * gq + h * DH + c4;
    dst[0] = r[0];
    dst[1] = r[1];
    dst[2] = r[2];
    dst[3] = r[3];
  }
}

template <int DH>
size_t fwd_lds(int Lq, int Lk) {
  (void)Lq;
  return sizeof(float) * ((size_t)(kDaQT + Lk) * DH + (size_t)kDaQT * lk_pitch(Lk));
}
template <int DH>
size_t bwd_lds(int Lq, int Lk) {
  (void)Lk;
  return sizeof(float) * ((size_t)(2 * Lq) * DH + (size_t)Lq);
}
template <int DH>
size_t dq_lds(int Lq, int Lk) {
  return sizeof(float) * ((size_t)Lk * DH + (size_t)std::min(dq_tile(Lk), Lq) * lk_pitch(Lk));
}

constexpr size_t kDaMaxLds = 160 * 1024;

inline int da_vec(const float* q, int64_t sq, const float* k, int64_t sk, const float* v,
                  int64_t sv) {
  auto al = [](const float* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  return (al(q) && al(k) && al(v) && sq % 4 == 0 && sk % 4 == 0 && sv % 4 == 0) ? 1 : 0;
}

#define OB_DA_DISPATCH(MACRO) \
  switch (dh) {               \
    case 16: MACRO(16); break; \
    case 32: MACRO(32); break; \
    case 36: MACRO(36); break; \
    case 64: MACRO(64); break; \
    default: break;           \
  }

}  // namespace

bool decattn_supported(int64_t Lq, int64_t Lk, int64_t dh) {
  if (Lq < 1 || Lk < 1 || Lk > kDaThreads) return false;
  size_t need = 0;
#define OB_DA_NEED(D) \
  need = std::max(fwd_lds<D>((int)Lq, (int)Lk), std::max(bwd_lds<D>((int)Lq, (int)Lk), dq_lds<D>((int)Lq, (int)Lk)))
  OB_DA_DISPATCH(OB_DA_NEED)
#undef OB_DA_NEED
  return need > 0 && need <= kDaMaxLds;
}

void launch_decattn_fwd(const float* q, int64_t sq, const float* k, int64_t sk, const float* v,
                        int64_t sv, const uint8_t* kmask, int causal, int64_t B, int64_t H,
                        int64_t Lq, int64_t Lk, int64_t dh, float p_drop, const uint64_t* rng,
                        uint64_t rng_off, float* probs, float* ctx, hipStream_t s) {
  if (B == 0) return;
  DaArgs a{q, k, v, sq, sk, sv, kmask, causal, (int)H, (int)Lq, (int)Lk,
           (float)(1.0 / sqrt((double)dh)), make_drop(p_drop), rng, rng_off,
           da_vec(q, sq, k, sk, v, sv)};
#define OB_DA_FWD(D)                                                                            \
  {                                                                                             \
    const size_t lds = fwd_lds<D>((int)Lq, (int)Lk);                                            \
    hipLaunchKernelGGL(decattn_fwd_kernel<D>, dim3((unsigned)(B * H * ((Lq + kDaQT - 1) / kDaQT))), \
                       dim3(kDaThreads), lds, s,                                                \
                       a, probs, ctx);                                                          \
  }
  OB_DA_DISPATCH(OB_DA_FWD)
#undef OB_DA_FWD
}

void launch_decattn_bwd(const float* dctx, const float* ctxo, const float* q, int64_t sq,
                        const float* k, int64_t sk,
                        const float* v, int64_t sv, int64_t B, int64_t H, int64_t Lq, int64_t Lk,
                        int64_t dh, float p_drop, float* probs, float* dq, int64_t gq,
                        float* dk, int64_t gk, float* dv, int64_t gv, hipStream_t s) {
  if (B == 0) return;
  DaArgs a{q, k, v, sq, sk, sv, nullptr, 0, (int)H, (int)Lq, (int)Lk,
           (float)(1.0 / sqrt((double)dh)), make_drop(p_drop), nullptr, 0,
           da_vec(q, sq, k, sk, v, sv) && (reinterpret_cast<uintptr_t>(dctx) & 15) == 0};
#define OB_DA_BWD(D)                                                                            \
  {                                                                                             \
    const size_t lds = bwd_lds<D>((int)Lq, (int)Lk);                                            \
    hipLaunchKernelGGL(decattn_bwd_kernel<D>, dim3((unsigned)(B * H)), dim3(kDaThreads),          \
                       lds, s, a, dctx, ctxo, probs, dq, gq, dk, gk, dv, gv);                   \
    const size_t lq = dq_lds<D>((int)Lq, (int)Lk);                                              \
    const int qt = dq_tile((int)Lk);                                                            \
    hipLaunchKernelGGL(decattn_dq_kernel<D>, dim3((unsigned)(B * H * ((Lq + qt - 1) / qt))),     \
                       dim3(kDaThreads), lq, s, a, (const float*)probs, dq, gq, qt);            \
  }
  OB_DA_DISPATCH(OB_DA_BWD)
#undef OB_DA_BWD
}

}  // namespace ob
