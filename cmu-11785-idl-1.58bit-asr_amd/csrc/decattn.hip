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

// dot of an LDS row (float4 broadcast reads) with a register row
template <int DH>
__device__ __forceinline__ float dot_row(const float* __restrict__ row, const float (&x)[DH]) {
  float d0 = 0.0f, d1 = 0.0f, d2 = 0.0f, d3 = 0.0f;  // four chains (c mod 4), fixed order
#pragma unroll
  for (int c = 0; c < DH; c += 4) {
    const f32x4 r4 = *reinterpret_cast<const f32x4*>(row + c);
    d0 = fmaf(r4[0], x[c], d0);
    d1 = fmaf(r4[1], x[c + 1], d1);
    d2 = fmaf(r4[2], x[c + 2], d2);
    d3 = fmaf(r4[3], x[c + 3], d3);
  }
  return (d0 + d1) + (d2 + d3);
}

// acc[c] += s * row[c] over an LDS row (float4 broadcast reads)
template <int DH>
__device__ __forceinline__ void axpy_row(float s, const float* __restrict__ row, float (&acc)[DH]) {
#pragma unroll
  for (int c = 0; c < DH; c += 4) {
    const f32x4 r4 = *reinterpret_cast<const f32x4*>(row + c);
    acc[c] = fmaf(s, r4[0], acc[c]);
    acc[c + 1] = fmaf(s, r4[1], acc[c + 1]);
    acc[c + 2] = fmaf(s, r4[2], acc[c + 2]);
    acc[c + 3] = fmaf(s, r4[3], acc[c + 3]);
  }
}

// out[0..3] = sum_j w[j] * M[j][c4 .. c4+3] for j < Lk: w an LDS row (pitch >= Lk, 16-byte
// aligned), M an LDS [Lk][DH] image; per column two interleaved partial sums (even / odd j)
// added in a fixed order; 4 keys per step (one float4 of w, four of M)
template <int DH>
__device__ __forceinline__ f32x4 row_times_cols4(const float* __restrict__ w,
                                                 const float* __restrict__ M, int c4, int Lk) {
  f32x4 a0 = f32x4{0.f, 0.f, 0.f, 0.f}, a1 = a0;
  int jj = 0;
  for (; jj + 4 <= Lk; jj += 4) {
    const f32x4 w4 = *reinterpret_cast<const f32x4*>(w + jj);
    const f32x4 m0 = *reinterpret_cast<const f32x4*>(M + jj * DH + c4);
    const f32x4 m1 = *reinterpret_cast<const f32x4*>(M + (jj + 1) * DH + c4);
    const f32x4 m2 = *reinterpret_cast<const f32x4*>(M + (jj + 2) * DH + c4);
    const f32x4 m3 = *reinterpret_cast<const f32x4*>(M + (jj + 3) * DH + c4);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      a0[q] = fmaf(w4[0], m0[q], a0[q]);
      a1[q] = fmaf(w4[1], m1[q], a1[q]);
      a0[q] = fmaf(w4[2], m2[q], a0[q]);
      a1[q] = fmaf(w4[3], m3[q], a1[q]);
    }
  }
  for (; jj < Lk; ++jj) {
    const f32x4 m = *reinterpret_cast<const f32x4*>(M + jj * DH + c4);
#pragma unroll
    for (int q = 0; q < 4; ++q) a0[q] = fmaf(w[jj], m[q], a0[q]);
  }
  return a0 + a1;
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
// Backward: block = (b, h). LDS: Q, dO [Lq][DH], K [Lk][DH], S = P then dS' [Lq][Lkp],
// delta [Lq]. The softmax backward's row term sum_j A_ij dA_ij equals delta_i = dO_i . ctx_i
// (ctx = Ad v), formed first, so thread j (= key j) finishes its column in one pass over
// the queries: dA, dS', its dv and dk rows (no partials: every query of the head is in the
// block); dq then reads the dS' image.
// ------------------------------------------------------------------------------------
template <int DH>
__global__ __launch_bounds__(kDaThreads) void decattn_bwd_kernel(
    DaArgs a, const float* __restrict__ dctx, const float* __restrict__ ctxo,
    const float* __restrict__ probs, float* __restrict__ dq, int64_t gq, float* __restrict__ dk,
    int64_t gk, float* __restrict__ dv, int64_t gv) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int b = blockIdx.x / a.H, h = blockIdx.x - b * a.H;
  const int Lq = a.Lq, Lk = a.Lk, H = a.H;
  const int Lkp = lk_pitch(Lk);
  const int e = H * DH;
  float* Qs = lds;
  float* Os = Qs + Lq * DH;
  float* Ks = Os + Lq * DH;
  float* S = Ks + Lk * DH;
  float* delta = S + Lq * Lkp;  // [Lq]
  const int64_t bh = (int64_t)b * H + h;
  stage_rows<DH>(Qs, a.q + (int64_t)b * Lq * a.sq + h * DH, a.sq, Lq, a.vec);
  stage_rows<DH>(Os, dctx + (int64_t)b * Lq * e + h * DH, e, Lq, a.vec);
  stage_rows<DH>(Ks, a.k + (int64_t)b * Lk * a.sk + h * DH, a.sk, Lk, a.vec);
  for (int t0 = threadIdx.x; t0 < Lq * Lkp; t0 += 8 * kDaThreads) {
    float pv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int t = t0 + u * kDaThreads;
      const int i = t / Lkp, jj = t - i * Lkp;
      pv[u] = (t < Lq * Lkp && jj < Lk) ? probs[(bh * Lq + i) * Lk + jj] : 0.0f;  // pads: 0
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (t0 + u * kDaThreads < Lq * Lkp) S[t0 + u * kDaThreads] = pv[u];
  }
  const int j = threadIdx.x;
  const bool live = j < Lk;
  float vr[DH];
  {
    const float* vp = a.v + ((int64_t)b * Lk + (live ? j : 0)) * a.sv + h * DH;
    if (a.vec) {
#pragma unroll
      for (int c = 0; c < DH; c += 4) {
        const f32x4 v4 = *reinterpret_cast<const f32x4*>(vp + c);
        vr[c] = live ? v4[0] : 0.0f;
        vr[c + 1] = live ? v4[1] : 0.0f;
        vr[c + 2] = live ? v4[2] : 0.0f;
        vr[c + 3] = live ? v4[3] : 0.0f;
      }
    } else {
#pragma unroll
      for (int c = 0; c < DH; ++c) vr[c] = live ? vp[c] : 0.0f;
    }
  }
  if (j < Lq) {  // delta_j = dO_j . ctx_j (row j of this head)
    const float* cr = ctxo + ((int64_t)b * Lq + j) * e + h * DH;
    const float* orow = dctx + ((int64_t)b * Lq + j) * e + h * DH;
    float d0 = 0.0f, d1 = 0.0f, d2 = 0.0f, d3 = 0.0f;
#pragma unroll
    for (int c = 0; c < DH; c += 4) {
      d0 = fmaf(orow[c], cr[c], d0);
      d1 = fmaf(orow[c + 1], cr[c + 1], d1);
      d2 = fmaf(orow[c + 2], cr[c + 2], d2);
      d3 = fmaf(orow[c + 3], cr[c + 3], d3);
    }
    delta[j] = (d0 + d1) + (d2 + d3);
  }
  __syncthreads();

  if (live) {
    float gv_[DH], gk_[DH];
#pragma unroll
    for (int c = 0; c < DH; ++c) {
      gv_[c] = 0.0f;
      gk_[c] = 0.0f;
    }
    for (int i = 0; i < Lq; ++i) {
      float o[DH];
#pragma unroll
      for (int c = 0; c < DH; c += 4) {
        const f32x4 r4 = *reinterpret_cast<const f32x4*>(Os + i * DH + c);
        o[c] = r4[0];
        o[c + 1] = r4[1];
        o[c + 2] = r4[2];
        o[c + 3] = r4[3];
      }
      float d0 = 0.0f, d1 = 0.0f, d2 = 0.0f, d3 = 0.0f;  // dAd = dO_i . v_j
#pragma unroll
      for (int c = 0; c < DH; c += 4) {
        d0 = fmaf(o[c], vr[c], d0);
        d1 = fmaf(o[c + 1], vr[c + 1], d1);
        d2 = fmaf(o[c + 2], vr[c + 2], d2);
        d3 = fmaf(o[c + 3], vr[c + 3], d3);
      }
      const float d = (d0 + d1) + (d2 + d3);
      const float pv = S[i * Lkp + j];
      const bool keep = !__builtin_signbit(pv);
      const float A = fabsf(pv);
      const float dA = a.dc.on ? (keep ? d * a.dc.scale : 0.0f) : d;
      const float Ad = a.dc.on ? (keep ? A * a.dc.scale : 0.0f) : A;
      const float ds = (A * (dA - delta[i])) * a.scale;
      S[i * Lkp + j] = ds;
#pragma unroll
      for (int c = 0; c < DH; ++c) gv_[c] = fmaf(Ad, o[c], gv_[c]);
      axpy_row<DH>(ds, Qs + i * DH, gk_);
    }
#pragma unroll
    for (int c = 0; c < DH; ++c) {
      dv[((int64_t)b * Lk + j) * gv + h * DH + c] = gv_[c];
      dk[((int64_t)b * Lk + j) * gk + h * DH + c] = gk_[c];
    }
  }
  __syncthreads();
  // dq[i][c] = sum_j dS'[i][j] k[j][c], four columns per task
  constexpr int CG = DH / 4;
  for (int o = threadIdx.x; o < Lq * CG; o += kDaThreads) {
    const int i = o / CG, c4 = 4 * (o - i * CG);
    const f32x4 r = row_times_cols4<DH>(S + i * Lkp, Ks, c4, Lk);
    float* dst = dq + ((int64_t)b * Lq + i) * gq + h * DH + c4;
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
  return sizeof(float) * ((size_t)(2 * Lq + Lk) * DH + (size_t)Lq * lk_pitch(Lk) + (size_t)Lq);
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
#define OB_DA_NEED(D) need = fwd_lds<D>((int)Lq, (int)Lk) > bwd_lds<D>((int)Lq, (int)Lk) ? fwd_lds<D>((int)Lq, (int)Lk) : bwd_lds<D>((int)Lq, (int)Lk)
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
                        int64_t dh, float p_drop, const float* probs, float* dq, int64_t gq,
                        float* dk, int64_t gk, float* dv, int64_t gv, hipStream_t s) {
  if (B == 0) return;
  DaArgs a{q, k, v, sq, sk, sv, nullptr, 0, (int)H, (int)Lq, (int)Lk,
           (float)(1.0 / sqrt((double)dh)), make_drop(p_drop), nullptr, 0,
           da_vec(q, sq, k, sk, v, sv) && (reinterpret_cast<uintptr_t>(dctx) & 15) == 0};
#define OB_DA_BWD(D)                                                                            \
  {                                                                                             \
    const size_t lds = bwd_lds<D>((int)Lq, (int)Lk);                                            \
    hipLaunchKernelGGL(decattn_bwd_kernel<D>, dim3((unsigned)(B * H)), dim3(kDaThreads), lds, s, \
                       a, dctx, ctxo, probs, dq, gq, dk, gk, dv, gv);                                 \
  }
  OB_DA_DISPATCH(OB_DA_BWD)
#undef OB_DA_BWD
}

}  // namespace ob
