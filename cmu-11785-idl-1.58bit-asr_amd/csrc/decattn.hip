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
};

template <int DH>
struct DaLds {
  static constexpr int P = DH + 1;  // odd row pitch: per-lane rows hit distinct banks
};

__device__ __forceinline__ bool key_masked(const DaArgs& a, int b, int i, int j) {
  return (a.kmask && a.kmask[(int64_t)b * a.Lk + j]) || (a.causal && j > i);
}

// rows [0, n) of a strided [rows][*] tensor's head slice into an LDS [n][DH + 1] image
template <int DH>
__device__ __forceinline__ void stage_rows(float* __restrict__ dst, const float* __restrict__ src,
                                           int64_t stride, int n) {
  for (int e = threadIdx.x; e < n * DH; e += kDaThreads) {
    const int r = e / DH, c = e - r * DH;
    dst[r * DaLds<DH>::P + c] = src[(int64_t)r * stride + c];
  }
}

// ------------------------------------------------------------------------------------
// Forward: block = (batch row b, head h). LDS: Q [Lq][DH+1], K, V [Lk][DH+1], S [Lq][Lk].
// ------------------------------------------------------------------------------------
template <int DH>
__global__ __launch_bounds__(kDaThreads) void decattn_fwd_kernel(DaArgs a, float* __restrict__ probs,
                                                                 float* __restrict__ ctx) {
  constexpr int P = DaLds<DH>::P;
  extern __shared__ float lds[];
  const int b = blockIdx.x / a.H, h = blockIdx.x - b * a.H;
  const int Lq = a.Lq, Lk = a.Lk, H = a.H;
  float* Qs = lds;
  float* Ks = Qs + Lq * P;
  float* Vs = Ks + Lk * P;
  float* S = Vs + Lk * P;
  stage_rows<DH>(Qs, a.q + (int64_t)b * Lq * a.sq + h * DH, a.sq, Lq);
  stage_rows<DH>(Ks, a.k + (int64_t)b * Lk * a.sk + h * DH, a.sk, Lk);
  stage_rows<DH>(Vs, a.v + (int64_t)b * Lk * a.sv + h * DH, a.sv, Lk);
  __syncthreads();

  // scores: thread j = key j, its k row in registers, q rows broadcast from LDS
  const int j = threadIdx.x;
  if (j < Lk) {
    float kr[DH];
#pragma unroll
    for (int c = 0; c < DH; ++c) kr[c] = Ks[j * P + c];
    for (int i = 0; i < Lq; ++i) {
      float d = 0.0f;
#pragma unroll
      for (int c = 0; c < DH; ++c) d = fmaf(Qs[i * P + c], kr[c], d);
      const float s = d * a.scale;
      S[i * Lk + j] = key_masked(a, b, i, j) ? -INFINITY : s;
    }
  }
  __syncthreads();

  // softmax + dropout per row: wave w takes rows w, w+4, ...; lanes over keys
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t dkey = a.dc.on ? drop_key(a.rng[0], a.rng[1] + a.rng_off) : 0u;
  const int64_t bh = (int64_t)b * H + h;
  for (int i = w; i < Lq; i += kDaThreads / 64) {
    float* row = S + i * Lk;
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

  // ctx[i][c] = sum_j Ad[i][j] v[j][c]
  const int e = H * DH;
  for (int o = threadIdx.x; o < Lq * DH; o += kDaThreads) {
    const int i = o / DH, c = o - i * DH;
    const float* row = S + i * Lk;
    float acc = 0.0f;
    for (int jj = 0; jj < Lk; ++jj) acc = fmaf(row[jj], Vs[jj * P + c], acc);
    ctx[((int64_t)b * Lq + i) * e + h * DH + c] = acc;
  }
}

// ------------------------------------------------------------------------------------
// Backward: block = (b, h). LDS: Q, dO [Lq][DH+1], K [Lk][DH+1], S = P then dS' [Lq][Lk],
// DA = dA [Lq][Lk], red [4][Lq]. Thread j owns key j: dA, dv row j, dk row j (no partials:
// every query of the head is in the block); dq from the dS' image.
// ------------------------------------------------------------------------------------
template <int DH>
__global__ __launch_bounds__(kDaThreads) void decattn_bwd_kernel(
    DaArgs a, const float* __restrict__ dctx, const float* __restrict__ probs,
    float* __restrict__ dq, int64_t gq, float* __restrict__ dk, int64_t gk, float* __restrict__ dv,
    int64_t gv) {
  constexpr int P = DaLds<DH>::P;
  extern __shared__ float lds[];
  const int b = blockIdx.x / a.H, h = blockIdx.x - b * a.H;
  const int Lq = a.Lq, Lk = a.Lk, H = a.H;
  const int e = H * DH;
  float* Qs = lds;
  float* Os = Qs + Lq * P;
  float* Ks = Os + Lq * P;
  float* S = Ks + Lk * P;
  float* DA = S + Lq * Lk;
  float* red = DA + Lq * Lk;  // [4][Lq]
  const int64_t bh = (int64_t)b * H + h;
  stage_rows<DH>(Qs, a.q + (int64_t)b * Lq * a.sq + h * DH, a.sq, Lq);
  stage_rows<DH>(Os, dctx + (int64_t)b * Lq * e + h * DH, e, Lq);
  stage_rows<DH>(Ks, a.k + (int64_t)b * Lk * a.sk + h * DH, a.sk, Lk);
  for (int t = threadIdx.x; t < Lq * Lk; t += kDaThreads) S[t] = probs[bh * Lq * Lk + t];
  __syncthreads();

  const int j = threadIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const bool live = j < Lk;
  float acc[DH];
  // dAd = dO v^T (v row j in registers), dA = dropout backward, dv row j = sum_i Ad_ij dO_i,
  // and the softmax-backward row terms sum_j A_ij dA_ij (wave sums, then 4 waves in order)
  {
    float vr[DH];
#pragma unroll
    for (int c = 0; c < DH; ++c) {
      vr[c] = live ? a.v[((int64_t)b * Lk + j) * a.sv + h * DH + c] : 0.0f;
      acc[c] = 0.0f;
    }
    for (int i = 0; i < Lq; ++i) {
      float t = 0.0f;
      if (live) {
        float d = 0.0f;
#pragma unroll
        for (int c = 0; c < DH; ++c) d = fmaf(Os[i * P + c], vr[c], d);
        const float pv = S[i * Lk + j];
        const bool keep = !__builtin_signbit(pv);
        const float A = fabsf(pv);
        const float dA = a.dc.on ? (keep ? d * a.dc.scale : 0.0f) : d;
        const float Ad = a.dc.on ? (keep ? A * a.dc.scale : 0.0f) : A;
        DA[i * Lk + j] = dA;
#pragma unroll
        for (int c = 0; c < DH; ++c) acc[c] = fmaf(Ad, Os[i * P + c], acc[c]);
        t = A * dA;
      }
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) t += __shfl_xor(t, o);
      if (lane == 0) red[w * Lq + i] = t;
    }
  }
  if (live) {
#pragma unroll
    for (int c = 0; c < DH; ++c) dv[((int64_t)b * Lk + j) * gv + h * DH + c] = acc[c];
  }
  __syncthreads();
  // dS' = A (dA - rowsum) * scale (the softmax backward, then the score scale); dk row j
  if (live) {
#pragma unroll
    for (int c = 0; c < DH; ++c) acc[c] = 0.0f;
    for (int i = 0; i < Lq; ++i) {
      const float rs = ((red[i] + red[Lq + i]) + red[2 * Lq + i]) + red[3 * Lq + i];
      const float A = fabsf(S[i * Lk + j]);
      const float ds = (A * (DA[i * Lk + j] - rs)) * a.scale;
      S[i * Lk + j] = ds;
#pragma unroll
      for (int c = 0; c < DH; ++c) acc[c] = fmaf(ds, Qs[i * P + c], acc[c]);
    }
#pragma unroll
    for (int c = 0; c < DH; ++c) dk[((int64_t)b * Lk + j) * gk + h * DH + c] = acc[c];
  }
  __syncthreads();
  // dq[i][c] = sum_j dS'[i][j] k[j][c]
  for (int o = threadIdx.x; o < Lq * DH; o += kDaThreads) {
    const int i = o / DH, c = o - i * DH;
    const float* row = S + i * Lk;
    float s = 0.0f;
    for (int jj = 0; jj < Lk; ++jj) s = fmaf(row[jj], Ks[jj * P + c], s);
    dq[((int64_t)b * Lq + i) * gq + h * DH + c] = s;
  }
}

template <int DH>
size_t fwd_lds(int Lq, int Lk) {
  return sizeof(float) * ((size_t)(Lq + 2 * Lk) * DaLds<DH>::P + (size_t)Lq * Lk);
}
template <int DH>
size_t bwd_lds(int Lq, int Lk) {
  return sizeof(float) * ((size_t)(2 * Lq + Lk) * DaLds<DH>::P + 2 * (size_t)Lq * Lk + 4 * (size_t)Lq);
}

constexpr size_t kDaMaxLds = 160 * 1024;

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
           (float)(1.0 / sqrt((double)dh)), make_drop(p_drop), rng, rng_off};
#define OB_DA_FWD(D)                                                                            \
  {                                                                                             \
    const size_t lds = fwd_lds<D>((int)Lq, (int)Lk);                                            \
    hipLaunchKernelGGL(decattn_fwd_kernel<D>, dim3((unsigned)(B * H)), dim3(kDaThreads), lds, s, \
                       a, probs, ctx);                                                          \
  }
  OB_DA_DISPATCH(OB_DA_FWD)
#undef OB_DA_FWD
}

void launch_decattn_bwd(const float* dctx, const float* q, int64_t sq, const float* k, int64_t sk,
                        const float* v, int64_t sv, int64_t B, int64_t H, int64_t Lq, int64_t Lk,
                        int64_t dh, float p_drop, const float* probs, float* dq, int64_t gq,
                        float* dk, int64_t gk, float* dv, int64_t gv, hipStream_t s) {
  if (B == 0) return;
  DaArgs a{q, k, v, sq, sk, sv, nullptr, 0, (int)H, (int)Lq, (int)Lk,
           (float)(1.0 / sqrt((double)dh)), make_drop(p_drop), nullptr, 0};
#define OB_DA_BWD(D)                                                                            \
  {                                                                                             \
    const size_t lds = bwd_lds<D>((int)Lq, (int)Lk);                                            \
    hipLaunchKernelGGL(decattn_bwd_kernel<D>, dim3((unsigned)(B * H)), dim3(kDaThreads), lds, s, \
                       a, dctx, probs, dq, gq, dk, gk, dv, gv);                                 \
  }
  OB_DA_DISPATCH(OB_DA_BWD)
#undef OB_DA_BWD
}

}  // namespace ob
