// seqloss.hip — the decoder losses of the stacked training step in two row passes.
//
// Reference: onebit_asr/losses.py:22-35 (label-smoothed attention CE with its scalar-mean
// quirk) and :50-59 (KL(teacher || student) over non-pad positions), as train.py:82-111
// uses them for the three passes (teacher 2-bit, student 1-bit, SP). torch evaluates them
// as ~20 kernels per direction over the [P, B, U, V] decoder logits (log_softmax, gather,
// sums, the teacher softmax, kl_div, masks, means). Here, with logits [P*B*U][V] (pass-major
// rows, the teacher's row of position q is row q):
//   fwd (one block per row): m = max x, logs = log sum exp(x - m) (torch's log_softmax:
//     logp = (x - m) - logs); ce_row = -(off * sum_v logp + (1 - ls - off) * logp[target]);
//     for a pass p >= 1 row also kl_row = sum_v pt (log pt - logp) with pt the softmax of
//     the teacher row (its stats recomputed in the same block);
//   reduce (one block, fixed order): l_att[p] = (mean_q ce) * msum / max(msum, 1) (the
//     quirk: the mean over ALL positions, scaled by the non-pad count over itself),
//     l_kl[p-1] = sum_q kl * keep_q / max(ksum, 1);
//   bwd (one block per row): dL/dx_w = w_att * ((off V + c2) sm_w - off - c2 [w == t])
//     + w_kl * keep * (sm_w - pt_w)   (c2 = 1 - ls - off; the teacher is detached).
// Sums are fixed-order block reductions: deterministic.
#include <math.h>

#include "ob_launch.h"

namespace ob {

namespace {

constexpr int kThreads = 256;
constexpr int kMaxQ = 8;  // float4 per thread kept in registers: V <= 8 * 4 * 256
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float block_sum(float v, float* red, bool is_max) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float w = __shfl_xor(v, o);
    v = is_max ? fmaxf(v, w) : v + w;
  }
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  float r = red[0];
#pragma unroll
  for (int w = 1; w < kThreads / 64; ++w) r = is_max ? fmaxf(r, red[w]) : r + red[w];
  return r;
}

// One row (V % 4 == 0, 16-byte aligned) into registers; out-of-range slots hold -inf.
__device__ __forceinline__ void load_row(const float* __restrict__ row, int nq, f32x4 (&v)[kMaxQ]) {
#pragma unroll
  for (int i = 0; i < kMaxQ; ++i) {
    const int q = threadIdx.x + i * kThreads;
    v[i] = q < nq ? reinterpret_cast<const f32x4*>(row)[q]
                  : f32x4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
  }
}

// (max, log sum exp(x - max), sum x) of a register row.
__device__ __forceinline__ void row_stats(const f32x4 (&v)[kMaxQ], int nq, float* red, float& m,
                                          float& logs, float& sx) {
  float a = -INFINITY;
#pragma unroll
  for (int i = 0; i < kMaxQ; ++i)
    a = fmaxf(a, fmaxf(fmaxf(v[i][0], v[i][1]), fmaxf(v[i][2], v[i][3])));
  m = block_sum(a, red, true);
  float s = 0.0f, t = 0.0f;
#pragma unroll
  for (int i = 0; i < kMaxQ; ++i) {
    if ((int)threadIdx.x + i * kThreads >= nq) continue;
    s += ((expf(v[i][0] - m) + expf(v[i][1] - m)) + expf(v[i][2] - m)) + expf(v[i][3] - m);
    t += ((v[i][0] + v[i][1]) + v[i][2]) + v[i][3];
  }
  logs = logf(block_sum(s, red, false));
  sx = block_sum(t, red, false);
}

__global__ __launch_bounds__(kThreads) void att_kl_fwd_kernel(
    const float* __restrict__ x, const int64_t* __restrict__ tgt, int BU, int V, float off,
    float c2, float* __restrict__ stats, float* __restrict__ ce, float* __restrict__ kl) {
  __shared__ float red[kThreads / 64];
  const int r = blockIdx.x, q = r % BU, p = r / BU;
  const int nq = V / 4;
  f32x4 xv[kMaxQ];
  load_row(x + (size_t)r * V, nq, xv);
  float m, logs, sx;
  row_stats(xv, nq, red, m, logs, sx);
  if (threadIdx.x == 0) {
    stats[2 * r] = m;
    stats[2 * r + 1] = logs;
    int64_t t = tgt[q];
    t = t < 0 ? 0 : (t >= V ? V - 1 : t);
    const float sum_logp = (sx - (float)V * m) - (float)V * logs;
    const float tl = (x[(size_t)r * V + t] - m) - logs;
    ce[r] = -(off * sum_logp + c2 * tl);
  }
  if (p == 0) return;
  // KL(pt || p) against the teacher row q: sum pt (lpt - lp)
  f32x4 yv[kMaxQ];
  load_row(x + (size_t)q * V, nq, yv);
  float mt, logst, syt;
  row_stats(yv, nq, red, mt, logst, syt);
  // log pt - log p = (y - x) + c with the row constant c = (m - mt) + (logs - logst): the
  // O(1) difference is rounded instead of two O(log V) log-probabilities (4x less error)
  const float c = (m - mt) + (logs - logst);
  float acc = 0.0f;
#pragma unroll
  for (int i = 0; i < kMaxQ; ++i) {
    if ((int)threadIdx.x + i * kThreads >= nq) continue;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float pt = expf((yv[i][e] - mt) - logst);
      acc += pt == 0.0f ? 0.0f : pt * ((yv[i][e] - xv[i][e]) + c);
    }
  }
  acc = block_sum(acc, red, false);
  if (threadIdx.x == 0) kl[r] = acc;
}

// out[0..P) = l_att, out[P..2P-1) = l_kl; aux[0] = msum, aux[1] = ksum (for the backward).
__global__ __launch_bounds__(kThreads) void att_kl_reduce_kernel(
    const float* __restrict__ ce, const float* __restrict__ kl, const int64_t* __restrict__ tgt,
    const uint8_t* __restrict__ pad, int P, int BU, int pad_id, float* __restrict__ l_att,
    float* __restrict__ l_kl, float* __restrict__ aux) {
  __shared__ float red[kThreads / 64];
  float ms = 0.0f, ks = 0.0f;
  for (int q = threadIdx.x; q < BU; q += kThreads) {
    ms += tgt[q] != pad_id ? 1.0f : 0.0f;
    ks += pad[q] ? 0.0f : 1.0f;
  }
  const float msum = block_sum(ms, red, false);
  const float ksum = block_sum(ks, red, false);
  for (int p = 0; p < P; ++p) {
    float a = 0.0f, k = 0.0f;
    for (int q = threadIdx.x; q < BU; q += kThreads) {
      a += ce[(size_t)p * BU + q];
      if (p > 0 && !pad[q]) k += kl[(size_t)p * BU + q];
    }
    const float sa = block_sum(a, red, false);
    const float sk = block_sum(k, red, false);
    if (threadIdx.x == 0) {
      const float mean = sa / (float)BU;
      l_att[p] = mean * msum / fmaxf(msum, 1.0f);
      if (p > 0) l_kl[p - 1] = sk / fmaxf(ksum, 1.0f);
    }
  }
  if (threadIdx.x == 0) {
    aux[0] = msum;
    aux[1] = ksum;
  }
}

__global__ __launch_bounds__(kThreads) void att_kl_bwd_kernel(
    const float* __restrict__ x, const int64_t* __restrict__ tgt, const uint8_t* __restrict__ pad,
    int BU, int V, float off, float c2, const float* __restrict__ stats,
    const float* __restrict__ aux, const float* __restrict__ g_att, const float* __restrict__ g_kl,
    float* __restrict__ grad) {
  const int r = blockIdx.x, q = r % BU, p = r / BU;
  const int nq = V / 4;
  const float msum = aux[0], ksum = aux[1];
  const float w_att = g_att[p] * (msum / fmaxf(msum, 1.0f)) / (float)BU;
  const float w_kl = (p > 0 && !pad[q]) ? g_kl[p - 1] / fmaxf(ksum, 1.0f) : 0.0f;
  const float m = stats[2 * r], logs = stats[2 * r + 1];
  const float mt = stats[2 * q], logst = stats[2 * q + 1];
  int64_t t = tgt[q];
  t = t < 0 ? 0 : (t >= V ? V - 1 : t);
  const float* row = x + (size_t)r * V;
  const float* trow = x + (size_t)q * V;
  float* g = grad + (size_t)r * V;
  const float ca = off * (float)V + c2;
  for (int qq = threadIdx.x; qq < nq; qq += kThreads) {
    const f32x4 v = reinterpret_cast<const f32x4*>(row)[qq];
    f32x4 y = {0.f, 0.f, 0.f, 0.f};
    if (w_kl != 0.0f) y = reinterpret_cast<const f32x4*>(trow)[qq];
    f32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float sm = expf((v[e] - m) - logs);
      float d = w_att * (ca * sm - off - (4 * qq + e == t ? c2 : 0.0f));
      if (w_kl != 0.0f) d += w_kl * (sm - expf((y[e] - mt) - logst));
      o[e] = d;
    }
    reinterpret_cast<f32x4*>(g)[qq] = o;
  }
}

}  // namespace

bool att_kl_supported(int64_t V) { return V >= 4 && V % 4 == 0 && V <= 4 * kMaxQ * kThreads; }

size_t att_kl_workspace(int64_t P, int64_t BU) {
  // stats [P*BU][2], ce [P*BU], kl [P*BU], aux [2]
  return sizeof(float) * (size_t)(4 * P * BU + 8);
}

void launch_att_kl_fwd(const float* x, const int64_t* tgt, const uint8_t* pad, int64_t P,
                       int64_t BU, int64_t V, int pad_id, float ls, float* l_att, float* l_kl,
                       void* ws, hipStream_t s) {
  float* stats = static_cast<float*>(ws);
  float* ce = stats + 2 * P * BU;
  float* kl = ce + P * BU;
  float* aux = kl + P * BU;
  const float off = ls / (float)(V - 1);
  const float c2 = 1.0f - ls - off;
  hipLaunchKernelGGL(att_kl_fwd_kernel, dim3((unsigned)(P * BU)), dim3(kThreads), 0, s, x, tgt,
                     (int)BU, (int)V, off, c2, stats, ce, kl);
  hipLaunchKernelGGL(att_kl_reduce_kernel, dim3(1), dim3(kThreads), 0, s, (const float*)ce,
                     (const float*)kl, tgt, pad, (int)P, (int)BU, pad_id, l_att, l_kl, aux);
}

void launch_att_kl_bwd(const float* x, const int64_t* tgt, const uint8_t* pad, int64_t P,
                       int64_t BU, int64_t V, float ls, const float* g_att, const float* g_kl,
                       float* grad, const void* ws, hipStream_t s) {
  const float* stats = static_cast<const float*>(ws);
  const float* aux = stats + 4 * P * BU;
  const float off = ls / (float)(V - 1);
  const float c2 = 1.0f - ls - off;
  hipLaunchKernelGGL(att_kl_bwd_kernel, dim3((unsigned)(P * BU)), dim3(kThreads), 0, s, x, tgt,
                     pad, (int)BU, (int)V, off, c2, stats, aux, g_att, g_kl, grad);
}

// ---------------------------------------------------------------------------------------
// The step's loss from its per-pass parts (train.py:95-111, the stacked form of
// train_step.OneBitStep): l_int = (1 - gamma) l_att + gamma l_ctc per pass, then
// loss = l_int[0] + lambda1 (l_int[1] + l_int[2]) + lambda2 (l_kl[0] + l_kl[1]) and the eight
// logged parts -- ONE single-thread launch, the rounding sequence of the torch expression it
// replaces (each mul and add rounded, in that order; no contraction), instead of ~20 scalar
// torch kernels forward and ~25 (index backwards: fills, copies, adds) backward.
namespace {
__device__ __forceinline__ float rmul(float a, float b) {
#pragma clang fp contract(off)
  return a * b;
}
__device__ __forceinline__ float radd(float a, float b) {
#pragma clang fp contract(off)
  return a + b;
}

__global__ void loss_combine_fwd_kernel(const float* __restrict__ l_att,
                                        const float* __restrict__ l_ctc,
                                        const float* __restrict__ l_kl, float g1, float g,
                                        float lam1, float lam2, float* __restrict__ loss,
                                        float* __restrict__ parts) {
  if (threadIdx.x != 0) return;
  float li[3];
#pragma unroll
  for (int p = 0; p < 3; ++p) li[p] = radd(rmul(g1, l_att[p]), rmul(g, l_ctc[p]));
  const float a = radd(li[0], rmul(lam1, radd(li[1], li[2])));
  loss[0] = radd(a, rmul(lam2, radd(l_kl[0], l_kl[1])));
  parts[0] = li[0];
  parts[1] = li[1];
  parts[2] = li[2];
  parts[3] = l_kl[0];
  parts[4] = l_kl[1];
  parts[5] = l_ctc[0];
  parts[6] = l_ctc[1];
  parts[7] = l_ctc[2];
}

// autograd of the same expression: dl_int = (gL, lam1 gL, lam1 gL), dl_att = (1 - gamma)
// dl_int, dl_ctc = gamma dl_int, dl_kl = (lam2 gL, lam2 gL)
__global__ void loss_combine_bwd_kernel(const float* __restrict__ gl, float g1, float g,
                                        float lam1, float lam2, float* __restrict__ d_att,
                                        float* __restrict__ d_ctc, float* __restrict__ d_kl) {
  if (threadIdx.x != 0) return;
  const float gv = gl[0];
  const float di[3] = {gv, rmul(lam1, gv), rmul(lam1, gv)};
#pragma unroll
  for (int p = 0; p < 3; ++p) {
    d_att[p] = rmul(g1, di[p]);
    d_ctc[p] = rmul(g, di[p]);
  }
  d_kl[0] = rmul(lam2, gv);
  d_kl[1] = rmul(lam2, gv);
}
}  // namespace

void launch_loss_combine_fwd(const float* l_att, const float* l_ctc, const float* l_kl,
                             float gamma, float lam1, float lam2, float* loss, float* parts,
                             hipStream_t s) {
  hipLaunchKernelGGL(loss_combine_fwd_kernel, dim3(1), dim3(64), 0, s, l_att, l_ctc, l_kl,
                     1.0f - gamma, gamma, lam1, lam2, loss, parts);
}

void launch_loss_combine_bwd(const float* gl, float gamma, float lam1, float lam2, float* d_att,
                             float* d_ctc, float* d_kl, hipStream_t s) {
  hipLaunchKernelGGL(loss_combine_bwd_kernel, dim3(1), dim3(64), 0, s, gl, 1.0f - gamma, gamma,
                     lam1, lam2, d_att, d_ctc, d_kl);
}

}  // namespace ob
