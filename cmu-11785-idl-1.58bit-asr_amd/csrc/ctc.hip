// ctc.hip — CTC loss with device-side lengths (stock op of the reference, made capturable).
//
// Reference: onebit_asr/losses.py:41-47 — log_softmax over the CTC head, then
// nn.CTCLoss(blank, zero_infinity=True) with 'mean' reduction. torch's CUDA CTC copies the
// length tensors to the host (a device->host sync), which makes a training step
// impossible to capture in a HIP graph. This is the same algorithm with the lengths read
// on device; its gradient w.r.t. log_probs is torch's (LossCTC):
//   grad[t,b,v] = (exp(lp[t,b,v]) - exp(logsumexp_{s: l'(s)=v}(alpha_t(s)+beta_t(s)) + nll_b
//                  - lp[t,b,v])) * grad_out_b        for t < T_b, 0 otherwise
// (composed with log_softmax this is the exact logits gradient; it is what torch returns).
// zero_infinity: an infeasible sample (nll = inf) gets loss 0 and gradient 0.
//
// Layout: log_probs [B][T][V] (batch-major; the reference's [T,B,V] transpose view is
// never materialised), targets [B][S] int64 (padded), lengths int64 [B].
// Kernels: alpha (one block per sample, states in parallel, t sequential), beta (same),
// dense grad (exp(lp) * scale over all (b, t, v)), label fix-up (one block per (b, t)).
// All sums are in a fixed order: deterministic.
#include <math.h>

#include "ob_launch.h"

namespace ob {

namespace {

constexpr int kThreads = 256;
constexpr int kMaxStates = 2 * 511 + 1;  // target length <= 511

__device__ __forceinline__ float lse2(float a, float b) {
  const float m = fmaxf(a, b);
  if (m == -INFINITY) return -INFINITY;
  return m + logf(expf(a - m) + expf(b - m));
}
__device__ __forceinline__ float lse3(float a, float b, float c) {
  const float m = fmaxf(a, fmaxf(b, c));
  if (m == -INFINITY) return -INFINITY;
  return m + logf(expf(a - m) + expf(b - m) + expf(c - m));
}

__device__ __forceinline__ int64_t ext_label(const int64_t* tg, int s, int blank) {
  return (s & 1) ? tg[s >> 1] : blank;
}

// alpha[b][t][s] for t < T_b (log space); nll[b] = -log p(l | x).
__global__ __launch_bounds__(kThreads) void ctc_alpha_kernel(
    const float* __restrict__ lp, const int64_t* __restrict__ targets,
    const int64_t* __restrict__ in_len, const int64_t* __restrict__ tg_len, int T, int V, int S,
    int blank, float* __restrict__ alpha, float* __restrict__ nll) {
  __shared__ float buf[2][kMaxStates + 2];
  const int b = blockIdx.x;
  const int Tb = (int)min<int64_t>(in_len[b], T);
  const int L = (int)tg_len[b];
  const int NS = 2 * L + 1;
  const int64_t* tg = targets + (int64_t)b * S;
  const float* lpb = lp + (int64_t)b * T * V;
  float* ab = alpha + (int64_t)b * T * (2 * S + 1);
  const int SS = 2 * S + 1;
  for (int t = 0; t < Tb; ++t) {
    const float* row = lpb + (int64_t)t * V;
    float* cur = buf[t & 1];
    const float* prev = buf[(t & 1) ^ 1];
    for (int s = threadIdx.x; s < NS; s += kThreads) {
      const int64_t lab = ext_label(tg, s, blank);
      const float l = row[lab];
      float a;
      if (t == 0) {
        a = (s <= 1) ? l : -INFINITY;
      } else {
        const float x0 = prev[s];
        const float x1 = s >= 1 ? prev[s - 1] : -INFINITY;
        const bool skip = s >= 2 && lab != blank && lab != ext_label(tg, s - 2, blank);
        const float x2 = skip ? prev[s - 2] : -INFINITY;
        a = lse3(x0, x1, x2) + l;
      }
      cur[s] = a;
      ab[(int64_t)t * SS + s] = a;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    float ll = -INFINITY;
    if (Tb > 0) {
      const float* last = buf[(Tb - 1) & 1];
      ll = NS >= 2 ? lse2(last[NS - 1], last[NS - 2]) : last[NS - 1];
    }
    nll[b] = -ll;
  }
}

// beta[b][t][s] for t < T_b (log space, includes lp[t] like alpha).
__global__ __launch_bounds__(kThreads) void ctc_beta_kernel(
    const float* __restrict__ lp, const int64_t* __restrict__ targets,
    const int64_t* __restrict__ in_len, const int64_t* __restrict__ tg_len, int T, int V, int S,
    int blank, float* __restrict__ beta) {
  __shared__ float buf[2][kMaxStates + 2];
  const int b = blockIdx.x;
  const int Tb = (int)min<int64_t>(in_len[b], T);
  const int L = (int)tg_len[b];
  const int NS = 2 * L + 1;
  const int64_t* tg = targets + (int64_t)b * S;
  const float* lpb = lp + (int64_t)b * T * V;
  const int SS = 2 * S + 1;
  float* bb = beta + (int64_t)b * T * SS;
  for (int t = Tb - 1; t >= 0; --t) {
    const float* row = lpb + (int64_t)t * V;
    float* cur = buf[t & 1];
    const float* nxt = buf[(t & 1) ^ 1];
    for (int s = threadIdx.x; s < NS; s += kThreads) {
      const int64_t lab = ext_label(tg, s, blank);
      const float l = row[lab];
      float v;
      if (t == Tb - 1) {
        v = (s >= NS - 2) ? l : -INFINITY;
      } else {
        const float x0 = nxt[s];
        const float x1 = s + 1 < NS ? nxt[s + 1] : -INFINITY;
        const bool skip = s + 2 < NS && lab != blank && lab != ext_label(tg, s + 2, blank);
        const float x2 = skip ? nxt[s + 2] : -INFINITY;
        v = lse3(x0, x1, x2) + l;
      }
      cur[s] = v;
      bb[(int64_t)t * SS + s] = v;
    }
    __syncthreads();
  }
}

// Per-sample loss and gradient scale: 'mean' = mean_b(nll_b / max(L_b, 1)); zero_infinity.
// G groups of B/G consecutive samples (the stacked passes of a training step, each the
// reference's own ctc_loss_from_logits call): loss[g], scale from grad_out[g]. Thread g
// sums its group in sample order (deterministic).
__global__ void ctc_reduce_kernel(const float* __restrict__ nll, const int64_t* __restrict__ tg_len,
                                  int B, int G, const float* __restrict__ grad_out,
                                  float* __restrict__ loss, float* __restrict__ scale) {
  const int g = threadIdx.x;
  if (blockIdx.x != 0 || g >= G) return;
  const int Bg = B / G;
  float s = 0.0f;
  for (int b = g * Bg; b < (g + 1) * Bg; ++b) {
    const float n = nll[b];
    const float L = (float)(tg_len[b] > 1 ? tg_len[b] : 1);
    const bool inf = isinf(n);
    s += inf ? 0.0f : n / L;
    if (scale) scale[b] = inf ? 0.0f : (grad_out ? grad_out[g] : 1.0f) / (L * (float)Bg);
  }
  if (loss) loss[g] = s / (float)Bg;
}

// grad[b][t][v] = exp(lp) * scale_b for t < T_b, else 0 (labels are fixed up afterwards).
__global__ __launch_bounds__(kThreads) void ctc_grad_dense_kernel(
    const float* __restrict__ lp, const int64_t* __restrict__ in_len,
    const float* __restrict__ scale, int T, int V, float* __restrict__ grad) {
  const int64_t rowid = blockIdx.x;  // b * T + t
  const int b = (int)(rowid / T), t = (int)(rowid % T);
  const bool live = t < in_len[b] && scale[b] != 0.0f;
  const float sc = scale[b];
  const float* src = lp + rowid * V;
  float* dst = grad + rowid * V;
  for (int v = threadIdx.x; v < V; v += kThreads) dst[v] = live ? expf(src[v]) * sc : 0.0f;
}

// For each distinct label v of sample b at time t: grad = (exp(lp) - exp(lcab + nll - lp)) *
// scale. State s "owns" label v if it is its first occurrence in l'; the owner sums
// alpha+beta over all occurrences in state order (deterministic).
__global__ __launch_bounds__(kThreads) void ctc_grad_fixup_kernel(
    const float* __restrict__ lp, const int64_t* __restrict__ targets,
    const int64_t* __restrict__ in_len, const int64_t* __restrict__ tg_len,
    const float* __restrict__ alpha, const float* __restrict__ beta, const float* __restrict__ nll,
    const float* __restrict__ scale, int T, int V, int S, int blank, float* __restrict__ grad) {
  const int64_t rowid = blockIdx.x;
  const int b = (int)(rowid / T), t = (int)(rowid % T);
  if (t >= in_len[b] || scale[b] == 0.0f) return;
  const int L = (int)tg_len[b];
  const int NS = 2 * L + 1;
  const int SS = 2 * S + 1;
  const int64_t* tg = targets + (int64_t)b * S;
  const float* a = alpha + ((int64_t)b * T + t) * SS;
  const float* be = beta + ((int64_t)b * T + t) * SS;
  const float n = nll[b];
  const float sc = scale[b];
  for (int s = threadIdx.x; s < NS; s += kThreads) {
    const int64_t lab = ext_label(tg, s, blank);
    bool first = true;
    for (int q = (s & 1); q < s; q += 2)  // same parity = same kind (blank / label)
      if (ext_label(tg, q, blank) == lab) { first = false; break; }
    if (!first) continue;
    float acc = -INFINITY;
    for (int q = s; q < NS; q += 2)
      if (ext_label(tg, q, blank) == lab) acc = lse2(acc, a[q] + be[q]);
    const float l = lp[rowid * V + lab];
    grad[rowid * V + lab] = (expf(l) - expf(acc + n - l)) * sc;
  }
}

}  // namespace

size_t ctc_workspace(int64_t B, int64_t T, int64_t S) {
  // alpha, beta [B][T][2S+1]; nll, scale [B]
  return sizeof(float) * (size_t)(2 * B * T * (2 * S + 1) + 2 * B + 64);
}

bool ctc_supported(int64_t S) { return 2 * S + 1 <= kMaxStates; }

void launch_ctc_fwd(const float* lp, const int64_t* targets, const int64_t* in_len,
                    const int64_t* tg_len, int64_t B, int64_t T, int64_t V, int64_t S, int blank,
                    int64_t G, float* loss, float* ws, hipStream_t s) {
  float* alpha = ws;
  float* nll = ws + 2 * B * T * (2 * S + 1);
  hipLaunchKernelGGL(ctc_alpha_kernel, dim3((unsigned)B), dim3(kThreads), 0, s, lp, targets,
                     in_len, tg_len, (int)T, (int)V, (int)S, blank, alpha, nll);
  hipLaunchKernelGGL(ctc_reduce_kernel, dim3(1), dim3(64), 0, s, nll, tg_len, (int)B, (int)G,
                     (const float*)nullptr, loss, (float*)nullptr);
}

void launch_ctc_bwd(const float* lp, const int64_t* targets, const int64_t* in_len,
                    const int64_t* tg_len, int64_t B, int64_t T, int64_t V, int64_t S, int blank,
                    int64_t G, const float* grad_out, float* grad, float* ws, hipStream_t s) {
  const int64_t SS = 2 * S + 1;
  float* alpha = ws;
  float* beta = ws + B * T * SS;
  float* nll = ws + 2 * B * T * SS;
  float* scale = nll + B;
  hipLaunchKernelGGL(ctc_beta_kernel, dim3((unsigned)B), dim3(kThreads), 0, s, lp, targets,
                     in_len, tg_len, (int)T, (int)V, (int)S, blank, beta);
  hipLaunchKernelGGL(ctc_reduce_kernel, dim3(1), dim3(64), 0, s, nll, tg_len, (int)B, (int)G,
                     grad_out, (float*)nullptr, scale);
  hipLaunchKernelGGL(ctc_grad_dense_kernel, dim3((unsigned)(B * T)), dim3(kThreads), 0, s, lp,
                     in_len, scale, (int)T, (int)V, grad);
  hipLaunchKernelGGL(ctc_grad_fixup_kernel, dim3((unsigned)(B * T)), dim3(kThreads), 0, s, lp,
                     targets, in_len, tg_len, alpha, beta, nll, scale, (int)T, (int)V, (int)S,
                     blank, grad);
}

}  // namespace ob
