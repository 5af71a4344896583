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

// One state per thread (2 L + 1 <= kThreads): the thread's extended label and its skip
// rule are read once, before the recursion (not per step from global memory), and the
// log-probs of its next kRing steps are kept in flight in a register ring (the loop is
// unrolled by kRing, so every ring index is static; the loads are unconditional, clamped to
// the last frame): a step then waits only on its LDS neighbours and the barrier. The same
// operations in the same order as the strided loop: the same bits.
constexpr int kRing = 8;

// A barrier that orders LDS only: __syncthreads()'s workgroup release also covers global
// memory, which on gfx950 waits for every outstanding vector-memory operation -- the ring's
// loads included -- at each step. The alpha / beta rows written to global memory are read
// only by later launches.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

__device__ __forceinline__ void ctc_alpha_one(const float* __restrict__ lpb,
                                              const int64_t* __restrict__ tg, int Tb, int NS,
                                              int V, int SS, int blank, float (*buf)[kMaxStates + 2],
                                              float* __restrict__ ab, float* __restrict__ nll,
                                              int b) {
  const int s = threadIdx.x;
  const bool act = s < NS;
  const int64_t lab = act ? ext_label(tg, s, blank) : 0;
  const bool skip = act && s >= 2 && lab != blank && lab != ext_label(tg, s - 2, blank);
  const float* col = lpb + lab;  // this state's column (inactive threads: column 0)
  const int tl = Tb > 0 ? Tb - 1 : 0;
  float ring[kRing];
#pragma unroll
  for (int i = 0; i < kRing; ++i) ring[i] = col[(int64_t)(i < tl ? i : tl) * V];
  for (int t0 = 0; t0 < Tb; t0 += kRing) {
#pragma unroll
    for (int i = 0; i < kRing; ++i) {
      const int t = t0 + i;
      if (t >= Tb) break;  // block-uniform
      const float l = ring[i];
      float* cur = buf[t & 1];
      const float* prev = buf[(t & 1) ^ 1];
      if (act) {
        float a;
        if (t == 0) {
          a = (s <= 1) ? l : -INFINITY;
        } else {
          const float x0 = prev[s];
          const float x1 = s >= 1 ? prev[s - 1] : -INFINITY;
          const float x2 = skip ? prev[s - 2] : -INFINITY;
          a = lse3(x0, x1, x2) + l;
        }
        cur[s] = a;
        ab[(int64_t)t * SS + s] = a;
      }
      // the slot's next value (step t + kRing), issued after l's last use so the load can
      // land in the slot's own register (no copy, hence no wait for it before the barrier)
      ring[i] = col[(int64_t)(t + kRing < tl ? t + kRing : tl) * V];
      lds_barrier();
    }
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

__device__ __forceinline__ void ctc_beta_one(const float* __restrict__ lpb,
                                             const int64_t* __restrict__ tg, int Tb, int NS, int V,
                                             int SS, int blank, float (*buf)[kMaxStates + 2],
                                             float* __restrict__ bb) {
  const int s = threadIdx.x;
  const bool act = s < NS;
  const int64_t lab = act ? ext_label(tg, s, blank) : 0;
  const bool skip = act && s + 2 < NS && lab != blank && lab != ext_label(tg, s + 2, blank);
  const float* col = lpb + lab;
  const int tl = Tb > 0 ? Tb - 1 : 0;
  float ring[kRing];
#pragma unroll
  for (int i = 0; i < kRing; ++i) ring[i] = col[(int64_t)(tl - i > 0 ? tl - i : 0) * V];
  for (int t0 = Tb - 1; t0 >= 0; t0 -= kRing) {
#pragma unroll
    for (int i = 0; i < kRing; ++i) {
      const int t = t0 - i;
      if (t < 0) break;  // block-uniform
      const float l = ring[i];
      float* cur = buf[t & 1];
      const float* nxt = buf[(t & 1) ^ 1];
      if (act) {
        float v;
        if (t == Tb - 1) {
          v = (s >= NS - 2) ? l : -INFINITY;
        } else {
          const float x0 = nxt[s];
          const float x1 = s + 1 < NS ? nxt[s + 1] : -INFINITY;
          const float x2 = skip ? nxt[s + 2] : -INFINITY;
          v = lse3(x0, x1, x2) + l;
        }
        cur[s] = v;
        bb[(int64_t)t * SS + s] = v;
      }
      ring[i] = col[(int64_t)(t - kRing > 0 ? t - kRing : 0) * V];
      lds_barrier();
    }
  }
}

// alpha[b][t][s] for t < T_b (log space); nll[b] = -log p(l | x).
__device__ __forceinline__ void ctc_alpha_body(
    const float* __restrict__ lp, const int64_t* __restrict__ targets,
    const int64_t* __restrict__ in_len, const int64_t* __restrict__ tg_len, int T, int V, int S,
    int blank, float* __restrict__ alpha, float* __restrict__ nll, int b) {
  __shared__ float buf[2][kMaxStates + 2];
  const int Tb = (int)min<int64_t>(in_len[b], T);
  const int L = (int)tg_len[b];
  const int NS = 2 * L + 1;
  const int64_t* tg = targets + (int64_t)b * S;
  const float* lpb = lp + (int64_t)b * T * V;
  float* ab = alpha + (int64_t)b * T * (2 * S + 1);
  const int SS = 2 * S + 1;
  if (NS <= kThreads) {  // the common case: alpha_one_state (same operations, same bits)
    ctc_alpha_one(lpb, tg, Tb, NS, V, SS, blank, buf, ab, nll, b);
    return;
  }
  // NS > kThreads: states strided over the threads
  const bool one = false;
  const int s1 = threadIdx.x;
  const int64_t lab1 = s1 < NS ? ext_label(tg, s1, blank) : 0;
  float l_next = (one && s1 < NS && Tb > 0) ? lpb[lab1] : 0.0f;
  for (int t = 0; t < Tb; ++t) {
    const float* row = lpb + (int64_t)t * V;
    float* cur = buf[t & 1];
    const float* prev = buf[(t & 1) ^ 1];
    const float l_cur = l_next;
    if (one && s1 < NS && t + 1 < Tb) l_next = row[V + lab1];
    for (int s = threadIdx.x; s < NS; s += kThreads) {
      const int64_t lab = ext_label(tg, s, blank);
      const float l = one ? l_cur : row[lab];
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

__global__ __launch_bounds__(kThreads) void ctc_alpha_kernel(
    const float* __restrict__ lp, const int64_t* __restrict__ targets,
    const int64_t* __restrict__ in_len, const int64_t* __restrict__ tg_len, int T, int V, int S,
    int blank, float* __restrict__ alpha, float* __restrict__ nll) {
  ctc_alpha_body(lp, targets, in_len, tg_len, T, V, S, blank, alpha, nll, blockIdx.x);
}

// beta[b][t][s] for t < T_b (log space, includes lp[t] like alpha).
__device__ __forceinline__ void ctc_beta_body(
    const float* __restrict__ lp, const int64_t* __restrict__ targets,
    const int64_t* __restrict__ in_len, const int64_t* __restrict__ tg_len, int T, int V, int S,
    int blank, float* __restrict__ beta, int b) {
  __shared__ float buf[2][kMaxStates + 2];
  const int Tb = (int)min<int64_t>(in_len[b], T);
  const int L = (int)tg_len[b];
  const int NS = 2 * L + 1;
  const int64_t* tg = targets + (int64_t)b * S;
  const float* lpb = lp + (int64_t)b * T * V;
  const int SS = 2 * S + 1;
  float* bb = beta + (int64_t)b * T * SS;
  if (NS <= kThreads) {
    ctc_beta_one(lpb, tg, Tb, NS, V, SS, blank, buf, bb);
    return;
  }
  const bool one = false;
  const int s1 = threadIdx.x;
  const int64_t lab1 = s1 < NS ? ext_label(tg, s1, blank) : 0;
  float l_next = (one && s1 < NS && Tb > 0) ? lpb[(int64_t)(Tb - 1) * V + lab1] : 0.0f;
  for (int t = Tb - 1; t >= 0; --t) {
    const float* row = lpb + (int64_t)t * V;
    float* cur = buf[t & 1];
    const float* nxt = buf[(t & 1) ^ 1];
    const float l_cur = l_next;
    if (one && s1 < NS && t > 0) l_next = row[lab1 - V];
    for (int s = threadIdx.x; s < NS; s += kThreads) {
      const int64_t lab = ext_label(tg, s, blank);
      const float l = one ? l_cur : row[lab];
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

__global__ __launch_bounds__(kThreads) void ctc_beta_kernel(
    const float* __restrict__ lp, const int64_t* __restrict__ targets,
    const int64_t* __restrict__ in_len, const int64_t* __restrict__ tg_len, int T, int V, int S,
    int blank, float* __restrict__ beta) {
  ctc_beta_body(lp, targets, in_len, tg_len, T, V, S, blank, beta, blockIdx.x);
}

// Both recursions in one launch (blocks 0..B-1 alpha, B..2B-1 beta): each is a chain of T
// dependent steps on one block, so running them side by side halves the sequential time.
__global__ __launch_bounds__(kThreads) void ctc_alpha_beta_kernel(
    const float* __restrict__ lp, const int64_t* __restrict__ targets,
    const int64_t* __restrict__ in_len, const int64_t* __restrict__ tg_len, int B, int T, int V,
    int S, int blank, float* __restrict__ alpha, float* __restrict__ nll, float* __restrict__ beta) {
  if ((int)blockIdx.x < B)
    ctc_alpha_body(lp, targets, in_len, tg_len, T, V, S, blank, alpha, nll, blockIdx.x);
  else
    ctc_beta_body(lp, targets, in_len, tg_len, T, V, S, blank, beta, blockIdx.x - B);
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

// ------------------------------------------------------------------------------------
// CTC straight from the CTC head's logits (losses.py:41-47: log_softmax, then the CTC):
// the recursion only reads log-probabilities at blank and at the utterance's labels, so
// the [B*T][V] log_softmax tensor (478 MB at Conformer-S, V = 5004) is never formed.
//   lse pass (one block per frame): m = max_v x, logs = log(sum_v exp(x - m)) (torch's
//     LogSoftMax: lp = (x - m) - logs) and the compact log-probs
//     lpc[frame][0] = lp[blank], lpc[frame][1 + u] = lp[target_u]; the t == 0 block of
//     each utterance also writes its compact labels tgc[u] = 1 + (first u' with
//     target_u' == target_u) (0 for a target equal to blank), so equal tokens keep equal
//     labels for the recursion's skip rule.
//   alpha / beta / reduce: the recursions above on lpc (V' = S + 1, blank' = 0, labels
//     tgc), alpha and beta side by side in the forward's launch.
//   gradient (one block per frame): dL/dx_v = scale * (softmax_v - gamma_v), written
//     densely as scale * softmax_v, then the label columns overwritten with torch's own
//     formula (exp(l) - exp(lcab + nll - l)) * scale. torch composes its log-prob gradient
//     with the log_softmax backward g - softmax * sum(g); sum(g) = scale * (1 - sum gamma)
//     is 0 up to rounding, the only difference.
// ------------------------------------------------------------------------------------
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float block_reduce(float v, bool is_max, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float w = __shfl_xor(v, o);
    v = is_max ? fmaxf(v, w) : v + w;
  }
  __syncthreads();  // red reused across calls
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  float r = red[0];
#pragma unroll
  for (int w = 1; w < kThreads / 64; ++w) r = is_max ? fmaxf(r, red[w]) : r + red[w];
  return r;
}

__global__ __launch_bounds__(kThreads) void ctc_lse_gather_kernel(
    const float* __restrict__ x, const int64_t* __restrict__ targets,
    const int64_t* __restrict__ in_len, const int64_t* __restrict__ tg_len, int T, int V, int S,
    int blank, float* __restrict__ mls, float* __restrict__ lpc, int64_t* __restrict__ tgc,
    int* __restrict__ occ) {
  __shared__ float red[kThreads / 64];
  __shared__ int lab_s[kMaxStates];
  const int64_t rowid = blockIdx.x;  // b * T + t
  const int b = (int)(rowid / T), t = (int)(rowid % T);
  const int64_t* tg = targets + (int64_t)b * S;
  if (t == 0) {
    // compact labels of utterance b, and per extended-label state s (frame-independent):
    // occ[s] = the next state with the same compact label (-1: none), occ[SS + s] = 1 when s
    // is the first state of its label; the gradient's label fix-up walks these chains
    const int L = (int)tg_len[b];
    const int NS = 2 * L + 1;
    for (int u = threadIdx.x; u < S; u += kThreads) {
      int c = 0;
      if (u < L && tg[u] != blank) {
        int f = u;
        for (int q = 0; q < u; ++q)
          if (tg[q] == tg[u]) { f = q; break; }
        c = 1 + f;
      }
      tgc[(int64_t)b * S + u] = c;
      if (u < L) lab_s[2 * u + 1] = c;
    }
    for (int st = 2 * threadIdx.x; st < NS; st += 2 * kThreads) lab_s[st] = 0;
    __syncthreads();
    int* ob = occ + (int64_t)b * 2 * (2 * S + 1);
    for (int st = threadIdx.x; st < NS; st += kThreads) {
      const int lab = lab_s[st];
      bool first = true;
      for (int q = 0; q < st; ++q)
        if (lab_s[q] == lab) { first = false; break; }
      int nx = -1;
      for (int q = st + 1; q < NS; ++q)
        if (lab_s[q] == lab) { nx = q; break; }
      ob[st] = nx;
      ob[2 * S + 1 + st] = first ? 1 : 0;
    }
  }
  if (t >= in_len[b]) return;
  const float* row = x + rowid * V;
  const bool vec = (V & 3) == 0;
  // one pass over the row: the thread's values stay in registers (V <= 8 * 4 * kThreads
  // here: up to 8 float4 per thread) between the max and the sum
  constexpr int kMaxQ = 8;
  const int nq = vec ? V / 4 : 0;
  f32x4 vals[kMaxQ];
  float m = -INFINITY;
  const bool regs = vec && nq <= kMaxQ * kThreads;
  if (regs) {
#pragma unroll
    for (int i = 0; i < kMaxQ; ++i) {
      const int q = threadIdx.x + i * kThreads;
      vals[i] = q < nq ? reinterpret_cast<const f32x4*>(row)[q]
                       : f32x4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
      m = fmaxf(m, fmaxf(fmaxf(vals[i][0], vals[i][1]), fmaxf(vals[i][2], vals[i][3])));
    }
  } else {
    for (int v = threadIdx.x; v < V; v += kThreads) m = fmaxf(m, row[v]);
  }
  m = block_reduce(m, true, red);
  float sum = 0.0f;
  if (regs) {
#pragma unroll
    for (int i = 0; i < kMaxQ; ++i) {
      const int q = threadIdx.x + i * kThreads;
      if (q < nq)
        sum += ((expf(vals[i][0] - m) + expf(vals[i][1] - m)) + expf(vals[i][2] - m)) +
               expf(vals[i][3] - m);
    }
  } else {
    for (int v = threadIdx.x; v < V; v += kThreads) sum += expf(row[v] - m);
  }
  sum = block_reduce(sum, false, red);
  const float logs = logf(sum);
  if (threadIdx.x == 0) {
    mls[2 * rowid] = m;
    mls[2 * rowid + 1] = logs;
  }
  for (int c = threadIdx.x; c <= S; c += kThreads) {
    int64_t lab = c == 0 ? blank : tg[c - 1];
    lab = lab < 0 ? 0 : (lab >= V ? V - 1 : lab);  // padded target slots: any valid column
    lpc[rowid * (S + 1) + c] = (row[lab] - m) - logs;
  }
}

__global__ __launch_bounds__(kThreads) void ctc_logits_grad_kernel(
    const float* __restrict__ x, const float* __restrict__ mls, const float* __restrict__ lpc,
    const int64_t* __restrict__ targets, const int64_t* __restrict__ tgc,
    const int64_t* __restrict__ in_len, const int64_t* __restrict__ tg_len,
    const float* __restrict__ alpha, const float* __restrict__ beta, const float* __restrict__ nll,
    const float* __restrict__ scale, const int* __restrict__ occ, int T, int V, int S, int blank,
    float* __restrict__ grad) {
  const int64_t rowid = blockIdx.x;
  const int b = (int)(rowid / T), t = (int)(rowid % T);
  const bool live = t < in_len[b] && scale[b] != 0.0f;
  const float* row = x + rowid * V;
  float* g = grad + rowid * V;
  const bool vec = (V & 3) == 0;
  const float sc = live ? scale[b] : 0.0f;
  const float m = live ? mls[2 * rowid] : 0.0f, logs = live ? mls[2 * rowid + 1] : 0.0f;
  if (vec) {
    for (int q = threadIdx.x; q < V / 4; q += kThreads) {
      f32x4 o = {0.f, 0.f, 0.f, 0.f};
      if (live) {
        const f32x4 v = reinterpret_cast<const f32x4*>(row)[q];
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = expf((v[e] - m) - logs) * sc;
      }
      reinterpret_cast<f32x4*>(g)[q] = o;
    }
  } else {
    for (int v = threadIdx.x; v < V; v += kThreads)
      g[v] = live ? expf((row[v] - m) - logs) * sc : 0.0f;
  }
  if (!live) return;
  // alpha + beta of every state and the label chains into LDS (one parallel load each), so
  // an owner's walk over its label's occurrences -- L + 1 of them for blank -- reads LDS
  // instead of a dependent global load per step
  __shared__ float xs[kMaxStates];
  __shared__ int nx[kMaxStates];
  __shared__ int own[kMaxStates];
  const int L = (int)tg_len[b];
  const int NS = 2 * L + 1;
  const int SS = 2 * S + 1;
  const int64_t* tgb = tgc + (int64_t)b * S;
  const int* ob = occ + (int64_t)b * 2 * SS;
  const float* a = alpha + rowid * SS;
  const float* be = beta + rowid * SS;
  for (int s = threadIdx.x; s < NS; s += kThreads) {
    xs[s] = a[s] + be[s];
    nx[s] = ob[s];
    own[s] = ob[SS + s];
  }
  __syncthreads();  // (also: the label columns below overwrite this block's dense values)
  const float n = nll[b];
  for (int s = threadIdx.x; s < NS; s += kThreads) {
    if (!own[s]) continue;  // not the first state of its label
    const int64_t lab = ext_label(tgb, s, 0);  // compact label
    // occurrences of the label in state order (lse2(-inf, x) == x: the chain's first step)
    float acc = xs[s];
    for (int q = nx[s]; q >= 0; q = nx[q]) acc = lse2(acc, xs[q]);
    const float l = lpc[rowid * (S + 1) + lab];
    const int64_t v = (s & 1) ? targets[(int64_t)b * S + (s >> 1)] : blank;  // vocabulary id
    g[v] = (expf(l) - expf(acc + n - l)) * sc;
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

// logits path workspace: the CTC workspace, then lpc [B*T][S+1], mls [B*T][2], tgc [B][S]
namespace {
struct LogitsWs {
  float* ctc;
  float* lpc;
  float* mls;
  int64_t* tgc;
  int* occ;
};
LogitsWs split_logits_ws(void* ws, int64_t B, int64_t T, int64_t S) {
  LogitsWs w;
  char* p = static_cast<char*>(ws);
  w.ctc = reinterpret_cast<float*>(p);
  p += (ctc_workspace(B, T, S) + 255) & ~size_t(255);
  w.lpc = reinterpret_cast<float*>(p);
  p += (sizeof(float) * (size_t)(B * T * (S + 1)) + 255) & ~size_t(255);
  w.mls = reinterpret_cast<float*>(p);
  p += (sizeof(float) * (size_t)(2 * B * T) + 255) & ~size_t(255);
  w.tgc = reinterpret_cast<int64_t*>(p);
  p += (sizeof(int64_t) * (size_t)(B * S + 8) + 255) & ~size_t(255);
  w.occ = reinterpret_cast<int*>(p);
  return w;
}
}  // namespace

size_t ctc_logits_workspace_bytes(int64_t B, int64_t T, int64_t S) {
  return ((ctc_workspace(B, T, S) + 255) & ~size_t(255)) +
         ((sizeof(float) * (size_t)(B * T * (S + 1)) + 255) & ~size_t(255)) +
         ((sizeof(float) * (size_t)(2 * B * T) + 255) & ~size_t(255)) +
         ((sizeof(int64_t) * (size_t)(B * S + 8) + 255) & ~size_t(255)) +
         sizeof(int) * (size_t)(2 * B * (2 * S + 1) + 8);
}

void launch_ctc_logits_fwd(const float* x, const int64_t* targets, const int64_t* in_len,
                           const int64_t* tg_len, int64_t B, int64_t T, int64_t V, int64_t S,
                           int blank, int64_t G, float* loss, void* ws, hipStream_t s) {
  const LogitsWs w = split_logits_ws(ws, B, T, S);
  if (B * T > 0)
    hipLaunchKernelGGL(ctc_lse_gather_kernel, dim3((unsigned)(B * T)), dim3(kThreads), 0, s, x,
                       targets, in_len, tg_len, (int)T, (int)V, (int)S, blank, w.mls, w.lpc, w.tgc,
                       w.occ);
  // alpha and beta side by side (beta kept in the workspace for the backward)
  const int64_t SS = 2 * S + 1;
  float* alpha = w.ctc;
  float* beta = w.ctc + B * T * SS;
  float* nll = w.ctc + 2 * B * T * SS;
  hipLaunchKernelGGL(ctc_alpha_beta_kernel, dim3((unsigned)(2 * B)), dim3(kThreads), 0, s,
                     (const float*)w.lpc, (const int64_t*)w.tgc, in_len, tg_len, (int)B, (int)T,
                     (int)(S + 1), (int)S, 0, alpha, nll, beta);
  hipLaunchKernelGGL(ctc_reduce_kernel, dim3(1), dim3(64), 0, s, (const float*)nll, tg_len, (int)B,
                     (int)G, (const float*)nullptr, loss, (float*)nullptr);
}

void launch_ctc_logits_bwd(const float* x, const int64_t* targets, const int64_t* in_len,
                           const int64_t* tg_len, int64_t B, int64_t T, int64_t V, int64_t S,
                           int blank, int64_t G, const float* grad_out, float* grad, void* ws,
                           hipStream_t s) {
  const LogitsWs w = split_logits_ws(ws, B, T, S);
  const int64_t SS = 2 * S + 1;
  float* alpha = w.ctc;
  float* beta = w.ctc + B * T * SS;
  float* nll = w.ctc + 2 * B * T * SS;
  float* scale = nll + B;
  hipLaunchKernelGGL(ctc_reduce_kernel, dim3(1), dim3(64), 0, s, (const float*)nll, tg_len, (int)B,
                     (int)G, grad_out, (float*)nullptr, scale);
  if (B * T > 0)
    hipLaunchKernelGGL(ctc_logits_grad_kernel, dim3((unsigned)(B * T)), dim3(kThreads), 0, s, x,
                       (const float*)w.mls, (const float*)w.lpc, targets, (const int64_t*)w.tgc,
                       in_len, tg_len, (const float*)alpha, (const float*)beta, (const float*)nll,
                       (const float*)scale, (const int*)w.occ, (int)T, (int)V, (int)S, blank,
                       grad);
}

}  // namespace ob
