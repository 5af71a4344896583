// dwconv.hip — depthwise Conv1d of the Conformer conv module.
//
// Reference: onebit_asr/conformer.py:147 nn.Conv1d(C, C, k, padding=k//2, groups=C), run
// in full precision on [B, C, T] (after GLU, :156-157). MIOpen's fp32 grouped-conv path is
// the largest single kernel of the eager step; this is a per-row streaming
// kernel instead:
//   y[b,c,t]  = bias[c] + sum_j w[c,j] * x[b,c,t+j-P]              (zero padding, P = k/2)
//   dx[b,c,t] = sum_j w[c,j] * dy[b,c,t-j+P]
//   dw[c,j]   = sum_b sum_t dy[b,c,t] * x[b,c,t+j-P],   db[c] = sum_b sum_t dy[b,c,t]
// One block per (b, c) row: the row (+ halo) is staged in LDS, one output per thread.
// The weight/bias gradient is a per-row partial written by the backward kernel and summed
// over b in a fixed order by a second launch (deterministic, no atomics).
#include "ob_launch.h"

namespace ob {

namespace {

constexpr int kThreads = 256;
constexpr int kTile = 256;     // outputs per LDS tile
constexpr int kMaxTaps = 64;   // kernel width limit (the Conformer uses 31)
constexpr int kGroups = 8;     // t-phase groups for the weight-gradient partials

__global__ __launch_bounds__(kThreads) void dwconv_fwd_kernel(const float* __restrict__ x,
                                                              const float* __restrict__ w,
                                                              const float* __restrict__ bias,
                                                              int C, int T, int KT,
                                                              float* __restrict__ y) {
  __shared__ float xs[kTile + kMaxTaps];
  const int64_t row = blockIdx.x;
  const int c = (int)(row % C);
  const int P = KT / 2;
  const float* xr = x + row * T;
  float* yr = y + row * T;
  const float* wc = w + (int64_t)c * KT;
  const float b = bias ? bias[c] : 0.0f;
  for (int t0 = 0; t0 < T; t0 += kTile) {
    for (int i = threadIdx.x; i < kTile + KT - 1; i += kThreads) {
      const int t = t0 + i - P;
      xs[i] = (t >= 0 && t < T) ? xr[t] : 0.0f;
    }
    __syncthreads();
    const int t = t0 + threadIdx.x;
    if (t < T) {
      float acc = 0.0f;
      for (int j = 0; j < KT; ++j) acc = fmaf(wc[j], xs[threadIdx.x + j], acc);
      yr[t] = acc + b;
    }
    __syncthreads();
  }
}

// dx for the row, plus this row's weight/bias-gradient partial:
//   part[row][j] = sum_t dy[t] * x[t+j-P] (j < KT), part[row][KT] = sum_t dy[t].
__global__ __launch_bounds__(kThreads) void dwconv_bwd_kernel(
    const float* __restrict__ x, const float* __restrict__ dy, const float* __restrict__ w,
    int C, int T, int KT, float* __restrict__ dx, float* __restrict__ part) {
  __shared__ float xs[kTile + kMaxTaps];
  __shared__ float gs[kTile + kMaxTaps];
  __shared__ float red[kGroups][kMaxTaps + 1];
  const int64_t row = blockIdx.x;
  const int c = (int)(row % C);
  const int P = KT / 2;
  const float* xr = x + row * T;
  const float* gr = dy + row * T;
  float* dxr = dx ? dx + row * T : nullptr;
  const float* wc = w + (int64_t)c * KT;
  // weight-gradient work split: thread (j, q) sums t = q, q+kGroups, ... of the tile
  float accw[2] = {0.0f, 0.0f};  // taps j = tid%32 and j+32 for group q = tid/32
  const int tj = threadIdx.x & 31;
  const int tq = threadIdx.x >> 5;  // 0..7
  float accb = 0.0f;
  for (int t0 = 0; t0 < T; t0 += kTile) {
    // xs[i] = x[t0 + i - P] (for dw), gs[i] = dy[t0 + i - (KT-1-P)] (for dx: flipped taps)
    for (int i = threadIdx.x; i < kTile + KT - 1; i += kThreads) {
      const int tx = t0 + i - P;
      xs[i] = (tx >= 0 && tx < T) ? xr[tx] : 0.0f;
      const int tg = t0 + i - (KT - 1 - P);
      gs[i] = (tg >= 0 && tg < T) ? gr[tg] : 0.0f;
    }
    __syncthreads();
    const int t = t0 + threadIdx.x;
    if (dxr && t < T) {
      // dx[t] = sum_j w[j] * dy[t - j + P]; dy[t - j + P] = gs[t - t0 + KT - 1 - j]
      float acc = 0.0f;
      for (int j = 0; j < KT; ++j) acc = fmaf(wc[j], gs[threadIdx.x + KT - 1 - j], acc);
      dxr[t] = acc;
    }
    // weight gradient: dy[t] = gs[t - t0 + KT-1-P]; x[t+j-P] = xs[t - t0 + j]
    const int tn = T - t0 < kTile ? T - t0 : kTile;
    for (int tt = tq; tt < tn; tt += kGroups) {
      const float g = gs[tt + KT - 1 - P];
      if (tj < KT) accw[0] = fmaf(g, xs[tt + tj], accw[0]);
      if (tj + 32 < KT) accw[1] = fmaf(g, xs[tt + tj + 32], accw[1]);
      if (tj == 0) accb += g;
    }
    __syncthreads();
  }
  if (tj < KT) red[tq][tj] = accw[0];
  if (tj + 32 < KT) red[tq][tj + 32] = accw[1];
  if (tj == 0) red[tq][kMaxTaps] = accb;
  __syncthreads();
  // fixed-order sum over the 8 phase groups
  for (int j = threadIdx.x; j <= KT; j += kThreads) {
    const int src = j < KT ? j : kMaxTaps;
    float s = 0.0f;
#pragma unroll
    for (int q = 0; q < kGroups; ++q) s += red[q][src];
    part[row * (KT + 1) + j] = s;
  }
}

// dw[c][j] = sum_b part[b*C + c][j] (b ascending); db[c] = sum_b part[b*C + c][KT].
__global__ __launch_bounds__(kThreads) void dwconv_wgrad_kernel(const float* __restrict__ part,
                                                                int B, int C, int KT,
                                                                float* __restrict__ dw,
                                                                float* __restrict__ db) {
  const int i = blockIdx.x * kThreads + threadIdx.x;
  if (i >= C * (KT + 1)) return;
  const int c = i / (KT + 1), j = i - c * (KT + 1);
  float s = 0.0f;
  for (int b = 0; b < B; ++b) s += part[((int64_t)b * C + c) * (KT + 1) + j];
  if (j < KT)
    dw[c * KT + j] = s;
  else if (db)
    db[c] = s;
}

}  // namespace

bool dwconv_supported(int KT) { return KT >= 1 && KT <= kMaxTaps; }

void launch_dwconv_fwd(const float* x, const float* w, const float* bias, int64_t B, int64_t C,
                       int64_t T, int64_t KT, float* y, hipStream_t s) {
  if (B * C == 0 || T == 0) return;
  hipLaunchKernelGGL(dwconv_fwd_kernel, dim3((unsigned)(B * C)), dim3(kThreads), 0, s, x, w, bias,
                     (int)C, (int)T, (int)KT, y);
}

size_t dwconv_bwd_workspace(int64_t B, int64_t C, int64_t KT) {
  return sizeof(float) * (size_t)(B * C * (KT + 1));
}

void launch_dwconv_bwd(const float* x, const float* dy, const float* w, int64_t B, int64_t C,
                       int64_t T, int64_t KT, float* dx, float* dw, float* db, float* part,
                       hipStream_t s) {
  if (B * C > 0) {
    if (T > 0) {
      hipLaunchKernelGGL(dwconv_bwd_kernel, dim3((unsigned)(B * C)), dim3(kThreads), 0, s, x, dy,
                         w, (int)C, (int)T, (int)KT, dx, part);
    } else {
      launch_zero_words(part, (int64_t)(dwconv_bwd_workspace(B, C, KT) / sizeof(float)), s);
    }
  }
  const int64_t n = C * (KT + 1);
  if (n > 0 && B > 0)
    hipLaunchKernelGGL(dwconv_wgrad_kernel, dim3((unsigned)ceil_div(n, kThreads)), dim3(kThreads),
                       0, s, part, (int)B, (int)C, (int)KT, dw, db);
}

}  // namespace ob
