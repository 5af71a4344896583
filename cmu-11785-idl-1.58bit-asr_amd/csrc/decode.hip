// decode.hip — batched greedy CTC decode (inference path, BASELINE configs[4]).
//
// Reference: onebit_asr/metrics.py:51-60 ``ctc_greedy_decode(logits [T, V], blank_id=3)``:
//   pred = argmax(logits, -1); emit t when t != blank and t != prev; prev = t (also for blanks)
// run per utterance in a Python loop over `.tolist()`. Here one launch does the argmax for
// every (utterance, frame) of the padded batch and one launch collapses every utterance,
// over its first lens[b] frames (the caller's valid frames, as eval.py:122-124 computes them).
//
// argmax: one wave per frame, strided coalesced reads of the V logits, ties to the lowest
// index (torch.argmax returns the first maximal index). NaN logits are outside the
// reference's working range.
// collapse: one wave per utterance walks its frames 64 at a time; the keep bits of a chunk
// come from one ballot, and each kept token's slot is base + popcount(keep & lanes below).
#include "ob_launch.h"

namespace ob {

namespace {

constexpr int kWaves = 4;

__global__ __launch_bounds__(64 * kWaves) void argmax_rows_kernel(const float* __restrict__ logits,
                                                                  int64_t rows, int V,
                                                                  int* __restrict__ ids) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* x = logits + row * (int64_t)V;
  float best = -INFINITY;
  int bi = V;  // larger than any index: loses every tie
  for (int v = lane; v < V; v += 64) {
    const float e = x[v];
    if (e > best) {  // strictly greater: the first (lowest) index of a lane's max is kept
      best = e;
      bi = v;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ob = __shfl_xor(best, o);
    const int oi = __shfl_xor(bi, o);
    if (ob > best || (ob == best && oi < bi)) {
      best = ob;
      bi = oi;
    }
  }
  if (lane == 0) ids[row] = bi < V ? bi : 0;  // an all -inf row: index 0, like torch
}

__global__ __launch_bounds__(64) void ctc_collapse_kernel(const int* __restrict__ ids,
                                                          const int64_t* __restrict__ lens,
                                                          int T, int blank,
                                                          int* __restrict__ out,
                                                          int* __restrict__ out_len) {
  const int b = blockIdx.x;
  const int lane = threadIdx.x;
  int64_t L = lens[b];
  L = L < 0 ? 0 : (L > T ? T : L);
  const int* row = ids + (int64_t)b * T;
  int* dst = out + (int64_t)b * T;
  int base = 0;
  for (int t0 = 0; t0 < L; t0 += 64) {
    const int t = t0 + lane;
    const bool in = t < L;
    const int cur = in ? row[t] : blank;
    const int prev = (in && t > 0) ? row[t - 1] : -1;  // prev = None at t == 0
    const bool keep = in && cur != blank && cur != prev;
    const uint64_t m = __ballot(keep);
    if (keep) dst[base + __popcll(m & ((1ull << lane) - 1ull))] = cur;
    base += __popcll(m);
  }
  for (int t = base + lane; t < T; t += 64) dst[t] = -1;  // unused slots
  if (lane == 0) out_len[b] = base;
}

}  // namespace

void launch_ctc_greedy(const float* logits, const int64_t* lens, int64_t B, int64_t T, int64_t V,
                       int blank, int* ids, int* out, int* out_len, hipStream_t s) {
  if (B == 0) return;
  if (T > 0) {
    const int64_t rows = B * T;
    hipLaunchKernelGGL(argmax_rows_kernel, dim3((unsigned)ceil_div(rows, kWaves)),
                       dim3(64 * kWaves), 0, s, logits, rows, (int)V, ids);
  }
  hipLaunchKernelGGL(ctc_collapse_kernel, dim3((unsigned)B), dim3(64), 0, s, ids, lens, (int)T,
                     blank, out, out_len);
}

}  // namespace ob
