// embed.hip — deterministic backward of the decoder's token embedding.
//
// Reference: onebit_asr/conformer.py:279-299, TransformerDecoder's
// nn.Embedding(vocab, d, padding_idx=pad) applied to the BOS-prefixed targets. torch's
// backward (sort + segmented partial sums) is replaced by a fixed-order segmented sum:
//   dW[v][c] = sum_{n ascending, idx[n] == v} g[n][c];   dW[pad] = 0 (padding_idx).
// Block = 32 vocabulary rows; the block streams the N indices once and accumulates the
// rows it owns in LDS in index order (one thread per (row slot, column) pair owns each
// accumulator, so there are no atomics).
#include "ob_launch.h"

namespace ob {

namespace {

constexpr int kThreads = 256;
constexpr int kRowsPerBlock = 32;
constexpr int kMaxC = 1024;
constexpr int kIdxChunk = 4096;

__global__ __launch_bounds__(kThreads) void embed_bwd_kernel(const int64_t* __restrict__ idx,
                                                             int64_t N, const float* __restrict__ g,
                                                             int C, int V, int64_t pad,
                                                             float* __restrict__ dW) {
  extern __shared__ float acc[];  // [kRowsPerBlock][C]
  const int v0 = blockIdx.x * kRowsPerBlock;
  for (int i = threadIdx.x; i < kRowsPerBlock * C; i += kThreads) acc[i] = 0.0f;
  __syncthreads();
  // Each thread owns columns c = threadIdx.x, +256, ... of every row slot; rows are
  // visited in index order, so each accumulator sums in ascending n. The indices are
  // staged through LDS in chunks (a global load per index made the scan latency-bound:
  // 350 us for 3936 decoder tokens).
  __shared__ int sidx[kIdxChunk];
  for (int64_t base = 0; base < N; base += kIdxChunk) {
    const int cnt = (int)min((int64_t)kIdxChunk, N - base);
    for (int i = threadIdx.x; i < cnt; i += kThreads) {
      const int64_t v = idx[base + i];
      sidx[i] = (v >= v0 && v < v0 + kRowsPerBlock) ? (int)(v - v0) : -1;
    }
    __syncthreads();
    for (int i = 0; i < cnt; ++i) {
      const int slot = sidx[i];
      if (slot < 0) continue;  // uniform across the block
      const float* gr = g + (base + i) * C;
      float* ar = acc + slot * C;
      for (int c = threadIdx.x; c < C; c += kThreads) ar[c] += gr[c];
    }
    __syncthreads();
  }
  for (int i = threadIdx.x; i < kRowsPerBlock * C; i += kThreads) {
    const int v = v0 + i / C;
    if (v < V) dW[(int64_t)v * C + (i % C)] = (v == pad) ? 0.0f : acc[i];
  }
}

}  // namespace

bool embed_supported(int64_t C) { return C >= 1 && C <= kMaxC; }

void launch_embed_bwd(const int64_t* idx, int64_t N, const float* g, int64_t C, int64_t V,
                      int64_t pad, float* dW, hipStream_t s) {
  if (V == 0 || C == 0) return;
  const size_t lds = sizeof(float) * kRowsPerBlock * (size_t)C;
  hipLaunchKernelGGL(embed_bwd_kernel, dim3((unsigned)ceil_div(V, kRowsPerBlock)), dim3(kThreads),
                     lds, s, idx, N, g, (int)C, (int)V, pad, dW);
}

}  // namespace ob
