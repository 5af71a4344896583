// embed.hip — deterministic backward of the decoder's token embedding.
//
// Reference: onebit_asr/conformer.py:279-299, TransformerDecoder's
// nn.Embedding(vocab, d, padding_idx=pad) applied to the BOS-prefixed targets. torch's
// backward (sort + segmented partial sums) is replaced by a fixed-order segmented sum:
//   dW[v][c] = sum_{n ascending, idx[n] == v} g[n][c];   dW[pad] = 0 (padding_idx).
// Block = 32 vocabulary rows; the block streams the N indices once, compacts the hits on
// its rows, and accumulates the rows it owns in LDS in index order (one thread per (row slot, column) pair owns each
// accumulator, so there are no atomics).
#include "ob_launch.h"

namespace ob {

namespace {

constexpr int kThreads = 256;
constexpr int kRowsPerBlock = 32;
constexpr int kMaxC = 1024;
constexpr int kIdxChunk = 1024;  // static LDS 8 KiB: with kMaxC the block stays < 160 KiB

__global__ __launch_bounds__(kThreads) void embed_bwd_kernel(const int64_t* __restrict__ idx,
                                                             int64_t N, const float* __restrict__ g,
                                                             int C, int V, int64_t pad,
                                                             float* __restrict__ dW) {
  extern __shared__ float acc[];  // [kRowsPerBlock][C]
  const int v0 = blockIdx.x * kRowsPerBlock;
  for (int i = threadIdx.x; i < kRowsPerBlock * C; i += kThreads) acc[i] = 0.0f;
  __syncthreads();
  // Each thread owns columns c = threadIdx.x, +256, ... of every row slot; rows are
  // visited in index order, so each accumulator sums in ascending n. Per chunk of
  // kIdxChunk indices the block first compacts the positions that hit its rows into an
  // ordered LDS list (wave ballots + a 4-wave prefix), then walks only that list: a scan
  // of every index per block was latency-bound (280-350 us for 3936 decoder tokens).
  // Padding positions are dropped up front (dW[pad] = 0).
  __shared__ int hit_n[kIdxChunk];
  __shared__ int hit_slot[kIdxChunk];
  __shared__ int wave_cnt[kThreads / 64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int64_t base = 0; base < N; base += kIdxChunk) {
    const int cnt = (int)min((int64_t)kIdxChunk, N - base);
    int nhit = 0;  // block-uniform
    // the chunk's indices are all loaded before the first ballot (one memory latency per
    // chunk, not one per 256 indices)
    constexpr int kPass = kIdxChunk / kThreads;
    int64_t vv[kPass];
#pragma unroll
    for (int q = 0; q < kPass; ++q) {
      const int i = q * kThreads + threadIdx.x;
      vv[q] = i < cnt ? idx[base + i] : -1;
    }
#pragma unroll
    for (int q = 0; q < kPass; ++q) {
      const int off = q * kThreads;
      if (off >= cnt) break;  // block-uniform
      const int i = off + threadIdx.x;
      int slot = -1;
      if (i < cnt) {
        const int64_t v = vv[q];
        if (v >= v0 && v < v0 + kRowsPerBlock && v != pad) slot = (int)(v - v0);
      }
      const unsigned long long m = __ballot(slot >= 0);
      if (lane == 0) wave_cnt[wid] = __popcll(m);
      __syncthreads();
      int before = nhit;
      for (int w = 0; w < wid; ++w) before += wave_cnt[w];
      if (slot >= 0) {
        const int pos = before + __popcll(m & ((1ull << lane) - 1ull));
        hit_n[pos] = i;
        hit_slot[pos] = slot;
      }
      for (int w = 0; w < kThreads / 64; ++w) nhit += wave_cnt[w];
      __syncthreads();
    }
    // the hits' gradient rows, 8 loads in flight (a dependent load per hit was the kernel's
    // time); each accumulator still adds its rows in ascending n (the same sums)
    for (int c = threadIdx.x; c < C; c += kThreads) {
      int h = 0;
      for (; h + 8 <= nhit; h += 8) {
        float gv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) gv[u] = g[(base + hit_n[h + u]) * C + c];
#pragma unroll
        for (int u = 0; u < 8; ++u) acc[hit_slot[h + u] * C + c] += gv[u];
      }
      for (; h < nhit; ++h) acc[hit_slot[h] * C + c] += g[(base + hit_n[h]) * C + c];
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
  static_assert(sizeof(float) * kRowsPerBlock * kMaxC + 2 * sizeof(int) * kIdxChunk + 64 <=
                    160 * 1024,
                "embed_bwd_kernel LDS exceeds 160 KiB");
  hipLaunchKernelGGL(embed_bwd_kernel, dim3((unsigned)ceil_div(V, kRowsPerBlock)), dim3(kThreads),
                     lds, s, idx, N, g, (int)C, (int)V, pad, dW);
}

}  // namespace ob
