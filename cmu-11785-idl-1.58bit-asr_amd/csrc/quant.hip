// quant.hip — weight quantizer kernels: pack (forward codes), dequant (quantize_weight
// forward) and the STE split-reduction finish (quantize_weight / BitLinear backward).
//
// Reference: onebit_asr/quant.py:44-92 (_QuantizeSTE.forward / .backward).
// All of these touch only the [N][K] weight-shaped tensors (<= 83k elements at
// Conformer-S), so they are launch-bound, not bandwidth-bound; they are written to be
// one launch each, deterministic and capture-safe.
#include "ob_launch.h"
#include "ob_quant.h"

namespace ob {

namespace {

constexpr int kThreads = 256;

// One thread per code: 16 consecutive lanes build one 32-bit word with a 4-step
// shuffle OR-reduction (lane j contributes code << 2j).
// Threads [0, 16*N*KW) build codes (row n, word w: K-contiguous, coalesced reads);
// threads [16*N*KW, 16*(N*KW + K*NW)) build codes_t with lanes (j = lane&15, kk = lane>>4)
// reading W[16w+j][k0+kk] (16 rows x 4 consecutive columns per wave).
__device__ __forceinline__ uint32_t or16(uint32_t v) {
  v |= __shfl_xor(v, 1, 64);
  v |= __shfl_xor(v, 2, 64);
  v |= __shfl_xor(v, 4, 64);
  v |= __shfl_xor(v, 8, 64);
  return v;
}

__global__ __launch_bounds__(kThreads) void quant_pack_kernel(
    const float* __restrict__ W, const float* __restrict__ alpha, int alpha_raw, int bits,
    const int* __restrict__ bits_dev, int64_t N, int64_t K, int64_t KW, int64_t NW,
    uint32_t* __restrict__ codes, uint32_t* __restrict__ codes_t) {
  if (bits_dev) bits = *bits_dev;  // graph mode: per-call bitwidth read on device
  const float a = effective_alpha(alpha, alpha_raw);
  const int64_t t = blockIdx.x * (int64_t)kThreads + threadIdx.x;
  const int j = threadIdx.x & 15;
  const int64_t n_words = codes ? N * KW : 0;
  const int64_t n_words_t = codes_t ? K * NW : 0;
  const int64_t wi = t >> 4;  // wave-uniform per 16-lane group
  if (wi < n_words) {
    const int64_t n = wi / KW, w = wi - n * KW;
    const int64_t k = 16 * w + j;
    const uint32_t c = (k < K) ? quant_code(W[n * K + k], a, bits) : 0u;
    const uint32_t word = or16(c << (2 * j));
    if (j == 0) codes[wi] = word;
    return;
  }
  // codes_t: 4 words per wave; word index = (w, k) with k fastest across the 4 groups.
  const int64_t wt = wi - n_words;
  if (wt < n_words_t) {
    const int64_t w = wt / K, k = wt - w * K;
    const int64_t n = 16 * w + j;
    const uint32_t c = (n < N) ? quant_code(W[n * K + k], a, bits) : 0u;
    const uint32_t word = or16(c << (2 * j));
    if (j == 0) codes_t[k * NW + w] = word;
  }
}

// Grouped pack: every (layer, bitwidth) item of a model in ONE launch. Item i owns blocks
// [block0_i, block0_{i+1}); a block finds its item by binary search over the (device)
// table, then does what quant_pack_kernel does for kPackIters x 256 of the item's threads
// (few blocks: the search's dependent loads are paid once per 4096 code slots). At
// Conformer-S this replaces 288 launch-bound 5 us packs per step with one launch.
constexpr int kPackIters = 16;  // 16-lane word groups per thread slot: blocks do 16x the work

__global__ __launch_bounds__(kThreads) void quant_pack_group_kernel(
    const ob_pack_item* __restrict__ items, int n_items) {
  int lo = 0, hi = n_items - 1;
  const int64_t blk = blockIdx.x;
  while (lo < hi) {  // last item with block0 <= blk
    const int mid = (lo + hi + 1) >> 1;
    if (items[mid].block0 <= blk) lo = mid; else hi = mid - 1;
  }
  const ob_pack_item it = items[lo];
  if (it.bits == 16) {  // bf16 weight images (quant-off): codes <- bf16(W), codes_t <- bf16(W^T)
    const int64_t nk = it.N * it.K;
    uint16_t* img = reinterpret_cast<uint16_t*>(it.codes);
    uint16_t* imgt = reinterpret_cast<uint16_t*>(it.codes_t);
#pragma unroll 4
    for (int i = 0; i < kPackIters; ++i) {
      const int64_t e = ((blk - it.block0) * kPackIters + i) * kThreads + threadIdx.x;
      if (e < nk) {
        img[e] = __builtin_bit_cast(uint16_t, (__bf16)it.W[e]);
      } else if (e < 2 * nk) {
        const int64_t e2 = e - nk, k = e2 / it.N, n = e2 - k * it.N;
        imgt[e2] = __builtin_bit_cast(uint16_t, (__bf16)it.W[n * it.K + k]);
      }
    }
    return;
  }
  const float a = effective_alpha(it.alpha, it.alpha_raw);
  const int64_t N = it.N, K = it.K, KW = (K + 15) >> 4, NW = (N + 15) >> 4;
  const int j = threadIdx.x & 15;
  const int64_t n_words = N * KW, n_words_t = K * NW;
#pragma unroll 4
  for (int i = 0; i < kPackIters; ++i) {
    const int64_t t = ((blk - it.block0) * kPackIters + i) * kThreads + threadIdx.x;
    const int64_t wi = t >> 4;
    if (wi < n_words) {
      const int64_t n = wi / KW, w = wi - n * KW;
      const int64_t k = 16 * w + j;
      const uint32_t c = (k < K) ? quant_code(it.W[n * K + k], a, it.bits) : 0u;
      const uint32_t word = or16(c << (2 * j));
      if (j == 0) it.codes[wi] = word;
      continue;
    }
    const int64_t wt = wi - n_words;
    if (wt < n_words_t) {
      const int64_t w = wt / K, k = wt - w * K;
      const int64_t n = 16 * w + j;
      const uint32_t c = (n < N) ? quant_code(it.W[n * K + k], a, it.bits) : 0u;
      const uint32_t word = or16(c << (2 * j));
      if (j == 0) it.codes_t[k * NW + w] = word;
    }
  }
}

// quant.py:68 W_hat = alpha * Q, elementwise, grid-stride.
__global__ __launch_bounds__(kThreads) void quant_dequant_kernel(const float* __restrict__ W,
                                                                 const float* __restrict__ alpha,
                                                                 int alpha_raw, int bits,
                                                                 int64_t n,
                                                                 float* __restrict__ W_hat) {
  const float a = effective_alpha(alpha, alpha_raw);
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  for (int64_t i = blockIdx.x * (int64_t)kThreads + threadIdx.x; i < n; i += stride) {
    W_hat[i] = a * code_value(quant_code(W[i], a, bits));
  }
}

// quant.py:80-91 applied to the fixed-order sum of `chunks` partial slabs.
// Block = 1024 elements (4 per thread, strided by 256 for coalescing); each thread sums its
// elements' chunks in chunk order with all loads independent. Few, wide blocks keep the
// number of ticket atomics on the one completion counter small (each costs ~12 ns
// serialised; 1300 blocks cost 16 us at Conformer-S). Deterministic.
constexpr int kReduceEPT = 2;  // 2: ~160 blocks for an 83k-element layer (4 left 2/3 of the CUs idle)
constexpr int kReduceElems = kThreads * kReduceEPT;

__global__ __launch_bounds__(kThreads) void ste_reduce_kernel(
    const float* __restrict__ part, int P, int cpp, int64_t nk, const float* __restrict__ part_db,
    int64_t n_db, const float* __restrict__ W, const float* __restrict__ alpha, int alpha_raw,
    int bits, const int* __restrict__ bits_dev, const int* __restrict__ pass_bits,
    float* __restrict__ dW, float* __restrict__ db, float* __restrict__ apart,
    uint32_t* __restrict__ ticket, float* __restrict__ dalpha) {
  // Per-pass bitwidth: pass_bits[p] (stacked passes), else one bitwidth (bits_dev: read on
  // device in graph mode). Passes of equal bitwidth share one alpha term (quant.py:86-90),
  // so the partial sums are kept per bitwidth: g1 (1-bit passes) and g2 (2-bit passes).
  if (bits_dev) bits = *bits_dev;
  int pb[kMaxPasses];
  bool has1 = false, has2 = false;
#pragma unroll
  for (int p = 0; p < kMaxPasses; ++p) {
    const int b = p < P ? (pass_bits ? pass_bits[p] : bits) : 2;
    pb[p] = b == 1 ? 1 : 2;
    if (p < P) {
      has1 |= pb[p] == 1;
      has2 |= pb[p] == 2;
    }
  }
  __shared__ float wsum[kThreads / 64];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const float a = effective_alpha(alpha, alpha_raw);
  float prod = 0.0f;
#pragma unroll
  for (int i = 0; i < kReduceEPT; ++i) {
    const int64_t e = blockIdx.x * (int64_t)kReduceElems + i * kThreads + threadIdx.x;
    const bool is_w = e < nk;
    const bool is_b = !is_w && e < nk + n_db;
    if (!is_w && !is_b) continue;
    const float* src = is_w ? part + e : part_db + (e - nk);
    const int64_t stride = is_w ? nk : n_db;
    float g1 = 0.0f, g2 = 0.0f;
#pragma unroll
    for (int p = 0; p < kMaxPasses; ++p) {
      if (p >= P) break;
      const float* sp = src + (int64_t)p * cpp * stride;
      float gp = 0.0f;
      int c = 0;
      for (; c + 8 <= cpp; c += 8) {  // 8 loads in flight, summed in chunk order
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = sp[(int64_t)(c + u) * stride];
#pragma unroll
        for (int u = 0; u < 8; ++u) gp += v[u];
      }
      for (; c + 4 <= cpp; c += 4) {
        const float v0 = sp[(int64_t)c * stride];
        const float v1 = sp[(int64_t)(c + 1) * stride];
        const float v2 = sp[(int64_t)(c + 2) * stride];
        const float v3 = sp[(int64_t)(c + 3) * stride];
        gp += v0;
        gp += v1;
        gp += v2;
        gp += v3;
      }
      for (; c < cpp; ++c) gp += sp[(int64_t)c * stride];
      if (pb[p] == 1) g1 += gp;
      else g2 += gp;
    }
    const float g = g2 + g1;
    if (is_w) {
      const float wa = W[e] / a;
      dW[e] = g * ste_indicator(wa);  // quant.py:81-82 (multiply: inf*0 -> NaN as in torch)
      float t = 0.0f;                 // quant.py:91 grad_out * term, per bitwidth
      if (has2) t += g2 * alpha_term(wa, 2);
      if (has1) t += g1 * alpha_term(wa, 1);
      prod += t;
    } else {
      db[e - nk] = g;
    }
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) prod += __shfl_xor(prod, off, 64);
  if (lane == 0) wsum[wave] = prod;
  __syncthreads();
  if (wave != 0) return;
  prod = ((wsum[0] + wsum[1]) + wsum[2]) + wsum[3];

  // Last-arriver finish of quant.py:91 .sum() (Guideline 16, write-through form, no
  // fences): the partial is stored sc1 (agent-scope relaxed atomic store = write-through),
  // drained, then a relaxed agent ticket is taken; the block that draws the last ticket
  // reads every partial with sc1 loads (L1 bypass) and sums them in index order, so the
  // result does not depend on which block finishes last. A release fence here instead
  // writes back the XCD L2 per block (measured 20 us for this kernel at Conformer-S).
  // `ticket` was zeroed by dw_partial (previous kernel on this stream) or a memset, and
  // is re-zeroed by the last block.
  // ISA assumption (pinned by the #error below): on CDNA (gfx9-family) an agent-scope
  // relaxed atomic store is a write-through (sc1) vector store counted by vmcnt, so the
  // s_waitcnt vmcnt(0) orders it before the ticket; gfx10+ count stores in vscnt and would
  // need a release / acquire pair here instead.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__) && !defined(__gfx942__) && \
    !defined(__gfx941__) && !defined(__gfx940__) && !defined(__gfx90a__)
#error "ste_reduce's last-block finish assumes CDNA (gfx9) store ordering; re-derive it for this target"
#endif
  int last = 0;
  if (lane == 0) {
    __hip_atomic_store(&apart[blockIdx.x], prod, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = (t == gridDim.x - 1) ? 1 : 0;
  }
  last = __shfl(last, 0, 64);
  if (!last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keep the loads below the ticket
  float s2 = 0.0f;
  for (uint32_t i = lane; i < gridDim.x; i += 64)
    s2 += __hip_atomic_load(&apart[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) s2 += __shfl_xor(s2, off, 64);
  if (lane == 0) {
    dalpha[0] = s2 * alpha_chain(alpha, alpha_raw);
    __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

}  // namespace

void launch_quant_pack(const float* W, const float* alpha, int alpha_raw, int bits,
                       const int* bits_dev, int64_t N, int64_t K, uint32_t* codes,
                       uint32_t* codes_t, hipStream_t s) {
  const int64_t KW = ceil_div(K, 16), NW = ceil_div(N, 16);
  const int64_t total = 16 * ((codes ? N * KW : 0) + (codes_t ? K * NW : 0));
  if (total == 0) return;
  const int64_t blocks = ceil_div(total, kThreads);
  hipLaunchKernelGGL(quant_pack_kernel, dim3((unsigned)blocks), dim3(kThreads), 0, s, W, alpha,
                     alpha_raw, bits, bits_dev, N, K, KW, NW, codes, codes_t);
}

int64_t quant_pack_item_blocks16(int64_t N, int64_t K) {
  return ceil_div(2 * N * K, (int64_t)kPackIters * kThreads);
}

int64_t quant_pack_item_blocks(int64_t N, int64_t K) {
  return ceil_div(16 * (N * ceil_div(K, 16) + K * ceil_div(N, 16)), (int64_t)kThreads * kPackIters);
}

void launch_quant_pack_group(const ob_pack_item* items_dev, int n_items, int64_t total_blocks,
                             hipStream_t s) {
  if (n_items <= 0 || total_blocks <= 0) return;
  hipLaunchKernelGGL(quant_pack_group_kernel, dim3((unsigned)total_blocks), dim3(kThreads), 0, s,
                     items_dev, n_items);
}

void launch_quant_dequant(const float* W, const float* alpha, int alpha_raw, int bits, int64_t n,
                          float* W_hat, hipStream_t s) {
  if (n == 0) return;
  int64_t blocks = ceil_div(n, kThreads);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(quant_dequant_kernel, dim3((unsigned)blocks), dim3(kThreads), 0, s, W,
                     alpha, alpha_raw, bits, n, W_hat);
}

int64_t ste_reduce_blocks(int64_t total) { return ceil_div(total, kReduceElems); }

void launch_ste_reduce(const float* part, int chunks, int64_t nk, const float* part_db,
                       int64_t n_db, const float* W, const float* alpha, int alpha_raw, int bits,
                       const int* bits_dev, float* dW, float* db, float* apart, uint32_t* ticket,
                       float* dalpha, hipStream_t s) {
  int64_t nb = ste_reduce_blocks(nk + n_db);
  if (nb == 0) nb = 1;  // an empty tensor still writes dalpha = 0
  hipLaunchKernelGGL(ste_reduce_kernel, dim3((unsigned)nb), dim3(kThreads), 0, s, part, 1, chunks,
                     nk, part_db, n_db, W, alpha, alpha_raw, bits, bits_dev, (const int*)nullptr,
                     dW, db, apart, ticket, dalpha);
}

void launch_ste_reduce_passes(const float* part, int P, int cpp, int64_t nk, const float* part_db,
                              int64_t n_db, const float* W, const float* alpha, int alpha_raw,
                              const int* pass_bits, float* dW, float* db, float* apart,
                              uint32_t* ticket, float* dalpha, hipStream_t s) {
  int64_t nb = ste_reduce_blocks(nk + n_db);
  if (nb == 0) nb = 1;
  hipLaunchKernelGGL(ste_reduce_kernel, dim3((unsigned)nb), dim3(kThreads), 0, s, part, P, cpp,
                     nk, part_db, n_db, W, alpha, alpha_raw, 2, (const int*)nullptr, pass_bits,
                     dW, db, apart, ticket, dalpha);
}

}  // namespace ob
