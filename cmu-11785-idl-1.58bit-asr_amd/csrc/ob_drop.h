// ob_drop.h — the counter-based dropout keep-hash shared by every fused-dropout kernel
// (attention probabilities, BitLinear epilogues, the dropout-backward scale kernel).
//
// keep(i) = the 16-bit field (i & 1) of drop_hash(drop_key(seed, ctr), i >> 1) >= thresh:
// one 32-bit murmur3-fmix hash of the element-PAIR index, mixed with a per-call key, draws
// two elements (its low and high halves). The key folds (seed, counter) -- a device
// int64[2] the host advances once per call -- so a captured HIP graph draws a fresh mask
// on every replay, and a backward kernel regenerates its forward's mask from the same
// (seed, counter) without storing it. ~8 VALU ops (2 multiplies) per PAIR of elements.
// Mask quality: fmix32 is a bijection whose every output bit depends on every input bit
// (full avalanche), so the two 16-bit halves of one hash are as independent as two hashes
// of nearby indices; the drop probability is thresh / 2^16 with thresh = round(p * 2^16),
// |p_eff - p| <= 2^-17 (p = 0.1: 6554 / 65536 = 0.100006), and the keep scale stays the
// reference's 1 / (1 - p).
// The mask is not torch's Philox stream; no reference-visible quantity depends on it
// (dropout is stochastic in the reference too, train.py:200; parity runs use p = 0).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ob {

__device__ __forceinline__ uint32_t fmix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x85EBCA6Bu;
  x ^= x >> 13;
  x *= 0xC2B2AE35u;
  x ^= x >> 16;
  return x;
}

__device__ __forceinline__ uint32_t drop_key(uint64_t seed, uint64_t ctr) {
  return fmix32((uint32_t)seed ^ fmix32((uint32_t)(seed >> 32) ^ 0x9E3779B9u) ^
                fmix32((uint32_t)ctr * 0x27D4EB2Fu + (uint32_t)(ctr >> 32)));
}

// Two 32-bit multiplies per element (the fmix32 avalanche; v_mul_lo_u32 is a
// quarter-rate instruction, and this hash runs once per element of every fused dropout):
// the index's high word is folded in by a rotate, not a multiply.
__device__ __forceinline__ uint32_t drop_hash(uint32_t key, uint64_t idx) {
  const uint32_t hi = (uint32_t)(idx >> 32);
  return fmix32((uint32_t)idx ^ ((hi << 16) | (hi >> 16)) ^ key);
}

// A run of consecutive element pairs from pair index p (64-bit): the hash of pair p + off
// (off < 2^32) from 32-bit arithmetic -- the low word plus a carry into the high word --
// bit-equal to drop_hash(key, p + off), without the 64-bit index math per pair.
struct DropPairRow {
  uint32_t lo, k0, k1;  // low word of p; key ^ rot16(high word), the same with the carry
};

__device__ __forceinline__ uint32_t drop_rot16(uint32_t x) { return (x << 16) | (x >> 16); }

__device__ __forceinline__ DropPairRow drop_pair_row(uint32_t key, uint64_t p) {
  const uint32_t hi = (uint32_t)(p >> 32);
  return DropPairRow{(uint32_t)p, key ^ drop_rot16(hi), key ^ drop_rot16(hi + 1u)};
}

__device__ __forceinline__ uint32_t drop_hash_at(const DropPairRow& r, uint32_t off) {
  const uint32_t lo = r.lo + off;
  return fmix32(lo ^ (lo < r.lo ? r.k1 : r.k0));
}

struct DropCfg {
  uint32_t thresh;  // keep iff the element's 16-bit field >= thresh
  float scale;      // 1 / (1 - p)
  int on;
};

inline DropCfg make_drop(float p_drop) {
  DropCfg dc;
  dc.on = p_drop > 0.0f ? 1 : 0;
  double t = (double)p_drop * 65536.0 + 0.5;
  if (t > 65536.0) t = 65536.0;  // p = 1: every field (< 2^16) drops
  dc.thresh = (uint32_t)t;
  dc.scale = p_drop > 0.0f && p_drop < 1.0f ? (float)(1.0 / (1.0 - (double)p_drop)) : 1.0f;
  return dc;
}

// keep bit of element i (one hash per element pair; pairs (2j, 2j+1))
__device__ __forceinline__ bool drop_keep(uint32_t key, uint64_t i, uint32_t thresh) {
  const uint32_t h = drop_hash(key, i >> 1);
  return ((i & 1) ? (h >> 16) : (h & 0xFFFFu)) >= thresh;
}

// keep scales of elements i .. i+3 (i % 4 == 0): two hashes
__device__ __forceinline__ void drop_scale4(uint32_t key, uint64_t i, const DropCfg& dc,
                                            float (&out)[4]) {
  const uint32_t h0 = drop_hash(key, i >> 1), h1 = drop_hash(key, (i >> 1) + 1);
  out[0] = (h0 & 0xFFFFu) >= dc.thresh ? dc.scale : 0.0f;
  out[1] = (h0 >> 16) >= dc.thresh ? dc.scale : 0.0f;
  out[2] = (h1 & 0xFFFFu) >= dc.thresh ? dc.scale : 0.0f;
  out[3] = (h1 >> 16) >= dc.thresh ? dc.scale : 0.0f;
}

}  // namespace ob
