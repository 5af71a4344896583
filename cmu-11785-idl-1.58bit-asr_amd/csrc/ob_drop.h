// ob_drop.h — the counter-based dropout keep-hash shared by every fused-dropout kernel
// (attention probabilities, BitLinear epilogues, the dropout-backward scale kernel).
//
// keep(i) = drop_hash(drop_key(seed, ctr), i) >= thresh: a 32-bit murmur3-fmix hash of the
// element index mixed with a per-call key. The key folds (seed, counter) -- a device
// int64[2] the host advances once per call -- so a captured HIP graph draws a fresh mask
// on every replay, and a backward kernel regenerates its forward's mask from the same
// (seed, counter) without storing it. ~8 VALU ops (2 multiplies) per element.
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

struct DropCfg {
  uint32_t thresh;  // keep iff hash >= thresh
  float scale;      // 1 / (1 - p)
  int on;
};

inline DropCfg make_drop(float p_drop) {
  DropCfg dc;
  dc.on = p_drop > 0.0f ? 1 : 0;
  double t = (double)p_drop * 4294967296.0;
  if (t > 4294967295.0) t = 4294967295.0;
  dc.thresh = (uint32_t)t;
  dc.scale = p_drop > 0.0f ? (float)(1.0 / (1.0 - (double)p_drop)) : 1.0f;
  return dc;
}

}  // namespace ob
