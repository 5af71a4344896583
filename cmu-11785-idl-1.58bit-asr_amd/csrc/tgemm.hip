// tgemm.hip — the ternary BitLinear GEMM on gfx950 matrix cores.
//
//   forward  Y  = a * X . Q^T + b     (quant.py:126, F.linear with W_hat = a*Q)
//   backward dX = a * dY . Q          (autograd of quant.py:126; same kernel, codes_t)
//
// fp32 parity with the reference's fp32 F.linear: each fp32 activation is split exactly
// into three bf16 parts x = hi + mid + lo (8+8+8 significand bits); Q in {-1,0,+1} is
// exact in bf16, so three v_mfma_f32_16x16x32_bf16 per k-step accumulate exact products
// in fp32 -- an fp32 GEMM up to summation order, at 3/16 of the fp32-MFMA cost. The scale
// `a` is applied once in the epilogue (Y = a*(X.Q^T)).
//
// Block = 4 waves, 64 rows x BN = 16*NT columns. At entry the block decodes its BN code
// rows into a bf16 image of Q in LDS ([BN][Kpad+16]: a row pitch of Kpad/2 + 8 dwords puts
// the 16 lanes of every ds_read_b128 lane group of the B fragments on disjoint banks at
// K = 144 and 576 -- the round-3 pad of 8 left 2-way conflicts at K = 576), then loops over
// its row tiles: each wave
// streams 16 rows of A (two dwordx4 per lane per 32-wide k-chunk, all chunks of a row in
// flight at once when K is a compile-time size), splits them in registers and issues 3
// MFMAs per 16-column tile. Blocks sharing a row tile are dealt to the same XCD so their
// A reads hit one L2.
//
// Fragment map of v_mfma_f32_16x16x32_bf16 (lane l, r = l&15, g = l>>4):
//   A[i=r][kk=8g+j] (j<8), B[kk=8g+j][col=r], D[row=4g+reg][col=r].
//
// Quant-off ceiling (BASELINE configs[3], quant.py:121-122 with bf16 weights): alpha_raw 2
// makes the "codes" argument a bf16 weight image [N][K] (uint16; for dX the transposed
// image, both packed once per step like the codes: ob_quant_pack_group items with bits 16);
// the block copies its rows into the LDS image instead of decoding codes, and the scale is
// 1 -- the same kernel, tiles and fused epilogues, only the weight format differs.
//
// An fp32-MFMA kernel (v_mfma_f32_16x16x4_f32, exact fp32 fma chain) is the path for shapes
// the bf16x3 kernel does not take (K % 4 != 0, misaligned A, B image over the LDS budget).
#include <cstdlib>

#include "ob_drop.h"
#include "ob_fp.h"
#include "ob_ln.h"
#include "ob_launch.h"
#include "ob_quant.h"

namespace ob {

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kThreads = 256;  // 4 waves
constexpr int kRows = 64;      // rows per row tile (16 per wave)
constexpr size_t kMaxLds = 80 * 1024;  // B image + epilogue staging: 2 blocks per CU
constexpr int kTargetBlocks = 512;  // 2 per CU
// K > 256 (K = 576: 18 chunks a row tile, NT 3): one block per CU. The 504-block grid left
// 13 of 56 row groups with a third 64-row tile (125 row tiles a pass) and CUs holding two
// such blocks: waves in flight averaged 1.27 per SIMD (tools/tgemm_stamps.py) and the
// launch ended on that tail. 252 blocks of <= 5 tiles: lin2 fwd 31.3 -> 27.4 us, lin1 dX
// 32.8 -> 29.2 us same box; the K = 144 launches stay at 512 (256 measured 2-6 us slower).
// (profiles/r4/tgemm_blocks/)
constexpr int kTargetBlocksLongK = 256;
// waves a byte-image block (K = 576; the q / k / v input-gradient sum): 8, two per SIMD
constexpr int kByteWaves = 8;
constexpr int kBPad = 16;           // B-image row pad (bf16 elements), see the header
// Byte image (K = 576 and N a multiple of 144: all 144 columns of a row tile in one block,
// so each A element is split once instead of once per 48 columns): one byte per weight,
// the high byte of the bf16 of Q/2 (0x00 -> 0, 0x3F -> +0.5, 0xBF -> -0.5; the low byte
// 0); the epilogue scales by 2a, so every product and sum is the bf16-image one halved
// exactly. 84 KB of LDS: one block (4 waves, up to 512 registers each) per CU. Row pitch
// Kpad + 8 bytes = 146 dwords at K = 576: the 16 lanes of a ds_read_b64 group on disjoint
// bank pairs. Same box: lin2 fwd 26.9 -> 20.9 us, lin1 dX 28.4 -> 22.8 us, lin2 fwd +
// residual 29.7 -> 26.8 us (profiles/r4/tgemm_blocks/kbench_byte_image.log).
constexpr int kBytePad = 8;

// code word (16 two-bit codes) -> 16 image bytes as 4 dwords (byte p of dword q = code 4q+p)
__device__ __forceinline__ void code_bytes(uint32_t word, u32x4& out) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t x = (word >> (8 * q)) & 0xFFu;                         // codes 4q .. 4q+3
    x = (x | (x << 6) | (x << 12) | (x << 18)) & 0x03030303u;       // one code per byte
    const uint32_t lo = x & 0x01010101u, hi = x & 0x02020202u;
    out[q] = ((lo << 6) - lo) | (hi << 6);                          // 1 -> 0x3F, 3 -> 0xBF
  }
}

// 8 image bytes (k .. k+7) -> the bf16x8 B fragment (byte = high byte, low byte 0)
__device__ __forceinline__ bf16x8 bytes_bf16x8(uint32_t d0, uint32_t d1) {
  u32x4 o;
  o[0] = __builtin_amdgcn_perm(d1, d0, 0x010C000Cu);
  o[1] = __builtin_amdgcn_perm(d1, d0, 0x030C020Cu);
  o[2] = __builtin_amdgcn_perm(d1, d0, 0x050C040Cu);
  o[3] = __builtin_amdgcn_perm(d1, d0, 0x070C060Cu);
  return __builtin_bit_cast(bf16x8, o);
}

#ifdef OB_TGEMM_STAMPS
// diagnostic build only (tools/tgemm_stamps.py): per wave the cycles of the prologue (B
// decode + barrier), of the main loops and of the epilogues, the row tiles done, and
// s_memrealtime (100 MHz) at start and end -- into buffers nothing else reads
__device__ uint64_t g_tg_stamps[32768];
__device__ uint64_t g_tg_rt[16384];
#define TG_DECL                                                              \
  uint64_t tg_t = __builtin_amdgcn_s_memtime(), tg_rt0 = __builtin_amdgcn_s_memrealtime(), \
           tg_acc[4] = {0, 0, 0, 0};
#define TG_STAMP(k)                                       \
  do {                                                    \
    const uint64_t tg_n = __builtin_amdgcn_s_memtime();   \
    tg_acc[k] += tg_n - tg_t;                             \
    tg_t = tg_n;                                          \
  } while (0)
#define TG_WRITE                                                                          \
  {                                                                                       \
    const uint64_t tg_rt1 = __builtin_amdgcn_s_memrealtime();                             \
    const size_t tg_w = ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * (blockDim.x / 64) + wave; \
    if (lane == 0 && tg_w * 4 + 4 <= 32768)                                               \
      for (int k_ = 0; k_ < 4; ++k_) g_tg_stamps[tg_w * 4 + k_] = tg_acc[k_];             \
    if (lane == 0 && tg_w * 2 + 2 <= 16384) {                                             \
      g_tg_rt[tg_w * 2] = tg_rt0;                                                         \
      g_tg_rt[tg_w * 2 + 1] = tg_rt1;                                                     \
    }                                                                                     \
  }
#else
#define TG_DECL
#define TG_STAMP(k) \
  do {              \
  } while (0)
#define TG_WRITE
#endif

__device__ __forceinline__ uint32_t code_bf16(uint32_t c) {
  return ((c & 1u) * 0x3F80u) | ((c & 2u) << 14);  // 0 -> 0, 1 -> +1.0, 3 -> -1.0
}

// x = hi + mid + lo exactly (RNE at each step; the residuals are exact in fp32).
__device__ __forceinline__ void split3(const f32x4& a, const f32x4& b, bf16x8& hi, bf16x8& mid,
                                       bf16x8& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float x = j < 4 ? a[j] : b[j - 4];
    const __bf16 h = (__bf16)x;
    const float r1 = x - (float)h;
    const __bf16 m = (__bf16)r1;
    const float r2 = r1 - (float)m;
    hi[j] = h;
    mid[j] = m;
    lo[j] = (__bf16)r2;
  }
}

__device__ __forceinline__ f32x4 mfma_bf16(const bf16x8& a, const bf16x8& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// Kernel-side form of TgemmEpi (ob_launch.h): the dropout config resolved on the host.
struct EpiArgs {
  // layers sharing A (q / k / v of one LN output) in one launch: the column tiles of layer i
  // follow those of layer i-1; glayers == 1: one layer (the kernel's own pointers)
  int glayers;
  const uint32_t* gcodes[3];
  const uint32_t* gcodes1[3];
  const float* galpha[3];
  const float* gbias[3];
  float* gC[3];
  // MS > 1 (the dX of q / k / v summed in one launch): the A operand of source s (its rows
  // [P][M][K]); source s reduces against gcodes[s] / gcodes1[s], scaled by galpha[s]
  const float* gA[3];
  // LayerNorms of the produced rows (residual epilogue, NT 9 byte image: a wave's 16 rows are
  // complete in its registers): nln of them, LN 1 of LN 0's output (ob_ln.h: the LN kernels'
  // own row code, so the results equal ob_layernorm_fwd / _pair bit for bit)
  int nln;
  const float* lng[2];
  const float* lnb[2];
  float lneps[2];
  float* lny[2];
  float* lnmean[2];
  float* lnrstd[2];
  int mode;
  const float* R;
  float* C2;
  float rscale;
  const int* lens;
  int T;
  DropCfg dc;
  const uint64_t* rng;
  uint64_t rng_off;
};

// torch's silu and silu backward formulas: x / (1 + exp(-x)) and
// (dy * s) * (1 + x * (1 - s)), s = 1 / (1 + exp(-x)), evaluated in that order.
// Fast math (ob_fp.h): exp through v_exp_f32 and the reciprocal through v_rcp_f32 -- a few
// ulp from torch's expf-based formula, well inside the fused-vs-unfused bar of
// tests/test_fused_gpu.py (1e-6 of max|ref|). (HIP's __fdividef / __frcp_rn are full IEEE
// divisions: ~10 VALU ops per element in these epilogues.)
__device__ __forceinline__ float silu_f(float z) { return fast_silu(z); }
__device__ __forceinline__ float silu_bwd_f(float dy, float z) {
  const float s = fast_sigmoid(z);
  return nc_mul(nc_mul(dy, s), 1.0f + z * (1.0f - s));
}

// Store y = a*acc + b through the fused epilogue. `c` is this element's output address,
// grow its pass-inclusive row. Non-contracting ops (ob_fp.h) keep hipcc from contracting the unfused
// reference sequence (y, then *scale, then +R) into an fma.
template <int MODE>
__device__ __forceinline__ void epi_store(const EpiArgs& ep, uint32_t dkey, float* c,
                                          int64_t grow, int col, int N, float y, float rv) {
  const int64_t i = grow * N + col;
  const float keep =
      ep.dc.on ? (drop_keep(dkey, (uint64_t)i, ep.dc.thresh) ? ep.dc.scale : 0.0f) : 1.0f;
  if constexpr (MODE == kEpiSwishDrop) {
    ep.C2[i] = y;
    const float sv = silu_f(y);
    *c = ep.dc.on ? nc_mul(sv, keep) : sv;
  } else if constexpr (MODE == kEpiResidual) {
    bool valid = true;
    if (ep.lens) {
      const int64_t b = grow / ep.T;
      valid = (grow - b * ep.T) < ep.lens[b];
    }
    float v = ep.dc.on ? nc_mul(y, keep) : y;
    v = valid ? v : nc_mul(v, 0.0f);
    *c = nc_add(rv, ep.rscale == 1.0f ? v : nc_mul(ep.rscale, v));
  } else {  // kEpiSwishDropBwd
    const float d = ep.dc.on ? nc_mul(y, keep) : y;
    *c = silu_bwd_f(d, rv);
  }
}

// Bijective XCD-aware remap (cdna_hip_programming.md §5 "XCD swizzle must be
// bijective"): consecutive logical ids land on one XCD under round-robin dispatch.
__device__ __forceinline__ int xcd_logical(int b, int nb) {
  const int q = nb / 8, r = nb % 8, x = b % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

// Two dwordx4 of one row at k and k+4. The address is clamped into the row instead of
// guarding the load: a guarded `cond ? *p : 0` makes hipcc branch around the load and wait
// vmcnt(0) at it. Clamped k positions (k >= K) meet zero codes, so they add nothing; rows
// past M are clamped to a valid row and never stored.
__device__ __forceinline__ void load8(const float* __restrict__ arow, int k, int K, f32x4& a,
                                      f32x4& b) {
  const int ka = k < K - 4 ? k : K - 4;
  const int kb = k + 4 < K - 4 ? k + 4 : K - 4;
  a = *reinterpret_cast<const f32x4*>(arow + ka);
  b = *reinterpret_cast<const f32x4*>(arow + kb);
}

// Stacked passes (pass_bits != nullptr): blockIdx.y = pass p; the pass's rows are
// A[p*M .. p*M+M) / C[p*M ..), and its codes are codes1 when pass_bits[p] == 1, else codes.
__device__ __forceinline__ void select_pass(const float* __restrict__& A, float* __restrict__& C,
                                            const uint32_t* __restrict__& codes,
                                            const uint32_t* codes1, const int* pass_bits,
                                            int64_t M, int K, int N) {
  if (!pass_bits) return;
  const int p = blockIdx.y;
  if (pass_bits[p] == 1) codes = codes1;
  A += (int64_t)p * M * K;
  C += (int64_t)p * M * N;
}

// byte offset of the epilogue staging tiles (after the B image, 16-B aligned) and their size
__host__ __device__ inline size_t epi_stage_off(int nt, int kpad, bool byte = false) {
  return ((byte ? (size_t)16 * nt * (kpad + kBytePad) : (size_t)2 * 16 * nt * (kpad + kBPad)) + 15) &
         ~(size_t)15;
}
__host__ __device__ inline size_t epi_stage_bytes(int nt, int waves = 4) {
  const int cw = nt < 4 ? nt : 4;
  return (size_t)waves * 16 * (16 * cw + 4) * sizeof(float);
}

// The same epilogue for 4 consecutive columns of one row (col % 4 == 0, N % 4 == 0): R loaded
// and C / C2 stored as dwordx4, so 16 lanes cover 256 contiguous bytes of the row.
template <int MODE>
__device__ __forceinline__ f32x4 epi_store4(const EpiArgs& ep, uint32_t dkey, float* c,
                                           int64_t grow, int col, int N, f32x4 y, bool valid,
                                           const f32x4& rv) {
  const int64_t i = grow * N + col;
  float keep[4] = {1.f, 1.f, 1.f, 1.f};
  if (ep.dc.on) drop_scale4(dkey, (uint64_t)i, ep.dc, keep);  // i % 4 == 0
  f32x4 out;
  if constexpr (MODE == kEpiNone) {
    out = y;
  } else if constexpr (MODE == kEpiSwishDrop) {
    *reinterpret_cast<f32x4*>(ep.C2 + i) = y;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float sv = silu_f(y[e]);
      out[e] = ep.dc.on ? nc_mul(sv, keep[e]) : sv;
    }
  } else if constexpr (MODE == kEpiResidual) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float v = ep.dc.on ? nc_mul(y[e], keep[e]) : y[e];
      v = valid ? v : nc_mul(v, 0.0f);
      out[e] = nc_add(rv[e], ep.rscale == 1.0f ? v : nc_mul(ep.rscale, v));
    }
  } else {  // kEpiSwishDropBwd
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float dd = ep.dc.on ? nc_mul(y[e], keep[e]) : y[e];
      out[e] = silu_bwd_f(dd, rv[e]);
    }
  }
  *reinterpret_cast<f32x4*>(c) = out;
  return out;
}

// MS (multi-source, > 1 only with BYTE): C = sum_s alpha_s A_s . Q_s over MS sources that share
// the output (the k / v / q input gradients of one LayerNorm output): the reduction runs over
// MS segments of NCH / MS chunks (K per source, zero-padded to 32 * NCH / MS), each chunk's A
// from its source, pre-scaled by that source's alpha (fp32 multiply: the product the
// reference forms with its alpha * Q weight, quant.py:126), the byte image holding the MS
// code blocks side by side.
// WV waves a block (8 for the byte-image launches: two per SIMD beside the one 84 KB image a
// CU holds, so one wave's loads / epilogue run under the other's MFMAs). Rows (n16 16-row
// subtiles a pass): WV > 4 -- an even, contiguous share of the subtiles per row group, dealt
// round-robin to the block's waves; WV == 4 -- 64-row tiles dealt round-robin to the row
// groups (measured 0.4-0.9 us a call faster than the even share for the K = 144 launches).
template <int NT, int NCH, int EPI, bool VEC_EPI, bool BYTE = false, int MS = 1, int WV = 4>
__global__ __launch_bounds__(64 * WV, BYTE ? 1 : 2) void tgemm_bf16x3_kernel(
    const float* __restrict__ A, int64_t M, int K, const uint32_t* __restrict__ codes, int KW,
    int N, int n_ct, int n16, int rgroups, const float* __restrict__ alpha, int alpha_raw,
    const float* __restrict__ bias, float* __restrict__ C, const uint32_t* __restrict__ codes1,
    const int* __restrict__ pass_bits, EpiArgs ep) {
  TG_DECL
  constexpr int kThr = 64 * WV;
  const int L = xcd_logical(blockIdx.x, gridDim.x);
  const int n_ct_l = n_ct / ep.glayers;  // column tiles of one layer
  if (ep.glayers > 1) {
    const int layer = (L % n_ct) / n_ct_l;
    codes = ep.gcodes[layer];
    codes1 = ep.gcodes1[layer];
    alpha = ep.galpha[layer];
    bias = ep.gbias[layer];
    C = ep.gC[layer];
  }
  select_pass(A, C, codes, codes1, pass_bits, M, K, N);
  const int64_t rowbase = pass_bits ? (int64_t)blockIdx.y * M : 0;
  static_assert(MS == 1 || (BYTE && NCH % MS == 0 && MS <= 3), "multi-source: byte image");
  constexpr int NCHS = NCH / MS;  // chunks per source
  // (three named scalars, not arrays: a runtime-indexed private array lives in scratch)
  const float *As0 = A, *As1 = A, *As2 = A;
  const uint32_t *Cs0 = codes, *Cs1 = codes, *Cs2 = codes;
  float al0 = 1.0f, al1 = 1.0f, al2 = 1.0f;
  if constexpr (MS > 1) {
    const bool one = pass_bits && pass_bits[blockIdx.y] == 1;
    As0 = ep.gA[0] + rowbase * (int64_t)K;
    As1 = ep.gA[1] + rowbase * (int64_t)K;
    As2 = ep.gA[2] + rowbase * (int64_t)K;
    Cs0 = one ? ep.gcodes1[0] : ep.gcodes[0];
    Cs1 = one ? ep.gcodes1[1] : ep.gcodes[1];
    Cs2 = one ? ep.gcodes1[2] : ep.gcodes[2];
    al0 = effective_alpha(ep.galpha[0], alpha_raw);
    al1 = effective_alpha(ep.galpha[1], alpha_raw);
    al2 = effective_alpha(ep.galpha[2], alpha_raw);
  }
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __bf16* bimg = reinterpret_cast<__bf16*>(smem);
  const int kpad = NCH > 0 ? 32 * NCH : ((K + 31) & ~31);
  const int stride = BYTE ? kpad + kBytePad : kpad + kBPad;  // image row pitch (bytes / bf16)
  const int kwp = kpad >> 4;
  // row-coalesced epilogue (vec_epi): per-wave staging [16][kEpiCC + 4] after the B image
  constexpr int kEpiCW = NT < 4 ? NT : 4, kEpiCC = 16 * kEpiCW, kEpiLd = kEpiCC + 4;
  // VEC_EPI (host-checked: N % 4 == 0, C / C2 / R 16-B aligned): the row-coalesced epilogue

  const int ct = (L % n_ct) % n_ct_l;
  const int rg = L / n_ct;
  const int n0 = ct * (16 * NT);
  // this row group's subtiles [s0, s1) (rgroups <= n16 / WV: at least one per wave), or its
  // 64-row tiles rg, rg + rgroups, ... (subtiles 4 rt .. 4 rt + 3)
  constexpr bool kShare = WV > 4;
  const int s0 = (int)((int64_t)rg * n16 / rgroups), s1 = (int)((int64_t)(rg + 1) * n16 / rgroups);
  const int n_rt4 = (n16 + 3) >> 2;

  // Decode this block's Q rows: one code word -> 16 bf16 (two 16-byte LDS stores).
  // Consecutive threads take consecutive words of the block's (contiguous) code rows, and
  // every word of the thread is loaded before any is decoded, so the prologue pays one
  // L2 latency instead of one per word.
  const int nwords = 16 * NT * kwp;
  auto decode_store = [&](int idx, uint32_t word) {
    const int nl = idx / kwp, w = idx - nl * kwp;
    // (multi-source: the pad words of each source block are zeroed by word_at)
    word = (n0 + nl < N && (MS > 1 || w < KW) && idx < nwords) ? word : 0u;
    if constexpr (BYTE) {
      u32x4 b4;
      code_bytes(word, b4);
      // the byte image's row pitch (kpad + 8 bytes) makes odd rows 8-byte aligned only: two
      // 8-byte stores (ds_write_b64), no reliance on unaligned-DS mode for a 16-byte one
      if (idx < nwords) {
        typedef uint32_t u32x2a __attribute__((ext_vector_type(2), aligned(8)));
        u32x2a* dst = reinterpret_cast<u32x2a*>(smem + nl * stride + 16 * w);
        dst[0] = u32x2a{b4[0], b4[1]};
        dst[1] = u32x2a{b4[2], b4[3]};
      }
      return;
    }
    u32x4 lo4, hi4;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      lo4[p] = code_bf16((word >> (4 * p)) & 3u) | (code_bf16((word >> (4 * p + 2)) & 3u) << 16);
      hi4[p] = code_bf16((word >> (4 * p + 16)) & 3u) |
               (code_bf16((word >> (4 * p + 18)) & 3u) << 16);
    }
    if (idx < nwords) {
      u32x4* dst = reinterpret_cast<u32x4*>(bimg + nl * stride + 16 * w);
      dst[0] = lo4;
      dst[1] = hi4;
    }
  };
  auto word_at = [&](int idx) -> uint32_t {
    const int nl = idx / kwp, w = idx - nl * kwp;
    int64_t n = n0 + nl;
    n = n < N ? n : N - 1;
    if constexpr (MS > 1) {  // source block q = w / (kwp / MS), its word ws
      const int wps = kwp / MS, q = w / wps, ws = w - q * wps;
      // the source's base as an offset from source 0 by arithmetic (a select chain over the
      // three pointers became a private lookup table in scratch)
      const int64_t off = (int64_t)(q == 1) * (Cs1 - Cs0) + (int64_t)(q == 2) * (Cs2 - Cs0);
      const uint32_t v = Cs0[off + n * KW + (ws < KW ? ws : KW - 1)];
      return ws < KW ? v : 0u;
    }
    const int wc = w < KW ? w : KW - 1;
    return codes[n * KW + wc];  // clamped, always valid; out-of-range words are zeroed above
  };
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int r = lane & 15;
  const int g = lane >> 4;
  const int kg = 8 * g;
  auto arow_of = [&](int j) {  // row r of subtile j (clamped into M)
    const int64_t row = (int64_t)16 * j + r < M ? (int64_t)16 * j + r : M - 1;
    return A + row * (int64_t)K;
  };
  // row loop: it = subtile (share) or 64-row tile (round-robin), this wave's subtile jof(it)
  const int it0 = kShare ? s0 + wave : rg, itN = kShare ? s1 : n_rt4, istep = kShare ? WV : rgroups;
  auto jof = [&](int it) { return kShare ? it : 4 * it + wave; };
  // chunk c of a row tile (arow = arow_of's pointer): multi-source, chunk c is chunk c % NCHS
  // of source c / NCHS (c is a compile-time constant wherever the chunk loops are unrolled)
  auto ldc = [&](const float* arow, int c, f32x4& x, f32x4& y) {
    if constexpr (MS > 1) {
      const int q = c / NCHS;
      const float* src = q == 0 ? As0 : (q == 1 ? As1 : As2);
      load8(src + (arow - A), 32 * (c - q * NCHS) + kg, K, x, y);
    } else {
      load8(arow, 32 * c + kg, K, x, y);
    }
  };
  // K compile-time (NCH > 0): A chunks are software-pipelined ACROSS row tiles. The first
  // tile's first kWin chunks are issued right after the code words (so the B decode and
  // the barrier run under their latency), and while a tile computes its last chunks the
  // next tile's first chunks are already loading (so the epilogue runs under them too).
  // vmcnt counts in issue order: the code words go first so the decode waits only on them.
#ifndef OB_TG_KWMAX_WIDE
#define OB_TG_KWMAX_WIDE 3
#endif
  // (multi-source: one block per CU with registers to spare, a deeper window)
#ifndef OB_TG_KWMAX_BYTE8
#define OB_TG_KWMAX_BYTE8 2  // (8-wave byte image: 2 chunks ahead 36.8 us a residual-LN call, 3: 38.1, 4: 40.1)
#endif
  constexpr int kWmax = MS > 1 ? 5 : (BYTE && WV > 4) ? OB_TG_KWMAX_BYTE8 : NT > 6 ? OB_TG_KWMAX_WIDE : 5;
  // NT 12: the cross-tile live range spills (and a 2-deep window measured slower), so it
  // keeps the per-tile window (issued at the top of each row tile)
  constexpr bool kCross = NT <= 9;
  constexpr int kWin = NCH > 0 ? (NCH < kWmax ? NCH : kWmax) : 1;
  f32x4 buf[NCH > 0 ? NCH : 1][2];
  // quant-off (alpha_raw 2): the LDS image is a copy of the block's rows of the bf16 weight
  // image [N][K]. Unit = 8 consecutive k of one row (one 16-byte load and store).
  auto weight_image = [&]() {
    if constexpr (BYTE) return;  // (the host never pairs the byte image with alpha_raw 2)
    const uint16_t* Wb = reinterpret_cast<const uint16_t*>(codes);
    const int upr = kpad >> 3;
    for (int u = threadIdx.x; u < 16 * NT * upr; u += kThr) {
      const int nl = u / upr, k0 = 8 * (u - nl * upr);
      const int n = n0 + nl;
      u32x4 v = u32x4{0u, 0u, 0u, 0u};
      if (n < N && (K & 7) == 0 && k0 + 8 <= K) {
        v = *reinterpret_cast<const u32x4*>(Wb + (int64_t)n * K + k0);
      } else if (n < N) {
        uint16_t h[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) h[j] = k0 + j < K ? Wb[(int64_t)n * K + k0 + j] : (uint16_t)0;
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = (uint32_t)h[2 * q] | ((uint32_t)h[2 * q + 1] << 16);
      }
      *reinterpret_cast<u32x4*>(bimg + nl * stride + k0) = v;
    }
  };
  if constexpr (NCH > 0) {
    if (alpha_raw >= 2) {
      if constexpr (kCross) {
        const float* a0 = arow_of(jof(it0 < itN ? it0 : rg));
#pragma unroll
        for (int c = 0; c < kWin; ++c) ldc(a0, c, buf[c][0], buf[c][1]);
      }
      __builtin_amdgcn_sched_barrier(0);
      weight_image();
    } else {
      constexpr int kWpt = (16 * NT * 2 * NCH + kThr - 1) / kThr;
      uint32_t wv[kWpt];
#pragma unroll
      for (int i = 0; i < kWpt; ++i) wv[i] = word_at(threadIdx.x + i * kThr);
      if constexpr (kCross) {
        const float* a0 = arow_of(jof(it0 < itN ? it0 : rg));  // (a real row, clamped)
#pragma unroll
        for (int c = 0; c < kWin; ++c) ldc(a0, c, buf[c][0], buf[c][1]);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < kWpt; ++i) decode_store(threadIdx.x + i * kThr, wv[i]);
    }
  } else if (alpha_raw >= 2) {
    weight_image();
  } else {
    for (int idx = threadIdx.x; idx < nwords; idx += kThr) decode_store(idx, word_at(idx));
  }
  // The residual byte launch's LayerNorm parameters (ep.nln, N = 144): gamma 0, beta 0,
  // gamma 1, beta 1 staged once per block after the epilogue tiles (an absent gamma / beta
  // as 1 / 0: the same fmaf) -- at one wave per SIMD nothing hides a global load's latency in
  // the per-row-group LN.
  [[maybe_unused]] float* lnp = nullptr;
  if constexpr (EPI == kEpiResidual && BYTE && NT == 9 && MS == 1) {
    lnp = reinterpret_cast<float*>(smem + epi_stage_off(NT, kpad, BYTE) +
                                   (size_t)WV * 16 * (16 * NT + 4) * sizeof(float));
    if (ep.nln > 0 && threadIdx.x < 16 * NT) {
      const int c = threadIdx.x;
      lnp[c] = ep.lng[0] ? ep.lng[0][c] : 1.0f;
      lnp[16 * NT + c] = ep.lnb[0] ? ep.lnb[0][c] : 0.0f;
      lnp[32 * NT + c] = ep.nln > 1 && ep.lng[1] ? ep.lng[1][c] : 1.0f;
      lnp[48 * NT + c] = ep.nln > 1 && ep.lnb[1] ? ep.lnb[1][c] : 0.0f;
    }
  }
  __syncthreads();
  TG_STAMP(0);

  const __bf16* brow = bimg + r * stride + kg;
  const unsigned char* brow8 = reinterpret_cast<const unsigned char*>(smem) + r * stride + kg;
  const float a_eff = MS > 1 ? 2.0f
                      : BYTE ? 2.0f * effective_alpha(alpha, alpha_raw)
                             : effective_alpha(alpha, alpha_raw);
  const uint32_t dkey = (EPI != kEpiNone && ep.dc.on) ? drop_key(ep.rng[0], ep.rng[1] + ep.rng_off) : 0u;
  float bcol[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int col = n0 + 16 * t + r;
    bcol[t] = (bias && col < N) ? bias[col] : 0.0f;
  }

  for (int it = it0; it < itN; it += istep) {
    const int64_t m0 = (int64_t)16 * jof(it);
    const float* arow = arow_of(jof(it));

    f32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};

    // All B fragments of the chunk are read first and the split runs while they are in
    // flight; each tile's MFMAs then wait only for their own read (counted lgkmcnt).
    auto compute = [&](const f32x4& x0in, const f32x4& x1in, int kc) {
      f32x4 x0 = x0in, x1 = x1in;
      if constexpr (MS > 1) {  // alpha of the chunk's source, applied before the exact split
        const int q = (kc >> 5) / NCHS;
        const float al = q == 0 ? al0 : (q == 1 ? al1 : al2);
#pragma unroll
        for (int j = 0; j < 4; ++j) {  // rounded products (no contraction into the split)
          x0[j] = nc_mul(x0[j], al);
          x1[j] = nc_mul(x1[j], al);
        }
      }
      bf16x8 bq[NT];
      typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
      u32x2 bb[BYTE ? NT : 1];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        if constexpr (BYTE)
          bb[t] = *reinterpret_cast<const u32x2*>(brow8 + t * 16 * stride + kc);
        else
          bq[t] = *reinterpret_cast<const bf16x8*>(brow + t * 16 * stride + kc);
      }
      __builtin_amdgcn_sched_barrier(0);  // keep the reads ahead (hipcc would pair them up)
      bf16x8 hi, mid, lo;
      split3(x0, x1, hi, mid, lo);
      if constexpr (BYTE) {
        // tile-major: a fragment is converted right before its three MFMAs (one live at a
        // time; dependent 16x16x32 MFMAs issue back to back at full rate), the same
        // per-accumulator order lo, mid, hi as the part-major loops below
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const bf16x8 b = bytes_bf16x8(bb[t][0], bb[t][1]);
          acc[t] = mfma_bf16(lo, b, acc[t]);
          acc[t] = mfma_bf16(mid, b, acc[t]);
          acc[t] = mfma_bf16(hi, b, acc[t]);
        }
        return;
      }
      // part-major: consecutive MFMAs update different accumulators (no back-to-back
      // dependence on the MFMA just issued)
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = mfma_bf16(lo, bq[t], acc[t]);
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = mfma_bf16(mid, bq[t], acc[t]);
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = mfma_bf16(hi, bq[t], acc[t]);
    };

    if constexpr (NCH > 0) {
      // Fully unrolled; a window of kWin chunks in flight (this tile's chunks 0..kWin-1
      // were issued by the previous iteration / the prologue). sched_barrier keeps hipcc
      // from sinking each load next to its use (one load in flight, vmcnt(0) per chunk).
      // The last tile re-reads its own rows as the "next" tile (L2 hits, never used).
      if constexpr (!kCross) {  // NT 12: this tile's window is issued here (no cross-tile)
#pragma unroll
        for (int c = 0; c < kWin; ++c) ldc(arow, c, buf[c][0], buf[c][1]);
        __builtin_amdgcn_sched_barrier(0);
      }
      const float* anext = arow_of(jof(it + istep < itN ? it + istep : it));
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        if (c + kWin < NCH)
          ldc(arow, c + kWin, buf[c + kWin][0], buf[c + kWin][1]);
        __builtin_amdgcn_sched_barrier(0);
        compute(buf[c][0], buf[c][1], 32 * c);
        // next tile's chunk into the slot just consumed (slot c + kWin - NCH <= c; it IS
        // slot c when kWin == NCH, so the load must follow this chunk's compute)
        if constexpr (kCross) {
          if (c + kWin >= NCH) {
            ldc(anext, c + kWin - NCH, buf[c + kWin - NCH][0], buf[c + kWin - NCH][1]);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
      }
    } else {
      // Generic K: three rotating register sets, unrolled so no register copy of an
      // in-flight load exists (a copy would make hipcc wait for it).
      f32x4 r0a, r0b, r1a, r1b, r2a, r2b;
      load8(arow, kg, K, r0a, r0b);
      load8(arow, 32 + kg, K, r1a, r1b);
      for (int kc = 0; kc < kpad; kc += 96) {
        load8(arow, kc + 64 + kg, K, r2a, r2b);
        compute(r0a, r0b, kc);
        load8(arow, kc + 96 + kg, K, r0a, r0b);
        if (kc + 32 < kpad) compute(r1a, r1b, kc + 32);
        load8(arow, kc + 128 + kg, K, r1a, r1b);
        if (kc + 64 < kpad) compute(r2a, r2b, kc + 64);
      }
    }

    // keep the epilogue's loads (residual / pre-activation) from being hoisted into the
    // main loop, where they would hold NT*4 VGPRs across it
    __builtin_amdgcn_sched_barrier(0);
    TG_STAMP(1);
#ifdef OB_TGEMM_STAMPS
    ++tg_acc[3];
#endif
    if constexpr (VEC_EPI) {
      // Row-coalesced epilogue: each chunk of <= 4 column tiles goes through the wave's LDS
      // staging tile, then every lane handles 4 consecutive columns of one row (dwordx4 R
      // loads and C / C2 stores; 16 lanes = 256 contiguous bytes). The wave's LDS ops run
      // in issue order; the waitcnt + sched barriers keep hipcc from reordering across them.
      float* stg = reinterpret_cast<float*>(smem + epi_stage_off(NT, kpad, BYTE)) + wave * 16 * kEpiLd;
      constexpr int kQ = kEpiCC / 4;  // float4s per staged row
      // The residual byte-image launch (the FFN lin2 of every block): all 144 columns of the
      // wave's 16 rows staged at once, then row group by row group (16 lanes a row, lane j
      // columns 4 (j + 16 i): ob_ln.h's LN row mapping) the residual output formed, stored,
      // and -- ep.nln -- normalised in registers: the LayerNorm(s) that read this output next
      // need no launch of their own.
      if constexpr (EPI == kEpiResidual && BYTE && NT == 9 && MS == 1) {
        constexpr int kLd = 16 * NT + 4;  // staged row pitch (floats)
        float* st = reinterpret_cast<float*>(smem + epi_stage_off(NT, kpad, BYTE)) + wave * 16 * kLd;
        const int c4 = lane & 15;
        auto r_of = [&](int it, f32x4 (&rr)[3]) {  // the residual operand of row group it
          const int64_t orow = m0 + it * 4 + (lane >> 4);
          const int64_t rr_row = rowbase + (orow < M ? orow : M - 1);
#pragma unroll
          for (int i = 0; i < 3; ++i) {
            const int col = min(n0 + 64 * i + 4 * c4, N - 4);
            rr[i] = *reinterpret_cast<const f32x4*>(ep.R + rr_row * N + col);
          }
        };
        f32x4 rr[2][3];
        r_of(0, rr[0]);
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int reg = 0; reg < 4; ++reg)
            st[(4 * g + reg) * kLd + 16 * t + r] = fmaf(a_eff, acc[t][reg], bcol[t]);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int it = 0; it < 4; ++it) {
          if (it + 1 < 4) r_of(it + 1, rr[(it + 1) & 1]);
          const int row = it * 4 + (lane >> 4);
          const int64_t orow = m0 + row;
          bool valid = true;
          if (ep.lens) {
            const int64_t grow = rowbase + orow;
            const int64_t bb = grow / ep.T;
            valid = (grow - bb * ep.T) < ep.lens[bb];
          }
          float v[3][4];
#pragma unroll
          for (int i = 0; i < 3; ++i) {
            const int cl = 64 * i + 4 * c4;  // column within the tile row
            f32x4 o = f32x4{0.f, 0.f, 0.f, 0.f};
            if (orow < M && cl < 16 * NT) {
              const f32x4 y = *reinterpret_cast<const f32x4*>(st + row * kLd + cl);
              o = epi_store4<EPI>(ep, dkey, C + orow * N + n0 + cl, rowbase + orow, n0 + cl, N, y,
                                  valid, rr[it & 1][i]);
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) v[i][e] = o[e];  // (zero past the row: the LN load)
          }
          if (ep.nln > 0 && orow < M) {  // (uniform over the row's 16 lanes: the DPP sums)
            float v2[3][4] = {};
            lnrow::ln_row_v<3, 4>(v, lnp, lnp + 16 * NT, rowbase + orow, N, ep.lneps[0],
                                  ep.lny[0], ep.lnmean[0], ep.lnrstd[0], nullptr, 0.0f, &v2);
            if (ep.nln > 1)
              lnrow::ln_row_v<3, 4>(v2, lnp + 32 * NT, lnp + 48 * NT, rowbase + orow, N,
                                    ep.lneps[1], ep.lny[1], ep.lnmean[1], ep.lnrstd[1]);
          }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        TG_STAMP(2);
        continue;
      }
      constexpr bool kHasR = EPI == kEpiResidual || EPI == kEpiSwishDropBwd;
      // residual rows past their utterance's length (pad-zeroed): a lane's rows are the same
      // in every column chunk, so each is tested once per row tile (32-bit division below
      // 2^31 rows)
      bool rvalid[kEpiCW];
#pragma unroll
      for (int it = 0; it < kEpiCW; ++it) {
        rvalid[it] = true;
        if (EPI == kEpiResidual && ep.lens) {
          const int64_t grow = rowbase + m0 + (it * 64 + lane) / kQ;
          if (grow < ((int64_t)1 << 31)) {
            const uint32_t bb = (uint32_t)grow / (uint32_t)ep.T;
            rvalid[it] = (int)((uint32_t)grow - bb * (uint32_t)ep.T) < ep.lens[bb];
          } else {
            const int64_t bb = grow / ep.T;
            rvalid[it] = (grow - bb * ep.T) < ep.lens[bb];
          }
        }
      }
#pragma unroll
      for (int c0 = 0; c0 < NT; c0 += kEpiCW) {
        // the chunk's residual / pre-activation operand, loaded unconditionally from clamped
        // addresses before the LDS staging: its latency runs under the staging instead of
        // one load-to-use wait per guarded store below
        f32x4 rpre[kEpiCW];
        if constexpr (kHasR) {
#pragma unroll
          for (int it = 0; it < kEpiCW; ++it) {
            const int idx = it * 64 + lane, row = idx / kQ, c4 = idx - row * kQ;
            const int64_t orow = m0 + row < M ? m0 + row : M - 1;
            const int col = min(n0 + 16 * c0 + 4 * c4, N - 4);
            rpre[it] = *reinterpret_cast<const f32x4*>(ep.R + (rowbase + orow) * N + col);
          }
        }
#pragma unroll
        for (int t = 0; t < kEpiCW; ++t) {
          if (c0 + t >= NT) continue;
#pragma unroll
          for (int reg = 0; reg < 4; ++reg)
            stg[(4 * g + reg) * kEpiLd + 16 * t + r] = fmaf(a_eff, acc[c0 + t][reg], bcol[c0 + t]);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int it = 0; it < kEpiCW; ++it) {
          const int idx = it * 64 + lane, row = idx / kQ, c4 = idx - row * kQ;
          const int64_t orow = m0 + row;
          const int col = n0 + 16 * c0 + 4 * c4;
          const f32x4 y = *reinterpret_cast<const f32x4*>(stg + row * kEpiLd + 4 * c4);
          // (the last chunk of an NT that is not a multiple of 4 holds fewer columns)
          if (orow < M && col < N && 4 * c4 < 16 * (NT - c0)) {
            if constexpr (EPI == kEpiNone) {
              *reinterpret_cast<f32x4*>(C + orow * N + col) = y;
              if (EPI == kEpiSwishDrop)
                *reinterpret_cast<f32x4*>(ep.C2 + (rowbase + orow) * N + col) = y;
            } else {
              epi_store4<EPI>(ep, dkey, C + orow * N + col, rowbase + orow, col, N, y, rvalid[it],
                              rpre[it]);
            }
          }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
      }
      TG_STAMP(2);
      continue;
    }
    if constexpr (!VEC_EPI) {

    // epilogue operand: all NT*4 loads issued before any is used (one latency, not 4*NT)
    // epilogue operand (residual / pre-activation): rolling prefetch kPre tiles ahead, so at
    // most (kPre + 1) * 4 values are live (all NT * 4 at once spilled at NT = 12)
    constexpr bool kHasR = EPI == kEpiResidual || EPI == kEpiSwishDropBwd;
    constexpr int kPre = 2;
    float rv[NT][4];
    auto load_r = [&](int t) {
      const int col = min(n0 + 16 * t + r, N - 1);
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int64_t orow = min(m0 + 4 * g + reg, M - 1);
        rv[t][reg] = ep.R[(rowbase + orow) * N + col];
      }
    };
    if constexpr (kHasR) {
#pragma unroll
      for (int t = 0; t < kPre && t < NT; ++t) load_r(t);
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      if constexpr (kHasR) {
        if (t + kPre < NT) load_r(t + kPre);
        __builtin_amdgcn_sched_barrier(0);
      }
      const int col = n0 + 16 * t + r;
      if (col >= N) continue;
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int64_t orow = m0 + 4 * g + reg;
        if (orow >= M) continue;
        const float y = fmaf(a_eff, acc[t][reg], bcol[t]);
        if constexpr (EPI == kEpiNone) {
          C[orow * N + col] = y;
          if (EPI == kEpiSwishDrop) ep.C2[(rowbase + orow) * N + col] = y;
        } else {
          epi_store<EPI>(ep, dkey, C + orow * N + col, rowbase + orow, col, N, y, rv[t][reg]);
        }
      }
      // one tile's elementwise work at a time: hipcc would otherwise interleave all NT*4
      // exp/div sequences and spill
      if constexpr (EPI != kEpiNone) __builtin_amdgcn_sched_barrier(0);
    }
    TG_STAMP(2);
    }
  }
  TG_WRITE
}

// ---------------------------------------------------------------------------------
// fp32-MFMA ternary GEMM (exact fp32 fma chain), 64 rows x 48 columns per block.
// Per 16-wide k chunk a lane loads X[row][kc+4g .. kc+4g+3] and one code word per n tile;
// byte g of that word holds the 4 codes of k = kc+4g+e, e = 0..3.
// ---------------------------------------------------------------------------------
constexpr int kF32NT = 3;

__global__ __launch_bounds__(kThreads) void tgemm_f32_kernel(
    const float* __restrict__ A, int64_t M, int64_t K, const uint32_t* __restrict__ codes,
    int64_t KW, int64_t N, const float* __restrict__ alpha, int alpha_raw,
    const float* __restrict__ bias, float* __restrict__ C, const uint32_t* __restrict__ codes1,
    const int* __restrict__ pass_bits, EpiArgs ep) {
  const int64_t rowbase = pass_bits ? (int64_t)blockIdx.z * M : 0;
  if (pass_bits) {  // stacked passes: blockIdx.z = pass
    const int p = blockIdx.z;
    if (pass_bits[p] == 1) codes = codes1;
    A += (int64_t)p * M * K;
    C += (int64_t)p * M * N;
  }
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int r = lane & 15;
  const int g = lane >> 4;
  const int64_t m0 = (int64_t)blockIdx.x * kRows + wave * 16;
  const int64_t n0 = (int64_t)blockIdx.y * (16 * kF32NT);
  const int64_t row = m0 + r < M ? m0 + r : M - 1;
  const float* arow = A + row * K;
  f32x4 acc[kF32NT];
#pragma unroll
  for (int t = 0; t < kF32NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int64_t kc = 0; kc < K; kc += 16) {
    float xa[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int64_t k = kc + 4 * g + e;
      xa[e] = arow[k < K ? k : K - 1];  // k >= K meets a zero code
    }
#pragma unroll
    for (int t = 0; t < kF32NT; ++t) {
      const int64_t n = n0 + 16 * t + r;
      if (alpha_raw >= 2) {  // quant-off: B from the bf16 weight image [N][K]
        const uint16_t* Wb = reinterpret_cast<const uint16_t*>(codes);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int64_t k = kc + 4 * g + e;
          const float w = (n < N && k < K) ? __uint_as_float((uint32_t)Wb[n * K + k] << 16) : 0.0f;
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[e], w, acc[t], 0, 0, 0);
        }
        continue;
      }
      const uint32_t word = codes[(n < N ? n : N - 1) * KW + (kc >> 4)];
      const uint32_t byte = (n < N) ? (word >> (8 * g)) : 0u;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[e], code_value((byte >> (2 * e)) & 3u),
                                                       acc[t], 0, 0, 0);
    }
  }
  const float a = effective_alpha(alpha, alpha_raw);
  const uint32_t dkey = ep.dc.on ? drop_key(ep.rng[0], ep.rng[1] + ep.rng_off) : 0u;
#pragma unroll
  for (int t = 0; t < kF32NT; ++t) {
    const int64_t col = n0 + 16 * t + r;
    if (col >= N) continue;
    const float b = bias ? bias[col] : 0.0f;
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      const int64_t orow = m0 + 4 * g + reg;
      if (orow >= M) continue;
      const float y = fmaf(a, acc[t][reg], b);
      float* c = C + orow * N + col;
      const float rv = ep.R ? ep.R[(rowbase + orow) * N + col] : 0.0f;
      if (ep.mode == kEpiNone) *c = y;
      else if (ep.mode == kEpiSwishDrop)
        epi_store<kEpiSwishDrop>(ep, dkey, c, rowbase + orow, (int)col, (int)N, y, rv);
      else if (ep.mode == kEpiResidual)
        epi_store<kEpiResidual>(ep, dkey, c, rowbase + orow, (int)col, (int)N, y, rv);
      else
        epi_store<kEpiSwishDropBwd>(ep, dkey, c, rowbase + orow, (int)col, (int)N, y, rv);
    }
  }
}

// The fp32-MFMA GEMM (tgemm_f32 kernels) serves the shapes the bf16x3 kernels do not take.
bool use_f32_gemm() { return false; }

size_t bimg_bytes(int nt, int64_t K) {
  const int64_t kpad = (K + 31) & ~int64_t(31);
  return sizeof(uint16_t) * (size_t)(16 * nt) * (size_t)(kpad + kBPad);
}

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// Widest column tile whose bf16 image fits the LDS budget, preferring tiles that divide N.
// Fused epilogues: widths whose instantiation spills are excluded (checked with
// -Rpass-analysis=kernel-resource-usage on the row-coalesced (VEC_EPI) kernels: every
// epilogue is spill-free up to NT 9 at K <= 160 and up to NT 4 beyond).
// K <= 160: the swish epilogues (lin1 forward, lin2 dX) at 64-column tiles -- 9 x 16
// columns measured 6 % / 2.4 % slower per launch than 4 (profiles/r5/ab_prof/r6o: the
// epilogue's VALU and stores spread over 2.25x the blocks); the residual epilogue keeps 9
// (3 tiles at N = 144 were 7 % slower); the plain launches at N = 144 (the grouped q / k / v
// forward, out_proj dX) take 3 tiles of 48 (8 % faster than 9 x 16: r6t)
bool epi_nt_ok(int nt, int64_t K, int epi_mode) {
  if (epi_mode == kEpiNone) return K > 160 || nt <= 4;
  if (K <= 160) return nt <= (epi_mode == kEpiResidual ? 9 : 4);
  return nt <= 4;
}

int pick_nt(int64_t N, int64_t K, int epi_mode) {
  static const int cands[] = {12, 9, 6, 4, 3, 2, 1};
  for (int nt : cands)
    if (epi_nt_ok(nt, K, epi_mode) && N % (16 * nt) == 0 &&
        bimg_bytes(nt, K) + 16 + epi_stage_bytes(nt) <= kMaxLds)
      return nt;
  for (int nt : cands)
    if (epi_nt_ok(nt, K, epi_mode) && 16 * nt <= ((N + 15) & ~int64_t(15)) &&
        bimg_bytes(nt, K) + 16 + epi_stage_bytes(nt) <= kMaxLds)
      return nt;
  return 0;
}

template <int NT>
void launch_bf16x3(const float* A, int64_t M, int64_t K, const uint32_t* codes, int64_t N,
                   const float* alpha, int alpha_raw, const float* bias, float* C,
                   const uint32_t* codes1, const int* pass_bits, int P, const EpiArgs& ep,
                   hipStream_t s, bool byte = false) {
  const int n_ct = ep.glayers * (int)ceil_div(N, 16 * NT);  // all layers' column tiles
  const int n16 = (int)ceil_div(M, 16);  // 16-row subtiles of a pass
  const int wv = byte ? kByteWaves : 4;
  // (the swish-backward epilogue -- lin2 dX, NT 4 -- at 768 blocks: 37.5 -> 35.8 us a call,
  // profiles/r5/ab_prof/r6w; the other K <= 256 kinds measured neutral or slower there)
  const int target = K > 256 ? kTargetBlocksLongK
                     : ep.mode == kEpiSwishDropBwd ? kTargetBlocks * 3 / 2
                                                   : kTargetBlocks;
  int rgroups = target / (n_ct * P);
  if (rgroups > ceil_div(n16, wv)) rgroups = (int)ceil_div(n16, wv);  // >= a subtile a wave
  if (rgroups < 1) rgroups = 1;
  const dim3 grid((unsigned)(rgroups * n_ct), (unsigned)P);
  const int kpad = (int)((K + 31) & ~int64_t(31));
  // (the residual byte-image launch stages all 16 * NT columns of a wave's rows at once)
  // (+ the LN parameters: 4 x 16 NT floats)
  const size_t lds = epi_stage_off(NT, kpad, byte) +
                     (byte && ep.mode == kEpiResidual
                          ? (size_t)wv * 16 * (16 * NT + 4) * sizeof(float) + 4 * 16 * NT * sizeof(float)
                          : epi_stage_bytes(NT, wv));
  const int KW = (int)ceil_div(K, 16);
  const bool vec = (N % 4 == 0) && aligned16(C) && (ep.mode != kEpiSwishDrop || aligned16(ep.C2)) &&
                   ((ep.mode != kEpiResidual && ep.mode != kEpiSwishDropBwd) || aligned16(ep.R));
#define OB_TGEMM_E(NCH, E)                                                                     \
  if (vec)                                                                                    \
    hipLaunchKernelGGL((tgemm_bf16x3_kernel<NT, NCH, E, true>), grid, dim3(kThreads), lds, s,  \
                       A, M, (int)K, codes, KW, (int)N, n_ct, n16, rgroups, alpha, alpha_raw,  \
                       bias, C, codes1, pass_bits, ep);                                         \
  else                                                                                        \
    hipLaunchKernelGGL((tgemm_bf16x3_kernel<NT, NCH, E, false>), grid, dim3(kThreads), lds, s, \
                       A, M, (int)K, codes, KW, (int)N, n_ct, n16, rgroups, alpha, alpha_raw,  \
                       bias, C, codes1, pass_bits, ep)
  if constexpr (NT == 9) {
    if (byte) {  // byte image: K = 576 (18 chunks), codes (alpha_raw < 2), plain / residual
#define OB_TGEMM_B(E)                                                                            \
  if (vec)                                                                                      \
    hipLaunchKernelGGL((tgemm_bf16x3_kernel<9, 18, E, true, true, 1, kByteWaves>), grid,         \
                       dim3(64 * kByteWaves), lds, s,                                            \
                       A, M, (int)K, codes, KW, (int)N, n_ct, n16, rgroups, alpha, alpha_raw,    \
                       bias, C, codes1, pass_bits, ep);                                           \
  else                                                                                          \
    hipLaunchKernelGGL((tgemm_bf16x3_kernel<9, 18, E, false, true, 1, kByteWaves>), grid,        \
                       dim3(64 * kByteWaves), lds,                                               \
                       s, A, M, (int)K, codes, KW, (int)N, n_ct, n16, rgroups, alpha, alpha_raw, \
                       bias, C, codes1, pass_bits, ep)
      if (ep.mode == kEpiResidual) OB_TGEMM_B(kEpiResidual);
      else OB_TGEMM_B(kEpiNone);
#undef OB_TGEMM_B
      return;
    }
  }
#define OB_TGEMM(NCH)                                                   \
  switch (ep.mode) {                                                    \
    case kEpiSwishDrop: OB_TGEMM_E(NCH, kEpiSwishDrop); break;          \
    case kEpiResidual: OB_TGEMM_E(NCH, kEpiResidual); break;            \
    case kEpiSwishDropBwd: OB_TGEMM_E(NCH, kEpiSwishDropBwd); break;    \
    default: OB_TGEMM_E(NCH, kEpiNone); break;                          \
  }
  switch ((K + 31) / 32) {  // Conformer widths: 64, 144, 256, 576
    case 2: OB_TGEMM(2); break;
    case 5: OB_TGEMM(5); break;
    case 8: OB_TGEMM(8); break;
    case 18: OB_TGEMM(18); break;
    default: OB_TGEMM(0); break;
  }
#undef OB_TGEMM
#undef OB_TGEMM_E
}

}  // namespace

void launch_ternary_gemm_passes(const float* A, int P, int64_t M, int64_t K,
                                const uint32_t* codes, const uint32_t* codes1,
                                const int* pass_bits, int64_t N, const float* alpha,
                                int alpha_raw, const float* bias, float* C, hipStream_t s,
                                const TgemmEpi* epi) {
  if (M == 0 || N == 0 || P == 0) return;
  EpiArgs ep{};
  ep.glayers = 1;
  ep.mode = kEpiNone;
  if (epi && epi->mode != kEpiNone) {
    ep.mode = epi->mode;
    ep.R = epi->R;
    ep.C2 = epi->C2;
    ep.rscale = epi->rscale;
    ep.lens = epi->lens;
    ep.T = epi->T > 0 ? epi->T : 1;
    ep.dc = make_drop(epi->p_drop);
    ep.rng = epi->rng;
    ep.rng_off = epi->rng_off;
    ep.nln = epi->nln;
    for (int i = 0; i < 2; ++i) {
      ep.lng[i] = epi->lng[i];
      ep.lnb[i] = epi->lnb[i];
      ep.lneps[i] = epi->lneps[i];
      ep.lny[i] = epi->lny[i];
      ep.lnmean[i] = epi->lnmean[i];
      ep.lnrstd[i] = epi->lnrstd[i];
    }
  }
  const bool vec = (K % 4 == 0) && K >= 4 && ((reinterpret_cast<uintptr_t>(A) & 15) == 0);
  const int nt = vec && !use_f32_gemm() ? pick_nt(N, K, ep.mode) : 0;
  // K = 576 with N a multiple of 144: every column in one block on the byte image (the A
  // split once per 144 columns instead of once per 48)
  if (nt > 0 && (K + 31) / 32 == 18 && N % 144 == 0 && alpha_raw < 2 &&
      (ep.mode == kEpiNone || ep.mode == kEpiResidual)) {
    launch_bf16x3<9>(A, M, K, codes, N, alpha, alpha_raw, bias, C, codes1, pass_bits, P, ep, s, true);
    return;
  }
#define OB_NT(V)                                                                            \
  case V:                                                                                   \
    launch_bf16x3<V>(A, M, K, codes, N, alpha, alpha_raw, bias, C, codes1, pass_bits, P, ep, s); \
    return;
  switch (nt) {
    OB_NT(12)
    OB_NT(9)
    OB_NT(6)
    OB_NT(4)
    OB_NT(3)
    OB_NT(2)
    OB_NT(1)
    default: break;
  }
#undef OB_NT
  // fp32 path (K == 0 included: its k-loop is empty and never reads A).
  const dim3 grid((unsigned)ceil_div(M, kRows), (unsigned)ceil_div(N, 16 * kF32NT), (unsigned)P);
  hipLaunchKernelGGL(tgemm_f32_kernel, grid, dim3(kThreads), 0, s, A, M, K, codes,
                     ceil_div(K, 16), N, alpha, alpha_raw, bias, C, codes1, pass_bits, ep);
}

bool launch_ternary_gemm_passes_group(const float* A, int P, int64_t M, int64_t K, int G,
                                      const uint32_t* const* codes,
                                      const uint32_t* const* codes1, const int* pass_bits,
                                      int64_t N, const float* const* alpha, int alpha_raw,
                                      const float* const* bias, float* const* C, hipStream_t s) {
  if (G < 1 || G > 3) return false;
  const bool vec = (K % 4 == 0) && K >= 4 && ((reinterpret_cast<uintptr_t>(A) & 15) == 0);
  const int nt = vec && !use_f32_gemm() ? pick_nt(N, K, kEpiNone) : 0;
  if (M == 0 || N == 0 || P == 0) return true;
  bool al = (N % 4 == 0);
  for (int i = 0; i < G; ++i) al = al && aligned16(C[i]);
  if (nt == 0 || N % (16 * nt) != 0 || !al) {  // one launch per layer
    for (int i = 0; i < G; ++i)
      launch_ternary_gemm_passes(A, P, M, K, codes[i], codes1[i], pass_bits, N, alpha[i],
                                 alpha_raw, bias[i], C[i], s);
    return true;
  }
  EpiArgs ep{};
  ep.glayers = G;
  ep.mode = kEpiNone;
  for (int i = 0; i < G; ++i) {
    ep.gcodes[i] = codes[i];
    ep.gcodes1[i] = codes1[i];
    ep.galpha[i] = alpha[i];
    ep.gbias[i] = bias[i];
    ep.gC[i] = C[i];
  }
#define OB_NTG(V)                                                                                \
  case V:                                                                                        \
    launch_bf16x3<V>(A, M, K, codes[0], N, alpha[0], alpha_raw, bias[0], C[0], codes1[0],       \
                     pass_bits, P, ep, s);                                                       \
    return true;
  switch (nt) {
    OB_NTG(12)
    OB_NTG(9)
    OB_NTG(6)
    OB_NTG(4)
    OB_NTG(3)
    OB_NTG(2)
    OB_NTG(1)
    default: return false;
  }
#undef OB_NTG
}

bool ternary_residual_ln_supported(int64_t K, int64_t N, int alpha_raw) {
  return (K + 31) / 32 == 18 && K % 4 == 0 && N == 144 && alpha_raw < 2 && !use_f32_gemm() &&
         pick_nt(N, K, kEpiResidual) > 0;  // exactly the byte-image branch's conditions
}

bool launch_ternary_dx_sum(int G, const float* const* dY, int P, int64_t M, int64_t N,
                           const uint32_t* const* codes_t, const uint32_t* const* codes_t1,
                           const int* pass_bits, const float* const* alpha, int alpha_raw,
                           int64_t K, float* dX, hipStream_t s) {
  // the Conformer shape: three 144-wide sources (q / k / v), outputs a multiple of 144
  if (G != 3 || N != 144 || K <= 0 || K % 144 != 0 || alpha_raw >= 2 || use_f32_gemm())
    return false;
  for (int i = 0; i < G; ++i)
    if (!aligned16(dY[i])) return false;
  if (!aligned16(dX)) return false;
  if (M == 0 || P == 0) return true;
  EpiArgs ep{};
  ep.glayers = 1;
  ep.mode = kEpiNone;
  for (int i = 0; i < G; ++i) {
    ep.gA[i] = dY[i];
    ep.gcodes[i] = codes_t[i];
    ep.gcodes1[i] = codes_t1[i];
    ep.galpha[i] = alpha[i];
  }
  constexpr int kNch = 15;  // 3 sources x 5 chunks (144 zero-padded to 160)
  const int n_ct = (int)(K / 144);
  const int n16 = (int)ceil_div(M, 16);
  int rgroups = kTargetBlocksLongK / (n_ct * P);
  if (rgroups > ceil_div(n16, kByteWaves)) rgroups = (int)ceil_div(n16, kByteWaves);
  if (rgroups < 1) rgroups = 1;
  const dim3 grid((unsigned)(rgroups * n_ct), (unsigned)P);
  const size_t lds = epi_stage_off(9, 32 * kNch, true) + epi_stage_bytes(9, kByteWaves);
  hipLaunchKernelGGL((tgemm_bf16x3_kernel<9, kNch, kEpiNone, true, true, 3, kByteWaves>), grid,
                     dim3(64 * kByteWaves), lds, s, dY[0], M, (int)N, codes_t[0],
                     (int)ceil_div(N, 16), (int)K, n_ct, n16, rgroups, alpha[0], alpha_raw,
                     nullptr, dX, codes_t1[0], pass_bits, ep);
  return true;
}

void launch_ternary_gemm(const float* A, int64_t M, int64_t K, const uint32_t* codes, int64_t N,
                         const float* alpha, int alpha_raw, const float* bias, float* C,
                         hipStream_t s) {
  launch_ternary_gemm_passes(A, 1, M, K, codes, codes, nullptr, N, alpha, alpha_raw, bias, C, s);
}

#ifdef OB_TGEMM_STAMPS
extern "C" int ob_tgemm_stamps(void* host_stamps, void* host_rt) {  // diagnostic build only
  if (hipMemcpyFromSymbol(host_stamps, HIP_SYMBOL(g_tg_stamps), sizeof(g_tg_stamps)) != hipSuccess) return -6;
  return hipMemcpyFromSymbol(host_rt, HIP_SYMBOL(g_tg_rt), sizeof(g_tg_rt)) == hipSuccess ? 0 : -6;
}
#endif

}  // namespace ob
