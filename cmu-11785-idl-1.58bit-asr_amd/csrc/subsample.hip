// subsample.hip — Conv2dSubsampling on gfx950 (reference onebit_asr/conformer.py:170-208):
//   Y1 = relu(conv2d(X[:, None], W0, b0, stride 2))          1 -> C channels, 3x3
//   Y2 = relu(conv2d(Y1, W2, b2, stride 2))                   C -> C channels, 3x3
// (the Linear over the flattened (C, F2) per frame stays a library GEMM on the host side,
// its weight columns permuted to this file's channel-last order).
//
// Layouts (channels last, no NCHW <-> NHWC transposes anywhere):
//   X  [B][T][F]          (feats; conv0 has one input channel)
//   Y1 [B][T1][F1][C]     T1 = (T-3)/2+1, F1 = (F-3)/2+1
//   Y2 [B][T2][F2][C]     T2 = (T1-3)/2+1, F2 = (F1-3)/2+1
//
// conv2 (C x 9C MACs per output: 28% of the encoder FLOPs at Conformer-S) runs as
// implicit GEMMs on the bf16 matrix cores with exact-fp32 products: both operands are
// split x = hi + mid + lo (bf16, round to nearest, exact) and the six products of weight
// >= 2^-16 are accumulated in fp32 (dropped terms < 2^-24 relative), as the dW GEMM
// (dw.hip) does:
//   fwd    Y2 = relu(im2col(Y1) . W2^T + b2)       M = B T2 F2, K = 9C, N = C
//   dgrad  dY1 = col2im(G . W2), G = dY2 * (Y2 > 0), by output parity class (t1 % 2, f1 % 2):
//          each class is a dense GEMM over its 1, 2 or 4 taps (no zero-stuffing); its
//          epilogue applies relu'(Y1) and folds conv0's weight gradient (9 taps + bias per
//          channel) into per-block partials, so dY1 is never written to memory;
//   wgrad  dW2 = G^T . im2col(Y1) as split-M partials (one 48x48 wave tile per tap and
//          channel block) summed in a fixed order by a finish kernel.
// conv0 (9 MACs per output) is a plain VALU kernel. Weights are re-split into bf16 planes
// once per call (ss_pack): the B images the GEMMs stage into LDS as they are.
//
// Every reduction has a fixed order (deterministic); no atomics.
#include "ob_launch.h"

namespace ob {

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int kThr = 256;
constexpr int kSlot = 224;  // LDS / image bytes per (row or column): 3 planes x 32 bf16 + pad
constexpr int kBM = 64;     // GEMM rows per row fragment of the 4 waves

__device__ __forceinline__ f32x4 mfma_bf16(const bf16x8& a, const bf16x8& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// Round two fp32 to bf16 (v_cvt_pk_bf16_f32), packed (a low, b high); also returns the
// rounded values as fp32.
__device__ __forceinline__ uint32_t cvt2(float a, float b, float& ra, float& rb) {
  const bf16x2 v = __builtin_convertvector(f32x2{a, b}, bf16x2);
  const uint32_t u = __builtin_bit_cast(uint32_t, v);
  ra = __uint_as_float(u << 16);
  rb = __uint_as_float(u & 0xFFFF0000u);
  return u;
}

// x = hi + mid + lo of two values, packed per plane
__device__ __forceinline__ void split2(float x0, float x1, uint32_t& ph, uint32_t& pm,
                                       uint32_t& pl) {
  float h0, h1, m0, m1, l0, l1;
  ph = cvt2(x0, x1, h0, h1);
  const float r0 = x0 - h0, r1 = x1 - h1;
  pm = cvt2(r0, r1, m0, m1);
  pl = cvt2(r0 - m0, r1 - m1, l0, l1);
}

// Bijective XCD-aware remap: consecutive logical ids land on one XCD under round-robin
// dispatch (hardware block b runs on XCD b % 8).
__device__ __forceinline__ int xcd_logical(int b, int nb) {
  const int q = nb / 8, r = nb % 8, x = b % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const float* base, int64_t bytes) {
  const uint32_t nrec = bytes > 0xFFFFFFF0ll ? 0xFFFFFFF0u : (uint32_t)bytes;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, (int)nrec,
                                           0x00020000);
}

constexpr int kProdA[6] = {1, 2, 0, 1, 0, 0};  // plane of A per product: mm lh hl mh hm hh
constexpr int kProdB[6] = {1, 0, 2, 0, 1, 0};

struct SsDims {
  int B, T, F, C, T1, F1, T2, F2;
};

// Taps of dgrad parity class cl = 2 * (t1 % 2) + (f1 % 2): i in {0, 2} for even t1, {1}
// for odd (and j likewise); tap list = i-major.
__device__ __host__ __forceinline__ int class_taps(int cl) {
  return ((cl >> 1) ? 1 : 2) * ((cl & 1) ? 1 : 2);
}
__device__ __forceinline__ void class_tap(int cl, int tidx, int& i, int& j) {
  const int nj = (cl & 1) ? 1 : 2;
  const int ii = tidx / nj, jj = tidx - ii * nj;
  i = (cl >> 1) ? 1 : 2 * ii;
  j = (cl & 1) ? 1 : 2 * jj;
}

// ------------------------------------------------------------------------------------
// conv0 forward: block = (kThr / (C/4)) positions x (C/4) channel quads; a thread keeps its
// quad's 36 weights and 4 biases in registers and walks positions grid-stride; per output,
// 9 taps in (i, j) order, then the bias, then the ReLU.
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(kThr) void ss_conv0_fwd_kernel(const float* __restrict__ X,
                                                            const float* __restrict__ W0,
                                                            const float* __restrict__ b0,
                                                            SsDims d, float* __restrict__ Y1) {
  const int cq = d.C / 4;
  const int ppb = kThr / cq;  // positions per block step
  if ((int)threadIdx.x >= ppb * cq) return;
  const int q = threadIdx.x % cq;
  const int pofs = threadIdx.x / cq;
  float w[4][9], bias[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
#pragma unroll
    for (int t = 0; t < 9; ++t) w[e][t] = W0[(4 * q + e) * 9 + t];
    bias[e] = b0[4 * q + e];
  }
  const int64_t total = (int64_t)d.B * d.T1 * d.F1;
  for (int64_t p = (int64_t)blockIdx.x * ppb + pofs; p < total; p += (int64_t)gridDim.x * ppb) {
    const uint32_t pp = (uint32_t)p;  // < 2^31 (C ABI)
    const uint32_t bt = pp / (uint32_t)d.F1, f1 = pp - bt * (uint32_t)d.F1;
    const uint32_t b = bt / (uint32_t)d.T1, t1 = bt - b * (uint32_t)d.T1;
    const float* xb = X + ((int64_t)b * d.T + 2 * t1) * d.F + 2 * f1;
    float x[9];
#pragma unroll
    for (int ii = 0; ii < 3; ++ii)
#pragma unroll
      for (int jj = 0; jj < 3; ++jj) x[3 * ii + jj] = xb[ii * d.F + jj];
    f32x4 y;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float acc = 0.0f;
#pragma unroll
      for (int t = 0; t < 9; ++t) acc = fmaf(w[e][t], x[t], acc);
      acc += bias[e];
      y[e] = acc > 0.0f ? acc : 0.0f;
    }
    *reinterpret_cast<f32x4*>(Y1 + p * d.C + 4 * q) = y;
  }
}

// ------------------------------------------------------------------------------------
// Weight images: for each 32-deep k step and output column n, one 224-B slot holding the
// hi / mid / lo bf16 planes of B[k][n] for the step's 32 k (the LDS layout of ss_gemm6).
//   fwd:   n = co, k = tap * C + ci,              B = W2[co][ci][tap]
//   dgrad: class cl, n = ci, k = tidx * C + co,   B = W2[co][ci][tap(cl, tidx)]
// Image order: fwd, then the four dgrad classes. Thread = (image, step, n, 2 k).
// ------------------------------------------------------------------------------------
__device__ __host__ __forceinline__ int ksteps_of(int K) { return (K + 31) / 32; }

__global__ __launch_bounds__(kThr) void ss_pack_kernel(const float* __restrict__ W2, int C,
                                                       unsigned char* __restrict__ img) {
  // image sizes in (step, n, pair) units
  int64_t base[6];
  base[0] = 0;
  for (int im = 0; im < 5; ++im) {
    const int K = im == 0 ? 9 * C : class_taps(im - 1) * C;
    base[im + 1] = base[im] + (int64_t)ksteps_of(K) * C * 16;
  }
  for (int64_t u = (int64_t)blockIdx.x * kThr + threadIdx.x; u < base[5];
       u += (int64_t)gridDim.x * kThr) {
    int im = 0;
    while (u >= base[im + 1]) ++im;
    const int64_t v = u - base[im];
    const int pr = (int)(v % 16);
    const int64_t sn = v / 16;
    const int n = (int)(sn % C);
    const int st = (int)(sn / C);
    const int K = im == 0 ? 9 * C : class_taps(im - 1) * C;
    float val[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int k = 32 * st + 2 * pr + e;
      float w = 0.0f;
      if (k < K) {
        const int tt = k / C, cc = k - tt * C;
        if (im == 0) {
          w = W2[((int64_t)n * C + cc) * 9 + tt];  // co = n, ci = cc, tap = tt
        } else {
          int i, j;
          class_tap(im - 1, tt, i, j);
          w = W2[((int64_t)cc * C + n) * 9 + 3 * i + j];  // co = cc, ci = n
        }
      }
      val[e] = w;
    }
    uint32_t ph, pm, pl;
    split2(val[0], val[1], ph, pm, pl);
    unsigned char* slot = img + (base[im] / 16 * kSlot) + ((int64_t)st * C + n) * kSlot;
    // base[im] / 16 = slots before this image
    *reinterpret_cast<uint32_t*>(slot + 4 * pr) = ph;
    *reinterpret_cast<uint32_t*>(slot + 64 + 4 * pr) = pm;
    *reinterpret_cast<uint32_t*>(slot + 128 + 4 * pr) = pl;
  }
}

int64_t image_slots(int C, int im) {
  const int K = im == 0 ? 9 * C : class_taps(im - 1) * C;
  return (int64_t)ksteps_of(K) * C;
}

// ------------------------------------------------------------------------------------
// ss_gemm6<NT, MR, DGRAD>: C_tile[64 MR][16 NT] = A[rows][K] . B[K][16 NT] with A gathered
// from Y1 (fwd) or G (dgrad class) and split into bf16 planes in registers (each wave's rows
// are its own: no LDS round trip for A); B = a weight image, staged in LDS double-buffered
// (one barrier per k step). Block = 4 waves (16 MR rows each, all 16 NT columns); a block
// takes a contiguous range of its class's row tiles (blockIdx.y = class; fwd: one class),
// consecutive ranges on one XCD (the taps of neighbouring tiles overlap in Y1 / G). The next
// k step's A (2 MR dwordx4 per lane) and B (image slots) are loaded into registers while the
// current step's MFMAs run. The image is re-read per tile (L2-resident, 64 MR rows share it).
// Same products in the same order as the LDS-A form (round 4): the same bits.
// ------------------------------------------------------------------------------------
struct GemmArgs {
  const float* src;             // fwd: Y1; dgrad: G
  const unsigned char* img;     // weight image base (fwd or the 4 dgrad classes)
  int64_t img_off[4];           // slot offsets of the images of the grid's classes
  int64_t rows[4];              // GEMM rows per class
  int blk_off[4];               // dgrad: first partial block of each class
  int nblk[4];                  // blocks per class (blockIdx.x >= nblk[cl] exits)
  const float* bias;            // fwd: b2
  float* out;                   // fwd: Y2
  const float* W0;              // dgrad: conv0 weight [C][9] and bias (relu'(Y1) recompute)
  const float* b0;
  const float* X;               // dgrad: conv0 input (for conv0's weight gradient)
  float* part0;                 // dgrad: [blocks][C * 10] conv0 weight / bias partials
  SsDims d;
};

template <int NT, int MR, bool DGRAD>
struct GemmCfg {
  static constexpr int BN = 16 * NT;
  // waves per block (8-wave forward blocks, one per CU, a B step serving 256 rows: 417 ->
  // 494 us a call -- the B image's L2 reads are not what limits it)
  static constexpr int WV = 4;
  static constexpr int kT = 64 * WV;
  static constexpr int BM = 16 * WV * MR;
  static constexpr int kBSlotsPT = (BN * kSlot / 16 + kT - 1) / kT;  // B dwordx4 / thread
  static constexpr size_t kLdsMain = (size_t)2 * BN * kSlot;  // B image steps, double-buffered
  static constexpr size_t kLdsEpi = DGRAD ? (size_t)(BM * 16 + 4 * BN * 16) * 4 : 0;
  static constexpr size_t kW0Off = kLdsMain > kLdsEpi ? kLdsMain : kLdsEpi;  // dgrad: W0|b0
  static constexpr size_t kLds = kW0Off + (DGRAD ? (size_t)BN * 12 * 4 : 0);
};

template <int NT, int MR, bool DGRAD>
__global__ __launch_bounds__((GemmCfg<NT, MR, DGRAD>::kT), 2) void ss_gemm6_kernel(
    GemmArgs ga) {
  using Cf = GemmCfg<NT, MR, DGRAD>;
  constexpr int BN = Cf::BN, BM = Cf::BM, kBSlotsPT = Cf::kBSlotsPT, WV = Cf::WV, kT = Cf::kT;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];  // B: 2 x BN columns x 224 B
  const SsDims& d = ga.d;
  const int C = d.C;
  const int cl = DGRAD ? (int)blockIdx.y : 0;
  const int K = DGRAD ? class_taps(cl) * C : 9 * C;
  const int ks = ksteps_of(K);
  const int64_t rows = ga.rows[cl];
  const int64_t tiles = (rows + BM - 1) / BM;
  const unsigned char* img = ga.img + ga.img_off[cl] * kSlot;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int pt = cl >> 1, pf = cl & 1;
  const int T1c = DGRAD ? (pt ? d.T1 / 2 : (d.T1 + 1) / 2) : 1;
  const int F1c = DGRAD ? (pf ? d.F1 / 2 : (d.F1 + 1) / 2) : 1;
  const int nblk = DGRAD ? ga.nblk[cl] : (int)gridDim.x;
  if ((int)blockIdx.x >= nblk) return;
  const int L = DGRAD ? (int)blockIdx.x : xcd_logical((int)blockIdx.x, nblk);
  const int64_t t_begin = tiles * L / nblk, t_end = tiles * (L + 1) / nblk;

  // row geometry: fwd m = (b, t2, f2); dgrad m = (b, t1 / 2, f1 / 2) of the class
  // (rows < 2^31, checked by the C ABI: 32-bit division)
  auto geom = [&](int64_t m, int& b, int& p1, int& p2) {
    const uint32_t mm = (uint32_t)m;
    if (DGRAD) {
      const uint32_t per = (uint32_t)T1c * F1c;
      const uint32_t bb = mm / per, rem = mm - bb * per, q = rem / (uint32_t)F1c;
      b = (int)bb;
      p1 = 2 * (int)q + pt;
      p2 = 2 * (int)(rem - q * (uint32_t)F1c) + pf;
    } else {
      const uint32_t per = (uint32_t)d.T2 * d.F2;
      const uint32_t bb = mm / per, rem = mm - bb * per, q = rem / (uint32_t)d.F2;
      b = (int)bb;
      p1 = (int)q;
      p2 = (int)(rem - q * (uint32_t)d.F2);
    }
  };

  if (DGRAD) {  // conv0's weights and bias, [C][12], for the relu'(Y1) recompute
    float* w0s = reinterpret_cast<float*>(lds + Cf::kW0Off);
    for (int e = threadIdx.x; e < BN * 12; e += kT) {
      const int c = e / 12, tp = e - 12 * (e / 12);
      w0s[e] = tp < 9 ? ga.W0[c * 9 + tp] : (tp == 9 ? ga.b0[c] : 0.0f);
    }
  }  // (read after the first tile's barriers)
  // conv0 weight-gradient running sums (dgrad): o = threadIdx.x + 256 j = c * 16 + tap
  constexpr int kW0J = DGRAD ? (BN * 16 + kT - 1) / kT : 1;
  float w0acc[kW0J];
#pragma unroll
  for (int j = 0; j < kW0J; ++j) w0acc[j] = 0.0f;

  for (int64_t tile = t_begin; tile < t_end; ++tile) {
    const int64_t m0 = tile * BM;
    // A never touches LDS: each wave loads, splits and feeds its own rows from registers --
    // lane (r, g) holds row 16 (wave + WV u) + r of the tile, k = 8g .. 8g + 7 of the step,
    // exactly the MFMA A fragment (A rows are not shared between waves).
    int ab[MR], ap1[MR], ap2[MR];
    bool aok[MR];
#pragma unroll
    for (int u = 0; u < MR; ++u) {
      const int64_t am = m0 + 16 * (wave + WV * u) + r;
      aok[u] = am < rows;
      geom(aok[u] ? am : rows - 1, ab[u], ap1[u], ap2[u]);
    }
    // Loads are unconditional from clamped addresses, and rows / taps outside the image are
    // zeroed before the split (a guarded load makes hipcc branch and wait vmcnt(0) at it,
    // which serializes the prefetch with the MFMAs).
    auto load_a = [&](int st, f32x4 (&ax)[MR][2], uint32_t& aval) {
      const int k = 32 * st + 8 * g;  // 8 consecutive k within one tap (C % 8 == 0)
      const bool kok = k < K;
      const int kc = kok ? k : 0;
      const int tt = kc / C, cc = kc - tt * C;
      int i = 0, j = 0;
      if (DGRAD) {
        class_tap(cl, tt, i, j);
      } else {
        i = tt / 3;
        j = tt - 3 * (tt / 3);
      }
      aval = 0;
#pragma unroll
      for (int u = 0; u < MR; ++u) {
        const float* src;
        bool ok;
        if (DGRAD) {
          const int t2 = (ap1[u] - i) >> 1, f2 = (ap2[u] - j) >> 1;  // parity exact
          ok = ap1[u] >= i && ap2[u] >= j && t2 < d.T2 && f2 < d.F2;
          src = ga.src + (((int64_t)ab[u] * d.T2 + (ok ? t2 : 0)) * d.F2 + (ok ? f2 : 0)) * C + cc;
        } else {
          ok = true;
          src = ga.src +
                (((int64_t)ab[u] * d.T1 + 2 * ap1[u] + i) * d.F1 + 2 * ap2[u] + j) * C + cc;
        }
        ok = ok && aok[u] && kok;
        aval |= (ok ? 1u : 0u) << u;
        ax[u][0] = *reinterpret_cast<const f32x4*>(src);
        ax[u][1] = *reinterpret_cast<const f32x4*>(src + 4);
      }
    };
    auto load_b = [&](int st, f32x4 (&bv)[kBSlotsPT]) {
      const f32x4* s4 = reinterpret_cast<const f32x4*>(img + (int64_t)st * BN * kSlot);
#pragma unroll
      for (int j = 0; j < kBSlotsPT; ++j) {
        const int e = threadIdx.x + j * kT;
        const int ec = e < BN * kSlot / 16 ? e : BN * kSlot / 16 - 1;  // clamped, unguarded
        bv[j] = s4[ec];
      }
    };
    auto store_b = [&](int buf, const f32x4 (&bv)[kBSlotsPT]) {
      f32x4* d4 = reinterpret_cast<f32x4*>(lds + (size_t)buf * BN * kSlot);
#pragma unroll
      for (int j = 0; j < kBSlotsPT; ++j) {
        const int e = threadIdx.x + j * kT;
        if (e < BN * kSlot / 16) d4[e] = bv[j];
      }
    };
    f32x4 ax[MR][2], bv[kBSlotsPT];
    uint32_t aval;
    load_a(0, ax, aval);
    load_b(0, bv);
    f32x4 acc[MR][NT];
#pragma unroll
    for (int u = 0; u < MR; ++u)
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[u][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    __syncthreads();  // (dgrad: the previous tile's epilogue is done with the LDS)
    store_b(0, bv);
    __syncthreads();
    // One barrier a step: step st reads B buffer st & 1 (stored during step st - 1) while
    // step st + 1's B goes into the other buffer, whose last readers (step st - 1) all
    // passed the previous barrier.
    for (int st = 0; st < ks; ++st) {
      bf16x8 a[MR][3];
#pragma unroll
      for (int u = 0; u < MR; ++u) {
        const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
        const bool ok = (aval >> u) & 1u;
        const f32x4 x0 = ok ? ax[u][0] : z4, x1 = ok ? ax[u][1] : z4;
        uint32_t ph[4], pm[4], pl[4];
        split2(x0[0], x0[1], ph[0], pm[0], pl[0]);
        split2(x0[2], x0[3], ph[1], pm[1], pl[1]);
        split2(x1[0], x1[1], ph[2], pm[2], pl[2]);
        split2(x1[2], x1[3], ph[3], pm[3], pl[3]);
        a[u][0] = __builtin_bit_cast(bf16x8, uint4{ph[0], ph[1], ph[2], ph[3]});
        a[u][1] = __builtin_bit_cast(bf16x8, uint4{pm[0], pm[1], pm[2], pm[3]});
        a[u][2] = __builtin_bit_cast(bf16x8, uint4{pl[0], pl[1], pl[2], pl[3]});
      }
      if (st + 1 < ks) {
        load_a(st + 1, ax, aval);
        load_b(st + 1, bv);
      }
      const unsigned char* lb = lds + (size_t)(st & 1) * BN * kSlot;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const unsigned char* sb = lb + (16 * t + r) * kSlot + 16 * g;
        bf16x8 bq[3];
#pragma unroll
        for (int q = 0; q < 3; ++q) bq[q] = *reinterpret_cast<const bf16x8*>(sb + 64 * q);
#pragma unroll
        for (int p = 0; p < 6; ++p)
#pragma unroll
          for (int u = 0; u < MR; ++u) {
            acc[u][t] = mfma_bf16(a[u][kProdA[p]], bq[kProdB[p]], acc[u][t]);
          }
      }
      if (st + 1 < ks) store_b((st + 1) & 1, bv);
      __syncthreads();
    }

    // D[row = 4g + reg][col = r] of (row frag u, column tile t): tile row 16 (wave + WV u) +
    // 4g + reg, column 16t + r
    if (!DGRAD) {
      // branch-free stores: rows past the end get an offset outside the descriptor (dropped)
      const __amdgpu_buffer_rsrc_t ro = make_rsrc(ga.out, rows * C * 4);
      float bb[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) bb[t] = ga.bias[16 * t + r];
#pragma unroll
      for (int u = 0; u < MR; ++u)
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
          const int64_t m = m0 + 16 * (wave + WV * u) + 4 * g + reg;
          const uint32_t ob = m < rows ? (uint32_t)(m * C + r) * 4 : 0xFFFFFFF0u;
#pragma unroll
          for (int t = 0; t < NT; ++t) {
            const float y = acc[u][t][reg] + bb[t];
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(y > 0.0f ? y : 0.0f), ro, ob,
                                                  64 * t, 0);
          }
        }
    } else {
      // conv0's weight gradient from this tile, on the matrix cores (fp32 MFMA, exact
      // products): dW0[c][tap] += sum over rows of dY1m[row][c] * Xw[row][tap], with
      // dY1m = relu'(Y1) * dY1 straight from the accumulators (A[i = c][k = row] of
      // v_mfma_f32_16x16x4f32 is acc[u][t][reg] of lane (r = c, g = row group)) and Xw the
      // rows' conv0 windows of X (tap 9 = 1 for the bias) staged in LDS [BM][16]. The 4
      // waves' 16x16 tiles are summed in wave order into thread-owned running sums.
      __syncthreads();  // all waves are done with la / lb
      float* xw = reinterpret_cast<float*>(lds);  // [BM][16]
      float* wred = xw + BM * 16;                 // [4 waves][BN][16]
      const float* w0s = reinterpret_cast<const float*>(lds + Cf::kW0Off);  // [BN][12]
      for (int e = threadIdx.x; e < BM * 16; e += kT) {
        const int lr = e >> 4, tp = e & 15;
        const int64_t m = m0 + lr;
        int bb, t1, f1;
        geom(m < rows ? m : rows - 1, bb, t1, f1);
        const int tq = tp < 9 ? tp : 0;
        const float xv = ga.X[((int64_t)bb * d.T + 2 * t1 + tq / 3) * d.F + 2 * f1 + tq % 3];
        xw[e] = tp < 9 ? xv : (tp == 9 ? 1.0f : 0.0f);
      }
      __syncthreads();
      // relu'(Y1) recomputed from the windows with conv0_fwd's exact fma chain (taps in
      // order, then the bias): the same bits as Y1 > 0, without 8 NT scattered Y1 loads
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const float* w = w0s + (16 * t + r) * 12;
        const f32x4 wa = *reinterpret_cast<const f32x4*>(w);  // [C][12] rows, 16-B aligned
        const f32x4 wb = *reinterpret_cast<const f32x4*>(w + 4);
        const float w8 = w[8], w9 = w[9];
#pragma unroll
        for (int u = 0; u < MR; ++u)
#pragma unroll
          for (int reg = 0; reg < 4; ++reg) {
            const int lr = 16 * (wave + WV * u) + 4 * g + reg;
            const bool ok = m0 + lr < rows;
            const f32x4 x0 = *reinterpret_cast<const f32x4*>(xw + lr * 16);
            const f32x4 x1 = *reinterpret_cast<const f32x4*>(xw + lr * 16 + 4);
            const float x8 = xw[lr * 16 + 8];
            float pre = 0.0f;
            pre = fmaf(wa[0], x0[0], pre);
            pre = fmaf(wa[1], x0[1], pre);
            pre = fmaf(wa[2], x0[2], pre);
            pre = fmaf(wa[3], x0[3], pre);
            pre = fmaf(wb[0], x1[0], pre);
            pre = fmaf(wb[1], x1[1], pre);
            pre = fmaf(wb[2], x1[2], pre);
            pre = fmaf(wb[3], x1[3], pre);
            pre = fmaf(w8, x8, pre);
            pre += w9;
            acc[u][t][reg] = (ok & (pre > 0.0f)) ? acc[u][t][reg] : 0.0f;
          }
      }
      f32x4 dw[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) dw[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < MR; ++u)
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
          const float xb = xw[(16 * (wave + WV * u) + 4 * g + reg) * 16 + r];
#pragma unroll
          for (int t = 0; t < NT; ++t)
            dw[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(acc[u][t][reg], xb, dw[t], 0, 0, 0);
        }
      // dw[t][reg] = D[c = 16t + 4g + reg][tap = r]
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int reg = 0; reg < 4; ++reg)
          wred[(wave * BN + 16 * t + 4 * g + reg) * 16 + r] = dw[t][reg];
      __syncthreads();
#pragma unroll
      for (int j = 0; j < kW0J; ++j) {
        const int o = threadIdx.x + j * kT;
        if (o < BN * 16)
          w0acc[j] += ((wred[o] + wred[BN * 16 + o]) + wred[2 * BN * 16 + o]) +
                      wred[3 * BN * 16 + o];
      }
    }
  }
  if (DGRAD) {
    float* dst = ga.part0 + (int64_t)(ga.blk_off[cl] + L) * (BN * 10);
#pragma unroll
    for (int j = 0; j < kW0J; ++j) {
      const int o = threadIdx.x + j * kT, c = o >> 4, tp = o & 15;
      if (o < BN * 16 && tp < 10) dst[c * 10 + tp] = w0acc[j];
    }
  }
}

// ------------------------------------------------------------------------------------
// conv2 weight gradient: part[c][co][tap * C + ci] = sum over the chunk's rows m of
// G[m][co] * Y1[b][2t2+i][2f2+j][ci]  (m = (b, t2, f2), tap = 3i + j), and part_db[c][co] =
// sum over the chunk of G[m][co]. Block = WN x WK waves of 16TW x 16TW tiles (block tile
// BN x BK, tap = the k-tile's tap); per 32-row step the block splits G[32][BN] and the
// gathered Y1 rows [32][BK] once into LDS planes (double-buffered), as dw_lds_kernel. The
// tap blocks of one chunk are consecutive logical blocks on one XCD (they share G rows).
// ------------------------------------------------------------------------------------
template <int TW, int WN, int WK>
struct WgCfg {
  static constexpr int BN = 16 * TW * WN, BK = 16 * TW * WK;
  static constexpr int kThrB = 64 * WN * WK;
  static constexpr int kCols = BN + BK;
  static constexpr int kBuf = kCols * kSlot;
  static constexpr int kUY = (BN * 4 + kThrB - 1) / kThrB;
  static constexpr int kUX = (BK * 4 + kThrB - 1) / kThrB;
};

template <int TW, int WN, int WK>
__global__ __launch_bounds__(64 * WN * WK) void ss_wgrad_kernel(
    const float* __restrict__ G, const float* __restrict__ Y1, SsDims d, int tiles_n,
    int tiles_k_per_tap, int64_t rows_per_chunk, float* __restrict__ part,
    float* __restrict__ part_db) {
  using Cf = WgCfg<TW, WN, WK>;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int C = d.C;
  const int64_t M = (int64_t)d.B * d.T2 * d.F2;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wn = wave / WK, wk = wave - wn * WK;
  const int r = lane & 15, g = lane >> 4;
  const int tiles = tiles_n * 9 * tiles_k_per_tap;
  const int L = xcd_logical((int)blockIdx.x, (int)gridDim.x);
  const int tile = L % tiles;
  const int64_t chunk = L / tiles;
  const int tn = tile / (9 * tiles_k_per_tap);
  const int tkk = tile - tn * 9 * tiles_k_per_tap;
  const int tap = tkk / tiles_k_per_tap;
  const int tk = tkk - tap * tiles_k_per_tap;
  const int n0 = tn * Cf::BN, c0 = tk * Cf::BK;  // co range, ci range (within the tap)
  const int ti = tap / 3, tj = tap - 3 * (tap / 3);
  const int64_t m_begin = chunk * rows_per_chunk;
  const int64_t m_end = m_begin + rows_per_chunk < M ? m_begin + rows_per_chunk : M;
  const int steps = (int)((m_end - m_begin + 31) / 32);
  const bool do_db = (part_db != nullptr) && tap == 0 && tk == 0;
  constexpr int UY = Cf::kUY, UX = Cf::kUX;

  // loader units: 2 rows x 4 columns (row pair fastest); rows past the chunk read 0
  int y_c[UY], y_rp[UY], x_c[UX], x_rp[UX];
  bool y_ok[UY], x_ok[UX];
#pragma unroll
  for (int j = 0; j < UY; ++j) {
    const int u = threadIdx.x + j * Cf::kThrB;
    y_ok[j] = u < Cf::BN * 4;
    const int uu = y_ok[j] ? u : 0;
    y_rp[j] = uu & 15;
    y_c[j] = 4 * (uu >> 4);
  }
#pragma unroll
  for (int j = 0; j < UX; ++j) {
    const int u = threadIdx.x + j * Cf::kThrB;
    x_ok[j] = u < Cf::BK * 4;
    const int uu = x_ok[j] ? u : 0;
    x_rp[j] = uu & 15;
    x_c[j] = 4 * (uu >> 4);
  }
  struct Raw {
    f32x4 y[UY][2];
    f32x4 x[UX][2];
  };
  // G rows of the chunk and all of Y1 through buffer descriptors (32-bit offsets, loads
  // past the range read 0: Y1 < 2 GB, checked by the C ABI)
  const __amdgpu_buffer_rsrc_t rg = make_rsrc(G + m_begin * C, (m_end - m_begin) * C * 4);
  const __amdgpu_buffer_rsrc_t r1 =
      make_rsrc(Y1, (int64_t)d.B * d.T1 * d.F1 * C * 4);
  const uint32_t per = (uint32_t)d.T2 * d.F2;
  auto y1_off = [&](int64_t m) -> uint32_t {  // byte offset of Y1's row of im2col row m
    if (m >= m_end) return 0x80000000u;       // past the chunk: out of range -> 0
    const uint32_t mm = (uint32_t)m;
    const uint32_t b = mm / per, rem = mm - b * per;
    const uint32_t t2 = rem / (uint32_t)d.F2, f2 = rem - t2 * (uint32_t)d.F2;
    return ((((b * d.T1 + 2 * t2 + ti) * d.F1 + 2 * f2 + tj) * C) + c0) * 4;
  };
  auto load = [&](Raw& raw, int step) {
    const int so = step * 32 * C * 4;
#pragma unroll
    for (int j = 0; j < UY; ++j)
      if (y_ok[j])
#pragma unroll
        for (int i = 0; i < 2; ++i)
          raw.y[j][i] = __builtin_amdgcn_raw_buffer_load_b128(
              rg, ((2 * y_rp[j] + i) * C + n0 + y_c[j]) * 4, so, 0);
#pragma unroll
    for (int j = 0; j < UX; ++j)
      if (x_ok[j])
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const uint32_t off = y1_off(m_begin + 32 * step + 2 * x_rp[j] + i);
          raw.x[j][i] = __builtin_amdgcn_raw_buffer_load_b128(r1, off + x_c[j] * 4, 0, 0);
        }
  };
  f32x4 dbacc[UY];
#pragma unroll
  for (int j = 0; j < UY; ++j) dbacc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto put = [&](unsigned char* base, int col, int rp, const f32x4& r0, const f32x4& r1) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      uint32_t ph, pm, pl;
      split2(r0[e], r1[e], ph, pm, pl);
      unsigned char* cb = base + (col + e) * kSlot + rp * 4;
      *reinterpret_cast<uint32_t*>(cb) = ph;
      *reinterpret_cast<uint32_t*>(cb + 64) = pm;
      *reinterpret_cast<uint32_t*>(cb + 128) = pl;
    }
  };
  auto store = [&](const Raw& raw, int buf) {
    unsigned char* base = lds + buf * Cf::kBuf;
#pragma unroll
    for (int j = 0; j < UY; ++j) {
      if (!y_ok[j]) continue;
      if (do_db) dbacc[j] += raw.y[j][0] + raw.y[j][1];
      put(base, y_c[j], y_rp[j], raw.y[j][0], raw.y[j][1]);
    }
#pragma unroll
    for (int j = 0; j < UX; ++j)
      if (x_ok[j]) put(base, Cf::BN + x_c[j], x_rp[j], raw.x[j][0], raw.x[j][1]);
  };
  f32x4 acc[TW][TW];
#pragma unroll
  for (int t = 0; t < TW; ++t)
#pragma unroll
    for (int u = 0; u < TW; ++u) acc[t][u] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto frag = [&](const unsigned char* base, int col, int plane) {
    return *reinterpret_cast<const bf16x8*>(base + col * kSlot + 64 * plane + 16 * g);
  };
  auto compute = [&](int buf) {
    const unsigned char* base = lds + buf * Cf::kBuf;
    bf16x8 bfr[TW][3];
#pragma unroll
    for (int u = 0; u < TW; ++u)
#pragma unroll
      for (int q = 0; q < 3; ++q) bfr[u][q] = frag(base, Cf::BN + 16 * (TW * wk + u) + r, q);
#pragma unroll
    for (int t = 0; t < TW; ++t) {
      bf16x8 a[3];
#pragma unroll
      for (int q = 0; q < 3; ++q) a[q] = frag(base, 16 * (TW * wn + t) + r, q);
#pragma unroll
      for (int p = 0; p < 6; ++p)
#pragma unroll
        for (int u = 0; u < TW; ++u)
          acc[t][u] = mfma_bf16(a[kProdA[p]], bfr[u][kProdB[p]], acc[t][u]);
    }
  };
  Raw ra, rb;
  load(ra, 0);
  if (steps > 1) load(rb, 1);
  store(ra, 0);
  if (steps > 2) load(ra, 2);
  __syncthreads();
  for (int s = 0; s < steps; s += 2) {
    compute(0);
    if (s + 1 < steps) {
      store(rb, 1);
      if (s + 3 < steps) load(rb, s + 3);
    }
    __syncthreads();
    if (s + 1 >= steps) break;
    compute(1);
    if (s + 2 < steps) {
      store(ra, 0);
      if (s + 4 < steps) load(ra, s + 4);
    }
    __syncthreads();
  }
  const int K9 = 9 * C;
  float* out = part + chunk * ((int64_t)C * K9);
#pragma unroll
  for (int t = 0; t < TW; ++t)
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      const int n = n0 + 16 * (TW * wn + t) + 4 * g + reg;
#pragma unroll
      for (int u = 0; u < TW; ++u)
        out[(int64_t)n * K9 + tap * C + c0 + 16 * (TW * wk + u) + r] = acc[t][u][reg];
    }
  if (do_db) {
    float* red = reinterpret_cast<float*>(lds);  // [16][BN]
#pragma unroll
    for (int j = 0; j < UY; ++j)
      if (y_ok[j])
#pragma unroll
        for (int e = 0; e < 4; ++e) red[y_rp[j] * Cf::BN + y_c[j] + e] = dbacc[j][e];
    __syncthreads();
    for (int c = threadIdx.x; c < Cf::BN; c += Cf::kThrB) {
      float v = 0.0f;
#pragma unroll
      for (int q = 0; q < 16; ++q) v += red[q * Cf::BN + c];
      part_db[chunk * C + n0 + c] = v;
    }
  }
}

// dW2 in torch's layout [co][ci][3][3] = sum over chunks (chunk order) of the partials
// (stored [co][tap * C + ci]); db2 likewise. One output per thread, 16 chunk loads in flight.
__global__ __launch_bounds__(kThr) void ss_wgrad_finish_kernel(const float* __restrict__ part,
                                                               const float* __restrict__ part_db,
                                                               int chunks, int C,
                                                               float* __restrict__ dW2,
                                                               float* __restrict__ db2) {
  const int64_t nk = (int64_t)C * 9 * C;
  const int64_t e = (int64_t)blockIdx.x * kThr + threadIdx.x;
  if (e >= nk + C) return;
  int64_t src_e, stride;
  if (e < nk) {  // e = torch index (co * C + ci) * 9 + tap -> partial index co * 9C + tap * C + ci
    const int tap = (int)(e % 9);
    const int64_t cc = e / 9;
    const int ci = (int)(cc % C), co = (int)(cc / C);
    src_e = (int64_t)co * 9 * C + tap * C + ci;
    stride = nk;
  } else {
    src_e = e - nk;
    stride = C;
  }
  const float* src = (e < nk ? part : part_db) + src_e;
  constexpr int Gn = 16;
  float cur[Gn], nxt[Gn];
  auto fetch = [&](int c0, float (&v)[Gn]) {
#pragma unroll
    for (int u = 0; u < Gn; ++u) v[u] = c0 + u < chunks ? src[(int64_t)(c0 + u) * stride] : 0.0f;
  };
  float s = 0.0f;
  fetch(0, cur);
  for (int c0 = 0; c0 < chunks; c0 += Gn) {
    if (c0 + Gn < chunks) fetch(c0 + Gn, nxt);
#pragma unroll
    for (int u = 0; u < Gn; ++u)
      if (c0 + u < chunks) s += cur[u];
#pragma unroll
    for (int u = 0; u < Gn; ++u) cur[u] = nxt[u];
  }
  if (e < nk) dW2[e] = s;
  else db2[e - nk] = s;
}

// dW0 [C][9], db0 [C] = sum over the dgrad blocks of their partials: block = 16 outputs x
// 16 block groups (group j sums blocks j, j + 16, ... in order), then the 16 group sums in
// order (fixed order).
__global__ __launch_bounds__(kThr) void ss_w0_finish_kernel(const float* __restrict__ part0,
                                                            int blocks, int C,
                                                            float* __restrict__ dW0,
                                                            float* __restrict__ db0) {
  __shared__ float red[16][17];
  const int ol = threadIdx.x & 15, grp = threadIdx.x >> 4;
  const int o = blockIdx.x * 16 + ol;
  float s = 0.0f;
  if (o < C * 10) {
    int b = grp;
    for (; b + 48 < blocks; b += 64) {
      const float v0 = part0[(int64_t)b * C * 10 + o];
      const float v1 = part0[(int64_t)(b + 16) * C * 10 + o];
      const float v2 = part0[(int64_t)(b + 32) * C * 10 + o];
      const float v3 = part0[(int64_t)(b + 48) * C * 10 + o];
      s += v0;
      s += v1;
      s += v2;
      s += v3;
    }
    for (; b < blocks; b += 16) s += part0[(int64_t)b * C * 10 + o];
  }
  red[grp][ol] = s;
  __syncthreads();
  if (grp == 0 && o < C * 10) {
    float t = 0.0f;
#pragma unroll
    for (int j = 0; j < 16; ++j) t += red[j][ol];
    const int c = o / 10, tp = o - 10 * (o / 10);
    if (tp < 9) dW0[c * 9 + tp] = t;
    else db0[c] = t;
  }
}

// G = dY2 * (Y2 > 0)  (relu backward on the output, torch's threshold_backward)
__global__ __launch_bounds__(kThr) void ss_relu_mask_kernel(const float* __restrict__ dY2,
                                                            const float* __restrict__ Y2,
                                                            int64_t n4, float* __restrict__ G) {
  for (int64_t i = (int64_t)blockIdx.x * kThr + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * kThr) {
    const f32x4 gv = reinterpret_cast<const f32x4*>(dY2)[i];
    const f32x4 yv = reinterpret_cast<const f32x4*>(Y2)[i];
    f32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = yv[e] > 0.0f ? gv[e] : 0.0f;
    reinterpret_cast<f32x4*>(G)[i] = o;
  }
}

SsDims dims(int64_t B, int64_t T, int64_t F, int64_t C) {
  SsDims d;
  d.B = (int)B;
  d.T = (int)T;
  d.F = (int)F;
  d.C = (int)C;
  d.T1 = (int)((T - 3) / 2 + 1);
  d.F1 = (int)((F - 3) / 2 + 1);
  d.T2 = (d.T1 - 3) / 2 + 1;
  d.F2 = (d.F1 - 3) / 2 + 1;
  return d;
}

// dgrad: 2 resident blocks per CU, 512 slots; class cl gets blocks in proportion to its
// tiles x (k steps + kDgradEpi, the per-tile prologue / epilogue cost in k-step units)
constexpr int kDgradBlocks = 508;
constexpr int kDgradEpi = 4;

struct WgPlan {
  int tw, wn, wk, tiles_n, tiles_k_per_tap, chunks;
  int64_t rows_per_chunk;
};

// wgrad block shapes: C = 144 -> one 144x144 block of 9 waves (48x48 wave tiles) per tap;
// 96 -> 96x96 of 4 waves (48x48); 64 -> 64x64 of 4 waves (32x32); 48 -> 1 wave (48x48);
// other multiples of 32 -> 64x64 blocks
WgPlan wg_plan(const SsDims& d) {
  WgPlan p;
  if (d.C == 144) p.tw = 3, p.wn = 3;
  else if (d.C == 96) p.tw = 3, p.wn = 2;
  else if (d.C == 48) p.tw = 3, p.wn = 1;
  else p.tw = 2, p.wn = 2;
  p.wk = p.wn;
  p.tiles_n = d.C / (16 * p.tw * p.wn);
  p.tiles_k_per_tap = d.C / (16 * p.tw * p.wk);
  const int64_t M = (int64_t)d.B * d.T2 * d.F2;
  const int tiles = p.tiles_n * 9 * p.tiles_k_per_tap;
  int64_t want = 256 / tiles;  // one block per CU (1 resident per CU: no second round)
  if (want < 1) want = 1;
  p.rows_per_chunk = 32 * ((M + want * 32 - 1) / (want * 32));
  p.chunks = (int)((M + p.rows_per_chunk - 1) / p.rows_per_chunk);
  return p;
}

}  // namespace

// C: the GEMM column tiles are instantiated for 48, 64, 96, 144 (NT = C / 16) and the
// wgrad tiles for multiples of 48 up to 144 or of 64
bool subsample_supported(int64_t T, int64_t F, int64_t C) {
  if (T < 7 || F < 7) return false;
  return C == 48 || C == 64 || C == 96 || C == 144;
}

size_t subsample_image_bytes(int64_t C) {
  int64_t slots = 0;
  for (int im = 0; im < 5; ++im) slots += image_slots((int)C, im);
  return (size_t)slots * kSlot;
}

void launch_subsample_pack(const float* W2, int64_t C, void* img, hipStream_t s) {
  const int64_t units = (int64_t)subsample_image_bytes(C) / kSlot * 16;
  int64_t blocks = (units + kThr - 1) / kThr;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(ss_pack_kernel, dim3((unsigned)blocks), dim3(kThr), 0, s, W2, (int)C,
                     static_cast<unsigned char*>(img));
}

template <int NT, bool DG>
static void launch_gemm6(const GemmArgs& ga, dim3 grid, hipStream_t s) {
  constexpr int MR = 2;
  constexpr size_t lds = GemmCfg<NT, MR, DG>::kLds;
  hipLaunchKernelGGL((ss_gemm6_kernel<NT, MR, DG>), grid, dim3(GemmCfg<NT, MR, DG>::kT), lds, s,
                     ga);
}

template <bool DG>
static void launch_gemm6_c(int64_t C, const GemmArgs& ga, dim3 grid, hipStream_t s) {
  if (C == 144) launch_gemm6<9, DG>(ga, grid, s);
  else if (C == 96) launch_gemm6<6, DG>(ga, grid, s);
  else if (C == 64) launch_gemm6<4, DG>(ga, grid, s);
  else launch_gemm6<3, DG>(ga, grid, s);
}

void launch_subsample_fwd(const float* X, int64_t B, int64_t T, int64_t F, int64_t C,
                          const float* W0, const float* b0, const void* img, const float* b2,
                          float* Y1, float* Y2, hipStream_t s) {
  const SsDims d = dims(B, T, F, C);
  {
    const int64_t total = (int64_t)d.B * d.T1 * d.F1, ppb = kThr / (C / 4);
    int64_t blocks = (total + ppb - 1) / ppb;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(ss_conv0_fwd_kernel, dim3((unsigned)blocks), dim3(kThr), 0, s, X, W0, b0,
                       d, Y1);
  }
  GemmArgs ga{};
  ga.src = Y1;
  ga.img = static_cast<const unsigned char*>(img);
  ga.img_off[0] = 0;
  ga.rows[0] = (int64_t)d.B * d.T2 * d.F2;
  ga.bias = b2;
  ga.out = Y2;
  ga.d = d;
  const int64_t bm = GemmCfg<9, 2, false>::BM;  // (BM does not depend on NT)
  const int64_t tiles = (ga.rows[0] + bm - 1) / bm;
  const dim3 grid((unsigned)(tiles < 512 ? tiles : 512));  // 2 resident per CU
  launch_gemm6_c<false>(C, ga, grid, s);
}

size_t subsample_bwd_workspace(int64_t B, int64_t T, int64_t F, int64_t C) {
  const SsDims d = dims(B, T, F, C);
  const WgPlan p = wg_plan(d);
  const int64_t M = (int64_t)d.B * d.T2 * d.F2;
  size_t w = 0;
  w += ((size_t)M * C * 4 + 255) & ~(size_t)255;                            // G
  w += ((size_t)p.chunks * C * 9 * C * 4 + 255) & ~(size_t)255;             // dW2 partials
  w += ((size_t)p.chunks * C * 4 + 255) & ~(size_t)255;                     // db2 partials
  w += ((size_t)kDgradBlocks * C * 10 * 4 + 255) & ~(size_t)255;           // conv0 partials
  return w;
}

void launch_subsample_bwd(const float* X, const float* W0, const float* b0, const float* Y1,
                          const float* Y2, const float* dY2, int64_t B, int64_t T, int64_t F,
                          int64_t C, const void* img,
                          float* dW0, float* db0, float* dW2, float* db2, void* ws,
                          hipStream_t s) {
  const SsDims d = dims(B, T, F, C);
  const WgPlan p = wg_plan(d);
  const int64_t M = (int64_t)d.B * d.T2 * d.F2;
  char* w = static_cast<char*>(ws);
  float* G = reinterpret_cast<float*>(w);
  w += ((size_t)M * C * 4 + 255) & ~(size_t)255;
  float* part2 = reinterpret_cast<float*>(w);
  w += ((size_t)p.chunks * C * 9 * C * 4 + 255) & ~(size_t)255;
  float* partb2 = reinterpret_cast<float*>(w);
  w += ((size_t)p.chunks * C * 4 + 255) & ~(size_t)255;
  float* part0 = reinterpret_cast<float*>(w);
  {
    const int64_t n4 = M * C / 4;
    int64_t blocks = (n4 + kThr - 1) / kThr;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(ss_relu_mask_kernel, dim3((unsigned)blocks), dim3(kThr), 0, s, dY2, Y2,
                       n4, G);
  }
  // dgrad by parity class + conv0 weight-gradient partials
  {
    GemmArgs ga{};
    ga.src = G;
    ga.img = static_cast<const unsigned char*>(img);
    int64_t off = image_slots((int)C, 0);
    double cost[4], total = 0.0;
    for (int cl = 0; cl < 4; ++cl) {
      ga.img_off[cl] = off;
      off += image_slots((int)C, cl + 1);
      const int pt = cl >> 1, pf = cl & 1;
      const int T1c = pt ? d.T1 / 2 : (d.T1 + 1) / 2, F1c = pf ? d.F1 / 2 : (d.F1 + 1) / 2;
      ga.rows[cl] = (int64_t)d.B * T1c * F1c;
      const int64_t tiles = (ga.rows[cl] + 2 * kBM - 1) / (2 * kBM);
      cost[cl] = (double)tiles * (ksteps_of(class_taps(cl) * (int)C) + kDgradEpi);
      total += cost[cl];
    }
    int dg_blocks = 0, maxb = 1;
    for (int cl = 0; cl < 4; ++cl) {
      int nb = (int)(kDgradBlocks * cost[cl] / total);
      nb = nb < 1 ? 1 : nb;
      ga.blk_off[cl] = dg_blocks;
      ga.nblk[cl] = nb;
      dg_blocks += nb;
      maxb = nb > maxb ? nb : maxb;
    }
    ga.W0 = W0;
    ga.b0 = b0;
    ga.X = X;
    ga.part0 = part0;
    ga.d = d;
    const dim3 grid(maxb, 4);
    launch_gemm6_c<true>(C, ga, grid, s);
    hipLaunchKernelGGL(ss_w0_finish_kernel, dim3((unsigned)((C * 10 + 15) / 16)), dim3(kThr), 0,
                       s, (const float*)part0, dg_blocks, (int)C, dW0, db0);
  }
  // wgrad
  {
    const int tiles = p.tiles_n * 9 * p.tiles_k_per_tap;
    const unsigned nb = (unsigned)(tiles * p.chunks);
#define OB_WG(TW, WN)                                                                        \
  hipLaunchKernelGGL((ss_wgrad_kernel<TW, WN, WN>), dim3(nb), dim3(64 * WN * WN),            \
                     (size_t)(2 * WgCfg<TW, WN, WN>::kBuf), s, (const float*)G, Y1, d,       \
                     p.tiles_n, p.tiles_k_per_tap, p.rows_per_chunk, part2, partb2)
    if (p.tw == 3 && p.wn == 3) OB_WG(3, 3);
    else if (p.tw == 3 && p.wn == 2) OB_WG(3, 2);
    else if (p.tw == 3) OB_WG(3, 1);
    else OB_WG(2, 2);
#undef OB_WG
    const int64_t outs = (int64_t)C * 9 * C + C;
    hipLaunchKernelGGL(ss_wgrad_finish_kernel, dim3((unsigned)((outs + kThr - 1) / kThr)),
                       dim3(kThr), 0, s, (const float*)part2, (const float*)partb2, p.chunks,
                       (int)C, dW2, db2);
  }
}

}  // namespace ob
