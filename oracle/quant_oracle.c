/*
 * quant_oracle.c — CPU restatement of the reference quantizer (TEST INFRASTRUCTURE ONLY).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this; the
 * product path (libonebit_hip.so) never does.
 *
 * Restates y00njaekim/CMU-11785-IDL-1.58bit-ASR onebit_asr/quant.py, element by element,
 * in the same fp32 operation order:
 *   quant.py:124   a   = |alpha| + 1e-8f            (alpha_raw = 1) or alpha (alpha_raw = 0)
 *   quant.py:49    wa  = W / a                        (IEEE fp32 division)
 *   quant.py:50    clip(wa, -1, 1)
 *   quant.py:52-55 bits 1: Q = sign(clip), Q==0 -> +1
 *   quant.py:56-60 bits 2: Q = |clip| < 0.5 ? 0 : sign(clip)
 *   quant.py:68    W_hat = a * Q
 *   quant.py:81-82 grad_W = g * 1[|wa| <= 1]
 *   quant.py:86-91 grad_alpha = sum g * term(wa)
 * The clamp is applied literally here (the device code folds it away); the KATs in
 * tests/golden/quant_kat.json check that both agree at every threshold.
 *
 * Parity anchor: the reference ships no golden vectors for this path and running it here
 * was denied, so this file is pinned by hand-derived known answers
 * (tests/golden/quant_kat.json) and by its numpy twin (oracle/quant_oracle.py).
 *
 * Build: make -C oracle   (gcc, no -ffast-math: SSE fp32 arithmetic, no x87 excess precision)
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

static float eff_alpha(float alpha, int alpha_raw) {
  return alpha_raw ? (fabsf(alpha) + 1e-8f) : alpha;
}

static float tsign(float x) { return x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : 0.0f); }

static float clampf(float x, float lo, float hi) { return x < lo ? lo : (x > hi ? hi : x); }

/* Q value in {-1, 0, +1} of one weight (quant.py:49-60). */
static float q_value(float w, float a, int bits) {
  const volatile float wa = w / a; /* volatile: keep the fp32 rounding of the quotient */
  const float c = clampf(wa, -1.0f, 1.0f);
  if (bits == 1) {
    float q = tsign(c);
    return q == 0.0f ? 1.0f : q;
  }
  return fabsf(c) < 0.5f ? 0.0f : tsign(c);
}

/* Q values as int8 for n weights. Returns 0, or -3 for a bad bitwidth. */
int orc_quant_q(const float* W, int64_t n, float alpha, int alpha_raw, int bits, int8_t* q) {
  if (bits != 1 && bits != 2) return -3;
  const float a = eff_alpha(alpha, alpha_raw);
  for (int64_t i = 0; i < n; ++i) q[i] = (int8_t)q_value(W[i], a, bits);
  return 0;
}

/* W_hat = a * Q (quant.py:68). */
int orc_quant_dequant(const float* W, int64_t n, float alpha, int alpha_raw, int bits, float* out) {
  if (bits != 1 && bits != 2) return -3;
  const float a = eff_alpha(alpha, alpha_raw);
  for (int64_t i = 0; i < n; ++i) out[i] = a * q_value(W[i], a, bits);
  return 0;
}

/* Device code words for W[N][K] (layout of include/onebit_hip.h). */
static uint32_t code_of(float q) { return q > 0.0f ? 1u : (q < 0.0f ? 3u : 0u); }

int orc_quant_pack(const float* W, int64_t N, int64_t K, float alpha, int alpha_raw, int bits,
                   uint32_t* codes, uint32_t* codes_t) {
  if (bits != 1 && bits != 2) return -3;
  const float a = eff_alpha(alpha, alpha_raw);
  const int64_t KW = (K + 15) / 16, NW = (N + 15) / 16;
  if (codes) memset(codes, 0, sizeof(uint32_t) * (size_t)(N * KW));
  if (codes_t) memset(codes_t, 0, sizeof(uint32_t) * (size_t)(K * NW));
  for (int64_t n = 0; n < N; ++n)
    for (int64_t k = 0; k < K; ++k) {
      const uint32_t c = code_of(q_value(W[n * K + k], a, bits));
      if (codes) codes[n * KW + k / 16] |= c << (2 * (k % 16));
      if (codes_t) codes_t[k * NW + n / 16] |= c << (2 * (n % 16));
    }
  return 0;
}

/* term(wa) of quant.py:86-90, in the reference's operation order (-wa) + piece. */
static float alpha_term(float wa, int bits) {
  const float awa = fabsf(wa);
  const float s = tsign(wa);
  if (awa < 1.0f) {
    const float piece = (bits == 2) ? (awa >= 0.5f ? s : 0.0f) : s;
    return (-wa) + piece;
  }
  return s;
}

/*
 * STE backward (quant.py:72-92) for one weight tensor of n elements.
 * grad_W[i] = g[i] * 1[|wa| <= 1]; *grad_alpha_f64 = sum_i (float)(g[i]*term) accumulated in
 * double (an order-independent, tighter reference for the device's fp32 sums);
 * *grad_alpha_f32 = the same sum accumulated sequentially in fp32.
 * alpha_raw = 1 multiplies both sums by sgn(alpha) (autograd through alpha.abs()).
 */
int orc_ste_bwd(const float* g, const float* W, int64_t n, float alpha, int alpha_raw, int bits,
                float* grad_W, double* grad_alpha_f64, float* grad_alpha_f32) {
  if (bits != 1 && bits != 2) return -3;
  const float a = eff_alpha(alpha, alpha_raw);
  double acc = 0.0;
  float acc32 = 0.0f;
  for (int64_t i = 0; i < n; ++i) {
    const volatile float wa = W[i] / a;
    const float ind = fabsf(wa) <= 1.0f ? 1.0f : 0.0f;
    grad_W[i] = g[i] * ind;
    const volatile float prod = g[i] * alpha_term(wa, bits);
    acc += (double)prod;
    acc32 += prod;
  }
  const float chain = alpha_raw ? tsign(alpha) : 1.0f;
  *grad_alpha_f64 = acc * (double)chain;
  *grad_alpha_f32 = acc32 * chain;
  return 0;
}

/*
 * Ternary GEMM reference in double: Y[m][n] = a * sum_k X[m][k] * Q[n][k] + b[n]
 * (quant.py:126 with W_hat = a*Q). Double accumulation gives a summation-order-free
 * reference for fp32 kernels.
 */
int orc_bitlinear_fwd(const float* X, int64_t M, int64_t K, const float* W, int64_t N,
                      float alpha, int alpha_raw, int bits, const float* bias, double* Y) {
  if (bits != 1 && bits != 2) return -3;
  const float a = eff_alpha(alpha, alpha_raw);
  for (int64_t n = 0; n < N; ++n) {
    for (int64_t m = 0; m < M; ++m) Y[m * N + n] = 0.0;
  }
  for (int64_t n = 0; n < N; ++n) {
    for (int64_t k = 0; k < K; ++k) {
      const float q = q_value(W[n * K + k], a, bits);
      if (q == 0.0f) continue;
      const double wq = (double)(a * q);
      for (int64_t m = 0; m < M; ++m) Y[m * N + n] += (double)X[m * K + k] * wq;
    }
  }
  if (bias)
    for (int64_t m = 0; m < M; ++m)
      for (int64_t n = 0; n < N; ++n) Y[m * N + n] += (double)bias[n];
  return 0;
}
