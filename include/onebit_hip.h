/*
 * onebit_hip.h — C ABI of the MI355X (gfx950) BitLinear / QuantizedLinear hot path.
 *
 * This is the drop-in boundary for the reference's quantized linear layer
 * (y00njaekim/CMU-11785-IDL-1.58bit-ASR, onebit_asr/quant.py). The reference is
 * pure Python over torch eager ops; each entry point below replaces the torch
 * op sequence cited next to it. The Python host side
 * (cmu-11785-idl-1.58bit-asr_amd/onebit_asr/quant.py) binds these with ctypes.
 *
 * Conventions (all entry points):
 *   - plain C types only: device pointers, int64 sizes, a hipStream_t passed as void*;
 *   - every tensor is dense row-major fp32 (last dim contiguous) unless stated;
 *   - caller owns every buffer, including workspaces; nothing here allocates,
 *     synchronises the device or copies to/from the host, so every call is legal
 *     inside hipStreamBeginCapture/hipGraph capture;
 *   - return value: OB_OK (0) or a negative OB_ERR_* status; no exceptions cross
 *     the ABI; launch failures are reported as OB_ERR_HIP;
 *   - alpha is a DEVICE pointer to one fp32. With alpha_raw = 1 it is the raw
 *     learnable parameter and the kernels use a = |alpha| + 1e-8f exactly as
 *     QuantizedLinear.forward does (quant.py:124); with alpha_raw = 0 it is used
 *     as given (the quantize_weight(W, alpha, bits) entry, quant.py:95-96).
 *   - quant-off ceiling (BASELINE configs[3]: BitLinear -> bf16 nn.Linear): on the GEMM
 *     entries (ob_bitlinear_fwd*, ob_bitlinear_bwd_dx*), alpha_raw = 2 makes each codes
 *     argument a bf16 weight image (uint16 [N][K] = bf16(W) for the forward entries, [K][N]
 *     = bf16(W^T) for the dX entries' codes_t; ob_pack_item bits = 16 packs both) and the
 *     GEMM's B operand that image, with no alpha scale (activations stay exact fp32, as in
 *     every entry). Same kernels, tiles and fused epilogues as the ternary path.
 *   - bits is 1 (binary {-1,+1}, zero -> +1) or 2 (ternary {-1,0,+1}, threshold 0.5)
 *     (quant.py:52-60). bits = 32 is the full-precision passthrough and never
 *     reaches this library (quant.py:121-122); any other value -> OB_ERR_BITWIDTH,
 *     which the host maps to ValueError("bitwidth must be one of {1,2,32}")
 *     (quant.py:65-66).
 *
 * Packed weight codes (2 bits / weight, 16 per uint32, little-end first):
 *   00 -> 0, 01 -> +1, 11 -> -1 (10 unused).
 *   codes   [N][ceil(K/16)] : code of W[n][16*w + j] in bits 2j..2j+1 of codes[n][w]
 *   codes_t [K][ceil(N/16)] : code of W[16*w + j][k] in bits 2j..2j+1 of codes_t[k][w]
 *   Padding positions hold 00.
 */
#ifndef ONEBIT_HIP_H_
#define ONEBIT_HIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OB_API __attribute__((visibility("default")))

enum {
  OB_OK = 0,
  OB_ERR_NULL = -1,      /* a required pointer is NULL */
  OB_ERR_SHAPE = -2,     /* negative / inconsistent size */
  OB_ERR_BITWIDTH = -3,  /* bits not in {1,2} */
  OB_ERR_WORKSPACE = -4, /* workspace smaller than the *_workspace() query */
  OB_ERR_ALIGN = -5,     /* pointer not 4-byte aligned */
  OB_ERR_HIP = -6        /* hipGetLastError() after launch was not hipSuccess */
};

/* ABI version (bumped on any signature change). */
OB_API int ob_abi_version(void);
/* sha256 (hex) of the sources the library was built from (the .hip / .h files of csrc/ and
 * the headers of include/; onebit_asr/_digest.py), generated at build time: the host side refuses a
 * library whose digest differs from the sources beside it. */
OB_API const char* ob_source_digest(void);
/* Static string for a status code. */
OB_API const char* ob_status_string(int status);

/*
 * Quantize + pack (replaces _QuantizeSTE.forward's quantization, quant.py:49-60,
 * without materialising W_hat): codes and codes_t from W[N][K] and alpha.
 * Either output may be NULL to skip it.
 */
OB_API int ob_quant_pack(const float* W, const float* alpha, int alpha_raw, int bits,
                         int64_t N, int64_t K, uint32_t* codes, uint32_t* codes_t,
                         void* stream);

/*
 * Grouped pack: ob_quant_pack over a whole model's (layer, bitwidth) items in ONE launch
 * (the reference quantizes each QuantizedLinear inside its own forward, quant.py:123-126;
 * at Conformer-S a step needs 144 layers x 2 bitwidths). `items` is a DEVICE array of
 * n_items descriptors in block order: items[0].block0 = 0 and
 * items[i+1].block0 = items[i].block0 + ob_quant_pack_item_blocks(N_i, K_i);
 * total_blocks = the sum over all items. The table is built once (it holds the
 * persistent parameter and code buffer addresses) and the call is capture-safe.
 */
typedef struct ob_pack_item {
  const float* W;      /* [N][K] */
  const float* alpha;  /* 1 fp32, device */
  uint32_t* codes;     /* [N][ceil(K/16)] */
  uint32_t* codes_t;   /* [K][ceil(N/16)] */
  int64_t N, K;
  int64_t block0;      /* first block of this item */
  int32_t bits;        /* 1 or 2; 16: bf16 weight images (quant-off), codes <- uint16 [N][K]
                          bf16(W), codes_t <- uint16 [K][N] bf16(W^T), block count from
                          ob_weight_bf16_item_blocks */
  int32_t alpha_raw;
} ob_pack_item;

OB_API int64_t ob_quant_pack_item_blocks(int64_t N, int64_t K);
OB_API int64_t ob_weight_bf16_item_blocks(int64_t N, int64_t K);
OB_API int ob_quant_pack_group(const ob_pack_item* items, int n_items, int64_t total_blocks,
                               void* stream);

/*
 * quantize_weight forward, elementwise (quant.py:49-70): W_hat[i] = a * Q(W[i]/a).
 */
OB_API int ob_quant_dequant(const float* W, const float* alpha, int alpha_raw, int bits,
                            int64_t n, float* W_hat, void* stream);

/*
 * quantize_weight backward (quant.py:72-92): grad_W = g * 1[|W/a| <= 1];
 * grad_alpha[0] = sum(g * term(W/a)) (times sign(alpha) when alpha_raw = 1,
 * i.e. the chain through alpha.abs() at quant.py:124). Deterministic.
 */
OB_API size_t ob_quant_ste_bwd_workspace(int64_t n);
OB_API int ob_quant_ste_bwd(const float* grad_W_hat, const float* W, const float* alpha,
                            int alpha_raw, int bits, int64_t n, float* grad_W,
                            float* grad_alpha, void* ws, size_t ws_bytes, void* stream);

/*
 * BitLinear forward (replaces F.linear(x, alpha*Q, bias), quant.py:124-126):
 *   Y[M][N] = a * (X[M][K] . Q^T) + bias        (bias may be NULL)
 */
OB_API int ob_bitlinear_fwd(const float* X, int64_t M, int64_t K, const uint32_t* codes,
                            const float* alpha, int alpha_raw, const float* bias, int64_t N,
                            float* Y, void* stream);

/*
 * The same forward as a VALU sign-accumulate (north_star's first inner-product option: every
 * x * q with q in {-1, 0, +1} an exact signed add on packed fp32 FMA, one k-ordered chain
 * per output) -- the A/B partner of ob_bitlinear_fwd's bf16x3 MFMA kernel, not used by the
 * module path. K % 4 == 0 and X 16-B aligned, else OB_ERR_SHAPE / OB_ERR_ALIGN.
 * Replaces the same call (quant.py:126).
 */
OB_API int ob_bitlinear_fwd_signacc(const float* X, int64_t M, int64_t K, const uint32_t* codes,
                                    const float* alpha, int alpha_raw, const float* bias,
                                    int64_t N, float* Y, void* stream);

/*
 * BitLinear backward, input gradient (autograd of F.linear at quant.py:126):
 *   dX[M][K] = a * (dY[M][N] . Q)       using codes_t (layout above)
 */
OB_API int ob_bitlinear_bwd_dx(const float* dY, int64_t M, int64_t N, const uint32_t* codes_t,
                               const float* alpha, int alpha_raw, int64_t K, float* dX,
                               void* stream);

/*
 * BitLinear backward, weight / scale / bias gradients (F.linear autograd at
 * quant.py:126 fused with _QuantizeSTE.backward, quant.py:72-92):
 *   G        = dY^T . X                       ([N][K], summed over all M rows)
 *   dW       = G * 1[|W/a| <= 1]
 *   dalpha[0]= sum(G * term(W/a)) (* sign(alpha) when alpha_raw = 1)
 *   db[n]    = sum_m dY[m][n]                 (db may be NULL)
 * Deterministic (fixed-order split-M reduction); ws must hold
 * ob_bitlinear_bwd_dw_workspace(M, N, K) bytes.
 */
OB_API size_t ob_bitlinear_bwd_dw_workspace(int64_t M, int64_t N, int64_t K);
OB_API int ob_bitlinear_bwd_dw(const float* dY, const float* X, int64_t M, int64_t N, int64_t K,
                               const float* W, const float* alpha, int alpha_raw, int bits,
                               float* dW, float* dalpha, float* db, void* ws, size_t ws_bytes,
                               void* stream);

/*
 * Graph-mode variants: the bitwidth is read on device from *bits_dev (int32, 1 or 2) when
 * the kernel runs, so one captured HIP graph serves the stochastic-precision pass whose
 * per-block bitwidths change every step (reference train.py:102-103, conformer.py:265-269).
 * Same semantics as ob_quant_pack / ob_bitlinear_bwd_dw otherwise.
 */
OB_API int ob_quant_pack_dyn(const float* W, const float* alpha, int alpha_raw,
                             const int32_t* bits_dev, int64_t N, int64_t K, uint32_t* codes,
                             uint32_t* codes_t, void* stream);
OB_API int ob_bitlinear_bwd_dw_dyn(const float* dY, const float* X, int64_t M, int64_t N,
                                   int64_t K, const float* W, const float* alpha, int alpha_raw,
                                   const int32_t* bits_dev, float* dW, float* dalpha, float* db,
                                   void* ws, size_t ws_bytes, void* stream);

/*
 * Conv-module depthwise Conv1d (reference conformer.py:147
 * nn.Conv1d(C, C, KT, padding=KT//2, groups=C), applied at conformer.py:157).
 * x, y: [B][C][T]; w: [C][KT] (the Conv1d weight [C,1,KT]); bias [C] or NULL; KT odd, <= 64.
 *   y[b,c,t] = bias[c] + sum_j w[c,j] * x[b,c,t+j-KT/2]   (zero padding)
 * Backward: dx (may be NULL), dw [C][KT], db [C] (may be NULL); deterministic.
 */
OB_API int ob_dwconv1d_fwd(const float* x, const float* w, const float* bias, int64_t B,
                           int64_t C, int64_t T, int64_t KT, float* y, void* stream);
OB_API size_t ob_dwconv1d_bwd_workspace(int64_t B, int64_t C, int64_t KT);
OB_API int ob_dwconv1d_bwd(const float* x, const float* dy, const float* w, int64_t B, int64_t C,
                           int64_t T, int64_t KT, float* dx, float* dw, float* db, void* ws,
                           size_t ws_bytes, void* stream);

/*
 * CTC loss (reference losses.py:41-47: nn.CTCLoss(blank, zero_infinity=True), 'mean'),
 * with the lengths read on device so a training step can be captured in a HIP graph.
 * log_probs [B][T][V] (log_softmax output), targets [B][S] int64 padded, lengths int64 [B].
 * fwd writes loss[0] and fills ws (alpha, per-sample nll); bwd needs the same ws and writes
 * grad [B][T][V] with torch's CTC gradient formula, scaled by grad_out[0] (NULL -> 1).
 */
OB_API size_t ob_ctc_loss_workspace(int64_t B, int64_t T, int64_t S);
OB_API int ob_ctc_loss_fwd(const float* log_probs, const int64_t* targets,
                           const int64_t* input_lengths, const int64_t* target_lengths, int64_t B,
                           int64_t T, int64_t V, int64_t S, int blank, float* loss, void* ws,
                           size_t ws_bytes, void* stream);
OB_API int ob_ctc_loss_bwd(const float* log_probs, const int64_t* targets,
                           const int64_t* input_lengths, const int64_t* target_lengths, int64_t B,
                           int64_t T, int64_t V, int64_t S, int blank, const float* grad_out,
                           float* grad, void* ws, size_t ws_bytes, void* stream);
/* The same over G groups of B/G consecutive utterances in ONE launch (the three stacked
 * passes of a training step, each the reference's own ctc_loss_from_logits call,
 * losses.py:41-47): loss[g] is group g's 'mean' loss, grad_out[g] its incoming gradient. */
OB_API int ob_ctc_loss_fwd_groups(const float* log_probs, const int64_t* targets,
                                  const int64_t* input_lengths, const int64_t* target_lengths,
                                  int64_t G, int64_t B, int64_t T, int64_t V, int64_t S,
                                  int blank, float* loss, void* ws, size_t ws_bytes,
                                  void* stream);
OB_API int ob_ctc_loss_bwd_groups(const float* log_probs, const int64_t* targets,
                                  const int64_t* input_lengths, const int64_t* target_lengths,
                                  int64_t G, int64_t B, int64_t T, int64_t V, int64_t S,
                                  int blank, const float* grad_out, float* grad, void* ws,
                                  size_t ws_bytes, void* stream);
/* The same grouped CTC loss taken straight from the CTC head's logits [B][T][V]
 * (losses.py:41-47 is log_softmax then the CTC): the log-probabilities are read only at
 * blank and the utterance's labels, and the backward returns d loss / d logits
 * (= scale * (softmax - occupancy), torch's log-prob gradient composed with the log_softmax
 * backward up to its rounding-level sum term), so no [B*T][V] log_softmax or log-prob
 * gradient tensor exists. ws: ob_ctc_logits_workspace(B, T, S) bytes, kept from fwd to bwd.
 * logits / grad 16-byte aligned when V % 4 == 0. */
OB_API size_t ob_ctc_logits_workspace(int64_t B, int64_t T, int64_t S);
OB_API int ob_ctc_loss_logits_fwd_groups(const float* logits, const int64_t* targets,
                                         const int64_t* input_lengths,
                                         const int64_t* target_lengths, int64_t G, int64_t B,
                                         int64_t T, int64_t V, int64_t S, int blank, float* loss,
                                         void* ws, size_t ws_bytes, void* stream);
OB_API int ob_ctc_loss_logits_bwd_groups(const float* logits, const int64_t* targets,
                                         const int64_t* input_lengths,
                                         const int64_t* target_lengths, int64_t G, int64_t B,
                                         int64_t T, int64_t V, int64_t S, int blank,
                                         const float* grad_out, float* grad, void* ws,
                                         size_t ws_bytes, void* stream);

/* Decoder losses of the stacked step (replaces the torch expression of
 * onebit_asr/losses.py:22-35 att_ce_loss with label smoothing and :50-59 kl_logits, as
 * train.py:82-111 calls them per pass). logits [P][BU][V] fp32 (pass-major, P <= 64, pass 0 =
 * the teacher, detached for the KL); tgt_out [BU] int64 (tgt_out != pad_id marks the CE
 * positions); tgt_pad [BU] uint8 (1 = padded decoder input, dropped from the KL).
 * fwd: l_att[P] = mean_q(per-position smoothed CE) * msum / max(msum, 1) (the reference's
 * scalar-mean quirk) and l_kl[P-1] = sum_{q kept} KL(softmax(teacher_q) || softmax(x_pq)) /
 * max(kept, 1). bwd: grad [P][BU][V] from g_att[P], g_kl[P-1] (the teacher rows get only
 * their CE gradient). 0 < label_smoothing < 1; V % 4 == 0, V <= 8192; logits / grad 16-byte
 * aligned. ws: ob_att_kl_workspace(P, BU) bytes, kept from fwd to bwd. */
OB_API size_t ob_att_kl_workspace(int64_t P, int64_t BU);
OB_API int ob_att_kl_loss_fwd(const float* logits, const int64_t* tgt_out,
                              const uint8_t* tgt_pad, int64_t P, int64_t BU, int64_t V,
                              int pad_id, float label_smoothing, float* l_att, float* l_kl,
                              void* ws, size_t ws_bytes, void* stream);
OB_API int ob_att_kl_loss_bwd(const float* logits, const int64_t* tgt_out,
                              const uint8_t* tgt_pad, int64_t P, int64_t BU, int64_t V,
                              float label_smoothing, const float* g_att, const float* g_kl,
                              float* grad, const void* ws, size_t ws_bytes, void* stream);
/* The training step's loss from its per-pass parts (train.py:95-111 with the three passes
 * stacked: teacher 2-bit, student 1-bit, SP): l_int[p] = (1 - gamma) l_att[p] + gamma l_ctc[p],
 * loss = l_int[0] + lambda1 (l_int[1] + l_int[2]) + lambda2 (l_kl[0] + l_kl[1]) -- each
 * multiply and add rounded in that order (the torch expression's sequence) -- and
 * parts[8] = (l_int[0..2], l_kl[0..1], l_ctc[0..2]). DEVICE pointers, one launch each way.
 * bwd: from g_loss [1]: d_att[3], d_ctc[3], d_kl[2] (the expression's autograd). */
OB_API int ob_loss_combine_fwd(const float* l_att, const float* l_ctc, const float* l_kl,
                               float gamma, float lambda1, float lambda2, float* loss,
                               float* parts, void* stream);
OB_API int ob_loss_combine_bwd(const float* g_loss, float gamma, float lambda1, float lambda2,
                               float* d_att, float* d_ctc, float* d_kl, void* stream);

/* ------------------------------------------------------------------------------------
 * Stacked passes. The reference's training step runs every BitLinear three times per
 * batch -- 2-bit teacher, 1-bit student and the stochastic-precision pass
 * (onebit_asr/train.py:82-105) -- each a separate QuantizedLinear.forward
 * (quant.py:120-127) whose autograd gradients torch then sums. These entries take the P
 * passes of one layer stacked along rows: X is [P][M][K] (P*M rows), pass p runs at
 * bitwidth pass_bits[p] (DEVICE int32 [P]; 1 selects the 1-bit codes, anything else the
 * 2-bit codes), so the per-step SP mask can change without re-launch decisions on the
 * host. codes2 / codes1 are the ob_quant_pack outputs of the same (W, alpha) for
 * bits 2 and 1.
 *   fwd : Y[p] = a * X[p] . Q_{bits_p}^T + bias
 *   dX  : dX[p] = a * dY[p] . Q_{bits_p}
 *   dW  : dW = 1[|W/a| <= 1] * sum_p dY[p]^T X[p]; dalpha = sum_p sum(G_p * term_{bits_p})
 *         * d|alpha|; db = sum over all P*M rows of dY -- the sum over passes the
 *         reference's autograd forms (the STE mask does not depend on the bitwidth).
 * P <= 4 for dW (ob_bitlinear_bwd_dw_passes_workspace returns 0 otherwise).
 * ------------------------------------------------------------------------------------ */
OB_API int ob_bitlinear_fwd_passes(const float* X, int64_t P, int64_t M, int64_t K,
                                   const uint32_t* codes2, const uint32_t* codes1,
                                   const int32_t* pass_bits, const float* alpha, int alpha_raw,
                                   const float* bias, int64_t N, float* Y, void* stream);
/* G <= 3 layers of one input (the q / k / v projections of one LayerNorm output,
 * conformer.py:111-113) as ONE launch: Y[i] = ob_bitlinear_fwd_passes(X, codes2[i],
 * codes1[i], alpha[i], bias[i]) for each i (same K, N; the arrays are HOST arrays of device
 * pointers, bias[i] may be NULL). Same arithmetic as G separate calls (bit-identical). */
OB_API int ob_bitlinear_fwd_passes_group(int64_t G, const float* X, int64_t P, int64_t M,
                                         int64_t K, const uint32_t* const* codes2,
                                         const uint32_t* const* codes1, const int32_t* pass_bits,
                                         const float* const* alpha, int alpha_raw,
                                         const float* const* bias, int64_t N, float* const* Y,
                                         void* stream);
/*
 * Opt-in int8 activation mode (north_star "per-tensor absmax int8 activations"; NOT the
 * reference's arithmetic, which keeps activations fp32 at quant.py:126 -- SURVEY.md §0
 * F3). Replaces, for QuantizedLinear.act_quant == "absmax_int8", the F.linear call of
 * quant.py:126 by BitNet-b1.58 activation quantization x int8 matrix cores:
 *   g_p = max(max|X_p|, 1e-5); sx = 127/g_p; xq = clamp(rint(x*sx), -127, 127);
 *   Y = float(sum_k xq*Q) * (a * (g_p/127)) + b   (mul then add, each rounded: no fma).
 * ob_act_absmax: amax[p] = max|X_p| over the n_per_pass elements of pass p (per-block
 *   partials in ws, then a final reduce; order-independent, so deterministic). X 16-byte
 *   aligned, n_per_pass % 4 == 0; ws of ob_act_absmax_workspace(P) bytes.
 * ob_act_dequant_i8: X_deq = xq * (g_p/127) (the activations the int8 forward multiplied;
 *   dW = dY^T X_deq under the straight-through estimator).
 * ob_bitlinear_fwd_i8: P passes stacked on rows like ob_bitlinear_fwd_passes; P == 1 may
 *   pass pass_bits = NULL (then codes is used and codes1 is ignored). Needs K % 16 == 0,
 *   K <= 576 (OB_ERR_SHAPE otherwise) and X 16-byte aligned.
 */
OB_API size_t ob_act_absmax_workspace(int64_t P);
OB_API int ob_act_absmax(const float* X, int64_t P, int64_t n_per_pass, float* amax, void* ws,
                         size_t ws_bytes, void* stream);
OB_API int ob_act_dequant_i8(const float* X, int64_t P, int64_t n_per_pass, const float* amax,
                             float* X_deq, void* stream);
OB_API int ob_bitlinear_fwd_i8(const float* X, int64_t P, int64_t M, int64_t K,
                               const uint32_t* codes, const uint32_t* codes1,
                               const int32_t* pass_bits, const float* alpha, int alpha_raw,
                               const float* amax, const float* bias, int64_t N, float* Y,
                               void* stream);

/* ob_bitlinear_fwd_i8 with the inference call sites' epilogues fused (conformer.py:36-45
 * and :131-138 at dropout 0), N % 4 == 0, X / Y / R 16-byte aligned:
 *   mode 1 (swish)    Y = silu(y) and amax_out[p] = max|Y_p| (amax_out zeroed first): the
 *                     producer-side int8 scale of the next BitLinear (ff.lin2);
 *   mode 2 (residual) Y = R + rscale * (valid ? y : 0*y), row r valid iff lens == NULL or
 *                     (r % T) < lens[r / T] (padded frames zeroed, :137);
 * where y = the ob_bitlinear_fwd_i8 output. */
OB_API int ob_bitlinear_fwd_i8_epi(const float* X, int64_t P, int64_t M, int64_t K,
                                   const uint32_t* codes, const uint32_t* codes1,
                                   const int32_t* pass_bits, const float* alpha, int alpha_raw,
                                   const float* amax, const float* bias, int64_t N, int mode,
                                   const float* R, float rscale, const int32_t* lens, int64_t T,
                                   float* amax_out, float* Y, void* stream);

/* ob_bitlinear_fwd_i8 on an int8 operand Xq [P*M][K] already quantised by its producer at
 * the scale of amax (ob_layernorm_fwd_i8, or mode 3 below): the A tiles are read as int8
 * (K bytes per row instead of 4K). N % 4 == 0; Xq / Y / R 16-byte aligned.
 *   mode 0  Y fp32 = y                              (as ob_bitlinear_fwd_i8)
 *   mode 2  Y fp32 = R + rscale * (valid ? y : 0*y)  (as ob_bitlinear_fwd_i8_epi mode 2)
 *   mode 3  Y int8 = the int8 image of silu(y) at amax_out[p] = max|silu(y)| over pass p
 *           (N % 16 == 0)
 *           (ff.lin1 -> ff.lin2, conformer.py:36-39 at dropout 0): the product is
 *           computed twice (absmax, then quantise + store), so silu(y) never reaches HBM
 *           in fp32; ff.lin2 on Y (mode 2) equals ob_bitlinear_fwd_i8_epi mode 1 -> mode 2
 *           bit for bit. */
OB_API int ob_bitlinear_fwd_i8q(const int8_t* Xq, int64_t P, int64_t M, int64_t K,
                                const uint32_t* codes, const uint32_t* codes1,
                                const int32_t* pass_bits, const float* alpha, int alpha_raw,
                                const float* amax, const float* bias, int64_t N, int mode,
                                const float* R, float rscale, const int32_t* lens, int64_t T,
                                float* amax_out, void* Y, void* stream);

OB_API int ob_bitlinear_bwd_dx_passes(const float* dY, int64_t P, int64_t M, int64_t N,
                                      const uint32_t* codes2_t, const uint32_t* codes1_t,
                                      const int32_t* pass_bits, const float* alpha,
                                      int alpha_raw, int64_t K, float* dX, void* stream);
/* The summed input gradient of G BitLinears that read the same input (the q / k / v
 * projections of one LayerNorm output, conformer.py:111-113; autograd sums their input
 * gradients): dX = sum_g alpha_g dY_g . Q_g (autograd of quant.py:126 per layer, summed) in
 * ONE launch, each dY_g [P*M][N] against its own codes (codes2_t[g] / codes1_t[g] as
 * ob_bitlinear_bwd_dx_passes, per-pass bitwidths from pass_bits), each product formed as
 * (alpha_g dY_g) Q_g (the reference's dY (alpha Q) product rounding). Host arrays of G
 * device pointers. Taken for G = 3, N = 144, K a multiple of 144, 16-byte aligned dY / dX;
 * otherwise OB_ERR_SHAPE with nothing launched (run ob_bitlinear_bwd_dx_passes per source). */
OB_API int ob_bitlinear_bwd_dx_passes_sum(int64_t G, const float* const* dY, int64_t P,
                                          int64_t M, int64_t N, const uint32_t* const* codes2_t,
                                          const uint32_t* const* codes1_t,
                                          const int32_t* pass_bits, const float* const* alpha,
                                          int alpha_raw, int64_t K, float* dX, void* stream);
OB_API size_t ob_bitlinear_bwd_dw_passes_workspace(int64_t P, int64_t M, int64_t N, int64_t K);
OB_API int ob_bitlinear_bwd_dw_passes(const float* dY, const float* X, int64_t P, int64_t M,
                                      int64_t N, int64_t K, const float* W, const float* alpha,
                                      int alpha_raw, const int32_t* pass_bits, float* dW,
                                      float* dalpha, float* db, void* ws, size_t ws_bytes,
                                      void* stream);
/* G (<= 3) layers of the same input X and shape (the q/k/v projections of one LayerNorm
 * output, conformer.py:111-113): ob_bitlinear_bwd_dw_passes of each, their finishes (chunk
 * sum, STE mask, db, dalpha) in ONE launch. Same arithmetic per layer. Arrays of G device
 * pointers (host arrays); db[i] may be NULL. ws: ..._group_workspace(G, P, M, N, K) bytes. */
OB_API size_t ob_bitlinear_bwd_dw_passes_group_workspace(int64_t G, int64_t P, int64_t M,
                                                         int64_t N, int64_t K);
OB_API int ob_bitlinear_bwd_dw_passes_group(int64_t G, const float* const* dY, const float* X,
                                            int64_t P, int64_t M, int64_t N, int64_t K,
                                            const float* const* W, const float* const* alpha,
                                            int alpha_raw, const int32_t* pass_bits,
                                            float* const* dW, float* const* dalpha,
                                            float* const* db, void* ws, size_t ws_bytes,
                                            void* stream);

/* Deferred weight-gradient finishes (reference train.py:104-111: the parameter gradients
 * are read only by clip_grad_norm_ / AdamW after loss.backward() ends). The *_defer entries
 * launch only the split-M partial GEMM; the partial launch itself writes the layer's finish
 * descriptor (chunk sum + STE mask + db + dalpha, as ob_bitlinear_bwd_dw_passes) into slot
 * `slot` of a caller-owned device table of ob_dw_finish_entry_bytes() entries, at finish
 * block offset `start`, and returns the layer's finish block count in *n_blocks (0: the shape
 * took a path that finished immediately -- no entry written). ob_dw_finish_table then runs
 * every entry's finish in ONE launch (total_blocks = the sum of the counts, entries in slot
 * order). Until it has run, dW / dalpha / db are undefined; the workspace must stay
 * allocated. The group form writes G consecutive entries (G <= 3). */
OB_API size_t ob_dw_finish_entry_bytes(void);
OB_API int ob_bitlinear_bwd_dw_passes_defer(const float* dY, const float* X, int64_t P,
                                            int64_t M, int64_t N, int64_t K, const float* W,
                                            const float* alpha, int alpha_raw,
                                            const int32_t* pass_bits, float* dW, float* dalpha,
                                            float* db, void* ws, size_t ws_bytes, void* table,
                                            int64_t slot, int64_t start, int64_t* n_blocks,
                                            void* stream);
OB_API int ob_bitlinear_bwd_dw_passes_group_defer(
    int64_t G, const float* const* dY, const float* X, int64_t P, int64_t M, int64_t N,
    int64_t K, const float* const* W, const float* const* alpha, int alpha_raw,
    const int32_t* pass_bits, float* const* dW, float* const* dalpha, float* const* db,
    void* ws, size_t ws_bytes, void* table, int64_t slot, int64_t start, int64_t* n_blocks,
    void* stream);
OB_API int ob_dw_finish_table(const void* table, int64_t n, int64_t total_blocks, void* stream);

/* Grouped deferred weight gradients. Every weight gradient of a backward whose N and K are
 * multiples of 144 -- a BitLinear's (autograd of quant.py:126 through quant.py:72-92: dW with
 * the STE mask, dalpha at each stacked pass's bitwidth, db) or a dense linear's (W == NULL:
 * dW = dY^T X, db) -- computed in ONE persistent launch after the backward (the reference reads
 * parameter gradients only after loss.backward(), train.py:104-111), instead of one split-M
 * launch per layer plus the finish table. Rows of pass p are rows p*M .. p*M+M-1 of dY and X.
 * `gemms` is a HOST array of G descriptors (device pointers inside). `tickets`: a caller-owned
 * device buffer of ob_dw_grouped_tickets(...) uint32 words, all zero before the first call;
 * every call leaves it zero. Deterministic: fixed partition of the rows, fixed summation order.
 * dY / X / W / alpha / pass_bits must stay valid until the launch has run. */
typedef struct ob_dwg_gemm {
  const float* dY;          /* [P*M][N] */
  const float* X;           /* [P*M][K] */
  const float* W;           /* [N][K] BitLinear weight; NULL = dense (no STE mask, no dalpha) */
  const float* alpha;       /* BitLinear: 0-dim alpha (alpha_raw as ob_bitlinear_bwd_dw) */
  const int32_t* pass_bits; /* DEVICE [P] bitwidths (1 or 2); NULL: `bits` for every pass */
  float* dW;                /* [N][K] */
  float* db;                /* [N] or NULL */
  float* dalpha;            /* 0-dim (BitLinear; unused when W == NULL) */
  int64_t N, K, M, P;       /* M = rows of one pass (>= 1), 1 <= P <= 4 */
  int32_t alpha_raw, bits;
} ob_dwg_gemm;
OB_API int ob_dw_grouped_supported(int64_t N, int64_t K);
OB_API size_t ob_dw_grouped_workspace(const ob_dwg_gemm* gemms, int64_t G);
OB_API size_t ob_dw_grouped_tickets(const ob_dwg_gemm* gemms, int64_t G);
OB_API int ob_dw_grouped(const ob_dwg_gemm* gemms, int64_t G, void* ws, size_t ws_bytes,
                         void* tickets, size_t ticket_words, void* stream);

/* ------------------------------------------------------------------------------------
 * The decoder's attention core (onebit_asr/conformer.py:275-299: the stock
 * nn.TransformerDecoderLayer self- and cross-attention, torch's
 * multi_head_attention_forward between the in- and out-projections):
 *   ctx = dropout(softmax((q k^T) * (1/sqrt(dh)) + mask)) v    per head
 * q [B][Lq][*] with row stride sq floats (head h = columns h*dh .. h*dh+dh-1), k / v
 * [B][Lk][*] (strides sk / sv): the packed projection outputs are read in place. mask: key j
 * of batch row b is -inf when kmask[b*Lk + j] != 0 (kmask may be NULL) and, causal != 0,
 * when j > i. ctx [B][Lq][H*dh]; probs [B][H][Lq][Lk] (the softmax output, a dropped
 * element stored negated) is kept for the backward. Dropout p_drop: the library's counter
 * hash on (rng, rng_offset), like every fused dropout. Supported: dh in {16, 32, 36, 64},
 * Lk <= 256 and the per-(b, h) working set within LDS (ob_decattn_supported).
 * ctx must be 16-byte aligned. bwd (ctx = the forward's output): dq [B][Lq][*] (row stride
 * gq), dk / dv [B][Lk][*] (gk / gv), every element of the heads' columns written -- e.g.
 * straight into the packed projection's gradient. The backward CONSUMES probs: it holds the
 * score gradients dS' afterwards (two launches: dk / dv, then dq from dS'); ABI 4. */
OB_API int ob_decattn_supported(int64_t Lq, int64_t Lk, int64_t dh);
OB_API int ob_decattn_fwd(const float* q, int64_t sq, const float* k, int64_t sk, const float* v,
                          int64_t sv, const uint8_t* kmask, int64_t causal, int64_t B, int64_t H,
                          int64_t Lq, int64_t Lk, int64_t dh, float p_drop, const int64_t* rng,
                          int64_t rng_offset, float* probs, float* ctx, void* stream);
OB_API int ob_decattn_bwd(const float* dctx, const float* ctx, const float* q, int64_t sq,
                          const float* k, int64_t sk, const float* v, int64_t sv, int64_t B, int64_t H, int64_t Lq,
                          int64_t Lk, int64_t dh, float p_drop, float* probs, float* dq,
                          int64_t gq, float* dk, int64_t gk, float* dv, int64_t gv, void* stream);

/* ------------------------------------------------------------------------------------
 * Relative-position attention core of MHSA.forward (onebit_asr/conformer.py:115-127),
 * fused: ac = (q+u) k^T, bd = rel_shift((q+v) pos^T) (:97-103), S = (ac + bd) / sqrt(d),
 * frames i or j >= lens[b] masked to -inf (:121-122), A = nan_to_num(softmax(S))
 * (:123-125), A = dropout(A) (:126), ctx = A v (:127).
 *   q, k, v, ctx, dq, dk, dv : [Bt][T][H*d]   (heads side by side, as the projections
 *                              produce them and out_proj consumes them)
 *   pos, dpos : [P][T][H*d]    (pass p = b / (Bt/P) for stacked passes; P = 1 otherwise)
 *   u, vb, du, dvb : [H][d]    (pos_bias_u / pos_bias_v)
 *   lens : DEVICE int32 [Bt]   (valid frames; the encoder's prefix masks)
 *   saved : the forward's state for the backward (ob_relattn_saved_elems fp32 elements,
 *           16-B aligned; NULL when no backward follows): row statistics [Bt*H][Tp][2]
 *           (max of the scaled masked scores, 1/sum; Tp = 16*ceil(T/16)), the dropout keep
 *           bits [Bt*H][Tp][W] (uint32, W = ceil(Tp/32), key j of row i = bit j%32 of word
 *           j/32), then (default backward mode) the probability tiles below -- the
 *           statistics region is reserved but not written -- or, in the flash backward mode
 *           (ob_relattn_set_bwd_mode(1) or OB_ATTN_BWD=flash; only T <= 256 and d <= 36, other
 *           shapes always take the probability tiles), the statistics, the keep bits and the
 *           X rows below each 32-query chunk: that backward recomputes the probabilities of
 *           32-query chunks (bitwise the forward's) and keeps every [T][T] quantity on chip.
 *           It is slower at Conformer-S, hence opt-in.
 *   probs : optional (NULL: not written) MFMA-fragment tiles [Bt*H][nt][nt][64][4],
 *           nt = ceil(T/16), of the softmax before dropout (ob_relattn_probs_elems floats):
 *           tile (a, t), lane r + 16g, element e holds P[16a + r][16t + 4g + e] (rows / keys
 *           >= T: 0); with p_drop > 0 a dropped element is stored as -P.
 *   ctx (bwd) : the forward's output (the softmax backward's row term is dO . ctx)
 *   rng : DEVICE int64 [2] (seed, counter), rng_offset a host offset added to the counter
 *         (the fused BitLinear entries' convention: one device state, a distinct offset per
 *         call site, the counter advanced once per step); dropout keeps element (i, j) of
 *         row bh when the 16-bit field (j & 1) of hash(seed, counter + rng_offset,
 *         ((bh*T + i)*Te + j) / 2) >= p_drop * 2^16, Te = T rounded up to even (the bwd
 *         reads the forward's decisions from the saved keep bits; ob_relattn_dropout_mask
 *         writes the mask out). Unused when p_drop == 0.
 * Supported: 1 <= T <= 512, d in {16, 32, 36, 64}.
 * ------------------------------------------------------------------------------------ */
OB_API int ob_relattn_fwd(const float* q, const float* k, const float* v, const float* pos,
                          const float* u, const float* vb, const int32_t* lens, int64_t Bt,
                          int64_t P, int64_t T, int64_t H, int64_t d, float p_drop,
                          const int64_t* rng, int64_t rng_offset, float* saved, float* probs,
                          float* ctx, void* stream);
OB_API int64_t ob_relattn_saved_elems(int64_t Bt, int64_t T, int64_t H, int64_t d);
OB_API int64_t ob_relattn_probs_elems(int64_t Bt, int64_t T, int64_t H);
OB_API size_t ob_relattn_bwd_workspace(int64_t Bt, int64_t T, int64_t H, int64_t d);
OB_API int ob_relattn_bwd(const float* dctx, const float* ctx, const float* q, const float* k,
                          const float* v, const float* pos, const float* u, const float* vb,
                          const int32_t* lens, int64_t Bt, int64_t P, int64_t T, int64_t H,
                          int64_t d, float p_drop, const int64_t* rng, int64_t rng_offset,
                          const float* saved, int64_t saved_elems,
                          float* dq, float* dk, float* dv, float* dpos, float* du, float* dvb,
                          void* ws, size_t ws_bytes, void* stream);
/* The attention backward mode, process-wide: 0 = probability tiles (default), 1 = flash style
 * (T <= 256, d <= 36); any other value only queries. Returns the previous mode. The initial
 * mode is OB_ATTN_BWD (read once). ob_relattn_saved_elems / ob_relattn_bwd_workspace follow the
 * current mode; ob_relattn_bwd returns OB_ERR_SHAPE when `saved_elems` (the size the forward's
 * buffer was allocated with) is not the current mode's -- the mode changed in between. */
OB_API int ob_relattn_set_bwd_mode(int mode);
/* The dropout keep-mask (1 = kept) of n elements laid out in rows of row_len: the attention
 * kernels' mask of [rows][T] probabilities with row_len = T, the BitLinear / LayerNorm /
 * residual-dropout kernels' mask of a flat tensor with row_len = n. */
OB_API int ob_relattn_dropout_mask(int64_t n, int64_t row_len, float p_drop, const int64_t* rng,
                                   int64_t rng_offset, uint8_t* out, void* stream);

/* Token-embedding backward of the decoder (conformer.py:279-299, nn.Embedding with
 * padding_idx): grad_weight[v] = sum over n ascending with indices[n] == v of grad[n]
 * (deterministic, graph-safe); grad_weight[padding_idx] = 0 (padding_idx < 0: none).
 * indices int64 [N] in [0, V); grad [N][C]; grad_weight [V][C]; C <= 1024. */
OB_API int ob_embedding_bwd(const int64_t* indices, int64_t N, const float* grad, int64_t C,
                            int64_t V, int64_t padding_idx, float* grad_weight, void* stream);

/* ------------------------------------------------------------------------------------
 * Optimizer tail of the training step: clip_grad_norm_(params, max_norm) followed by
 * AdamW.step() (reference onebit_asr/train.py:116-118 with the optimizer of train.py:259:
 * betas (0.9, 0.98), eps 1e-8, weight_decay 1e-2). torch issues per-tensor launches for
 * the ~800 parameter tensors; this is three launches over a table of tensors.
 *
 * table     : DEVICE array of n_tensors descriptors (param, grad, exp_avg, exp_avg_sq are
 *             device fp32 buffers of numel elements; exp_avg / exp_avg_sq start at 0)
 * chunk_map : DEVICE int64 [2 * n_blocks] from ob_adamw_plan (host) for the same numels
 * lr        : DEVICE fp32 learning rate (the warmup-cosine schedule writes it)
 * step      : DEVICE fp32 step counter shared by all tensors; incremented by the call
 * grad_scale: every gradient is multiplied by it first (1/world after a SUM all-reduce)
 * max_norm  : <= 0 disables clipping. total_norm (optional DEVICE fp32) receives the
 *             pre-clip global L2 norm, as clip_grad_norm_ returns it.
 * Gradients are clipped in registers (the grad buffers are not modified).
 * ------------------------------------------------------------------------------------ */
typedef struct ob_adamw_tensor {
  float* param;
  const float* grad;
  float* exp_avg;
  float* exp_avg_sq;
  int64_t numel;
} ob_adamw_tensor;

/* Host-only. Number of blocks for these tensor sizes; fills chunk_map (HOST int64
 * [2 * n_blocks]) when non-NULL. Negative status for an empty table or numel < 1. */
OB_API int64_t ob_adamw_plan(const int64_t* numels, int64_t n_tensors, int64_t* chunk_map);
OB_API size_t ob_adamw_workspace(int64_t n_blocks);
OB_API int ob_adamw_clip_step(const ob_adamw_tensor* table, int64_t n_tensors,
                              const int64_t* chunk_map, int64_t n_blocks, const float* lr,
                              float* step, float grad_scale, double beta1, double beta2,
                              double eps, double weight_decay, double max_norm,
                              float* total_norm, void* ws,
                              size_t ws_bytes, void* stream);

/*
 * LayerNorm over the last dim (the Conformer's LayerNorm wrappers, conformer.py:19-24:
 * nn.LayerNorm(d) before every BitLinear call site). x, y [rows][d], d <= 512;
 * gamma/beta [d] or NULL (1 / 0); mean, rstd [rows] (either may be NULL when no backward
 * follows). var is biased (torch), rstd = 1/sqrt(var + eps).
 * Backward: dx [rows][d]; dgamma/dbeta [d] (NULL to skip) summed over rows in a fixed
 * order (deterministic) through the workspace.
 */
OB_API int ob_layernorm_fwd(const float* x, const float* gamma, const float* beta, int64_t rows,
                            int64_t d, float eps, float* y, float* mean, float* rstd,
                            void* stream);
/* Two LayerNorms back to back (a Conformer block's final LN, conformer.py:228, and the next
 * module's input LN, :28 / the encoder's output LN): y1 = LN1(x) (gamma g1, beta b1), y2 =
 * LN2(y1), with both rows' mean / rstd (each may be NULL), in one pass over x -- bit-identical
 * to two ob_layernorm_fwd calls. */
OB_API int ob_layernorm_fwd_pair(const float* x, const float* g1, const float* b1,
                                 const float* g2, const float* b2, int64_t rows, int64_t d,
                                 float eps1, float eps2, float* y1, float* mean1, float* rstd1,
                                 float* y2, float* mean2, float* rstd2, void* stream);
/* ob_layernorm_fwd plus amax[p] = max|y| over pass p (rows split into P equal passes,
 * P <= 8): the producer-side per-tensor scale of the int8 BitLinear that consumes y.
 * ws: ob_layernorm_fwd_amax_workspace(P) bytes (per-block partial maxima). */
OB_API size_t ob_layernorm_fwd_amax_workspace(int64_t P);
OB_API int ob_layernorm_fwd_amax(const float* x, const float* gamma, const float* beta,
                                 int64_t rows, int64_t d, float eps, float* y, float* mean,
                                 float* rstd, int64_t P, float* amax, void* ws,
                                 size_t ws_bytes, void* stream);
/* The int8 image of LN(x) for an int8 BitLinear consumer (north_star "int8 activation tiles"
 * in HBM): amax[p] = max|LN(x)| over pass p, then yq = clamp(rint(LN(x) * 127 /
 * max(amax[p], 1e-5)), -127, 127) int8 [rows][d] -- the quantisation ob_bitlinear_fwd_i8
 * applies in registers to an fp32 operand, so ob_bitlinear_fwd_i8q on yq is bit-identical to
 * ob_bitlinear_fwd_i8 on LN(x). Two row passes (LN is recomputed; no fp32 y in HBM);
 * ws: ob_layernorm_fwd_amax_workspace(P) bytes; yq 4-byte aligned. Replaces the pair
 * LayerNorm (conformer.py:19-24) -> activation quantisation of the consumer. */
OB_API int ob_layernorm_fwd_i8(const float* x, const float* gamma, const float* beta,
                               int64_t rows, int64_t d, float eps, int64_t P, float* amax,
                               int8_t* yq, void* ws, size_t ws_bytes, void* stream);
OB_API size_t ob_layernorm_bwd_workspace(int64_t rows, int64_t d);
OB_API int ob_layernorm_bwd(const float* dy, const float* x, const float* gamma,
                            const float* mean, const float* rstd, int64_t rows, int64_t d,
                            float* dx, float* dgamma, float* dbeta, void* ws, size_t ws_bytes,
                            void* stream);
/* ob_layernorm_bwd plus an additive gradient: dx = LN_backward(dy) + dres. At a residual
 * junction x -> (LN -> module) + x (conformer.py:34-45, :105-138, :149-167) this is the
 * sum autograd would form with a separate add kernel. */
OB_API int ob_layernorm_bwd_res(const float* dy, const float* x, const float* gamma,
                                const float* mean, const float* rstd, int64_t rows, int64_t d,
                                const float* dres, float* dx, float* dgamma, float* dbeta,
                                void* ws, size_t ws_bytes, void* stream);
/* ob_layernorm_bwd / _res (dres may be NULL) with an optional second output for the module
 * whose output this LN normalises: dy2 = rscale * rowvalid * drop(dx), element for element
 * ob_drop_scale_bwd(dx, rows, d, rscale, p_drop, rng, rng_offset, lens, T) -- the backward
 * of that module's residual tail "R + rscale * rowvalid * dropout(y)" (conformer.py:39-45,
 * :131-138, :160-167), formed while dx is in registers instead of in a pass of its own.
 * dy2 == NULL: plain ob_layernorm_bwd_res. */
OB_API int ob_layernorm_bwd_ex(const float* dy, const float* x, const float* gamma,
                               const float* mean, const float* rstd, int64_t rows, int64_t d,
                               const float* dres, float* dx, float* dgamma, float* dbeta,
                               void* ws, size_t ws_bytes, float* dy2, float rscale,
                               float p_drop, const uint64_t* rng, int64_t rng_offset,
                               const int32_t* lens, int64_t T, void* stream);
/* ob_layernorm_bwd_ex with the dgamma / dbeta reduction deferred (table != NULL): the
 * backward launch writes its partials' descriptor into slot `slot` of a caller-owned device
 * table of ob_ln_param_entry_bytes() entries; ob_ln_param_table reduces entries 0 .. n-1 in
 * one launch (dmax = the largest d) with the same fixed-order arithmetic. ws stays allocated
 * until then. dres / dy2 may be NULL. */
OB_API int ob_layernorm_bwd_defer(const float* dy, const float* x, const float* gamma,
                                  const float* mean, const float* rstd, int64_t rows, int64_t d,
                                  const float* dres, float* dx, float* dgamma, float* dbeta,
                                  void* ws, size_t ws_bytes, float* dy2, float rscale,
                                  float p_drop, const uint64_t* rng, int64_t rng_offset,
                                  const int32_t* lens, int64_t T, void* table, int64_t slot,
                                  void* stream);
/* The backward of two LayerNorms back to back (ob_layernorm_fwd_pair: y1 = LN1(x), y2 =
 * LN2(y1); gres = the gradient of y1's other (residual) use, may be NULL): dx =
 * LN1_backward(LN2_backward(dy) + gres), the sum never written to memory; dy2 (may be NULL):
 * the residual-tail gradient of ob_layernorm_bwd_ex for x; dgamma / dbeta of both layers,
 * deferred into `table` at slot2 / slot1 (>= 0) or reduced now (table NULL or slot < 0).
 * ws: ob_layernorm_bwd_pair_workspace(rows, d) bytes, 16-byte aligned. */
OB_API size_t ob_layernorm_bwd_pair_workspace(int64_t rows, int64_t d);
OB_API int ob_layernorm_bwd_pair(const float* dy, const float* y1, const float* g2,
                                 const float* mean2, const float* rstd2, const float* gres,
                                 const float* x, const float* g1, const float* mean1,
                                 const float* rstd1, int64_t rows, int64_t d, float* dx,
                                 float* dg2, float* db2, float* dg1, float* db1, void* ws,
                                 size_t ws_bytes, float* dy2, float rscale, float p_drop,
                                 const uint64_t* rng, int64_t rng_offset, const int32_t* lens,
                                 int64_t T, void* table, int64_t slot2, int64_t slot1,
                                 void* stream);
OB_API size_t ob_ln_param_entry_bytes(void);
OB_API int ob_ln_param_table(const void* table, int64_t n, int64_t dmax, void* stream);

/*
 * Batched greedy CTC decode (inference path). Replaces onebit_asr/metrics.py:51-60
 * ctc_greedy_decode(logits[T, V], blank_id) called per utterance: for utterance b over its
 * first lens[b] frames, pred = argmax_v logits[b][t][v] (lowest index on ties, as
 * torch.argmax), emit pred[t] when pred[t] != blank and pred[t] != pred[t-1].
 *   logits [B][T][V] fp32; lens int64 [B] (device); ids int32 [B][T] workspace (the
 *   per-frame argmax, left for the caller); out int32 [B][T] (tokens first, -1 after);
 *   out_len int32 [B].
 */
OB_API int ob_ctc_greedy_decode(const float* logits, const int64_t* lens, int64_t B, int64_t T,
                                int64_t V, int blank, int32_t* ids, int32_t* out,
                                int32_t* out_len, void* stream);

/* ------------------------------------------------------------------------------------
 * Fused epilogues: the elementwise ops that follow a BitLinear GEMM at its call sites in
 * the reference, applied in the GEMM's store instead of separate torch kernels.
 * X / Y rows are P stacked passes as in ob_bitlinear_fwd_passes; pass_bits may be NULL
 * when P == 1 (codes2 is used). Element (row, col) of a [P*M][N] output has dropout index
 * row * N + col; keep = hash(seed, counter, index) >= p * 2^32, kept values scale by
 * 1 / (1 - p); rng is a DEVICE {seed, counter} int64[2] (required when p_drop > 0) and the
 * mask is drawn for counter + rng_offset (a per-call-site offset: no per-call device copy).
 * Outputs must not alias inputs.
 *
 * swish_drop   Y_pre = a X.Q^T + b;  Y_act = dropout(silu(Y_pre))
 *              (FeedForwardModule lin1 -> swish -> dropout, conformer.py:36-38)
 * residual     Y = R + rscale * rowvalid * dropout(a X.Q^T + b),
 *              rowvalid = (lens == NULL) || (row % T < lens[row / T])
 *              (lin2 -> dropout -> x + 0.5 h, conformer.py:39-45, rscale 0.5, lens NULL;
 *               out_proj -> dropout -> pad zero -> x + out, conformer.py:131-138, rscale 1)
 * bwd_dx_swish_drop
 *              dPre = (a dY.Q) * keep * scale * silu'(pre): the dX GEMM of lin2 chained
 *              through the dropout and swish backward of swish_drop (same rng, same p)
 * drop_scale_bwd
 *              dY = rscale * rowvalid * dropout(dOut) with the residual entry's mask:
 *              the gradient of `residual`'s output w.r.t. its GEMM output.
 * ------------------------------------------------------------------------------------ */
OB_API int ob_bitlinear_fwd_swish_drop(const float* X, int64_t P, int64_t M, int64_t K,
                                       const uint32_t* codes2, const uint32_t* codes1,
                                       const int32_t* pass_bits, const float* alpha,
                                       int alpha_raw, const float* bias, int64_t N, float p_drop,
                                       const uint64_t* rng, int64_t rng_offset, float* Y_pre,
                                       float* Y_act, void* stream);
OB_API int ob_bitlinear_fwd_residual(const float* X, int64_t P, int64_t M, int64_t K,
                                     const uint32_t* codes2, const uint32_t* codes1,
                                     const int32_t* pass_bits, const float* alpha, int alpha_raw,
                                     const float* bias, int64_t N, const float* R, float rscale,
                                     float p_drop, const uint64_t* rng, int64_t rng_offset,
                                     const int32_t* lens, int64_t T, float* Y, void* stream);
/* ob_bitlinear_fwd_residual whose epilogue also forms the LayerNorm(s) that read Y next
 * (conformer.py:19-24, nn.LayerNorm(d)): nln = 1: ln_y0 = LN0(Y) with its per-row mean / rstd
 * (the statistics ob_layernorm_bwd takes); nln = 2: also ln_y1 = LN1(ln_y0) (a block's final LN
 * and the next block's first, as ob_layernorm_fwd_pair). Same row arithmetic as the LN kernels
 * (bit-identical results). Taken for the K = 576 byte-image launch with N = 144 (the Conformer
 * FFN's second linear); otherwise OB_ERR_SHAPE with nothing launched (run
 * ob_bitlinear_fwd_residual and ob_layernorm_fwd[_pair]). X, R, Y, ln_y*, ln_w*, ln_b* 16-byte
 * aligned; rows of all outputs [P*M][N]. */
OB_API int ob_bitlinear_fwd_residual_ln(
    const float* X, int64_t P, int64_t M, int64_t K, const uint32_t* codes2,
    const uint32_t* codes1, const int32_t* pass_bits, const float* alpha, int alpha_raw,
    const float* bias, int64_t N, const float* R, float rscale, float p_drop, const uint64_t* rng,
    int64_t rng_offset, const int32_t* lens, int64_t T, float* Y, int nln, const float* ln_w0,
    const float* ln_b0, float eps0, float* ln_y0, float* ln_mean0, float* ln_rstd0,
    const float* ln_w1, const float* ln_b1, float eps1, float* ln_y1, float* ln_mean1,
    float* ln_rstd1, void* stream);
OB_API int ob_bitlinear_bwd_dx_swish_drop(const float* dY, int64_t P, int64_t M, int64_t N,
                                          const uint32_t* codes2_t, const uint32_t* codes1_t,
                                          const int32_t* pass_bits, const float* alpha,
                                          int alpha_raw, int64_t K, const float* pre,
                                          float p_drop, const uint64_t* rng, int64_t rng_offset,
                                          float* dPre, void* stream);
OB_API int ob_drop_scale_bwd(const float* dOut, int64_t rows, int64_t N, float rscale,
                             float p_drop, const uint64_t* rng, int64_t rng_offset,
                             const int32_t* lens, int64_t T, float* dY, void* stream);

/* out = R + rscale * rowvalid * dropout(Y) over [rows][N]: the residual/dropout tail of a
 * call site whose producer is not a BitLinear GEMM (the conv module's pw2, conformer.py:
 * 160-167), with the mask convention of the fused entries above. */
OB_API int ob_residual_drop_fwd(const float* R, const float* Y, int64_t rows, int64_t N,
                                float rscale, float p_drop, const uint64_t* rng,
                                int64_t rng_offset, const int32_t* lens, int64_t T, float* out,
                                void* stream);

/* Conv2dSubsampling's conv -> +bias -> ReLU tails (conformer.py:183-186), NCHW planes of
 * hw = H*W elements: fwd y = max(y + b[c], 0) in place; bwd g' = g * (y > 0) (torch's
 * threshold_backward on the ReLU output) and db[c] = sum over (b, h, w) of g'. */
OB_API int ob_bias_relu_fwd(float* y, const float* bias, int64_t B, int64_t C, int64_t hw,
                            void* stream);
OB_API size_t ob_relu_bias_bwd_workspace(int64_t B, int64_t C);
OB_API int ob_relu_bias_bwd(const float* g, const float* y, int64_t B, int64_t C, int64_t hw,
                            float* gout, float* dbias, void* ws, size_t ws_bytes, void* stream);
/* out[n] = sum over rows of x[rows][N], fixed order: the bias gradient of a GEMM on rows
 * (the conv module's pointwise convolutions, conformer.py:143,147). */
OB_API size_t ob_colsum_workspace(int64_t N);
OB_API int ob_colsum(const float* x, int64_t rows, int64_t N, float* out, void* ws,
                     size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------------------
 * Dense fp32 GEMMs of the conv module's pointwise Conv1d(kernel 1) layers
 * (conformer.py:143,147; replaces the fp32 matmuls / addmm of a 1x1 conv on channels-last
 * rows). Exact-fp32 products on the bf16 matrix cores (6 MFMAs per k-step, csrc/dgemm.hip).
 *   ob_dense_gemm: w_trans = 0: Y[M][N] = X[M][K] . W^T + bias, W [N][K] (the forward);
 *                  w_trans = 1: Y[M][N] = X[M][K] . W,          W [K][N] (dX = dY . W).
 *                  bias may be NULL. X, W, Y 16-byte aligned; K, N multiples of 4.
 *                  A K too long for the whole-K weight image (N <= 144) runs the K-chunked
 *                  form (round 6): the CTC head's input gradient, K = V = 5004, replacing the
 *                  library fp32 `g @ W` of the head's backward (losses.py:41-47 through
 *                  conformer.py:275).
 *   ob_dense_dw:   dW[N][K] = dY[M][N]^T . X[M][K], db[N] = column sums of dY (db may be
 *                  NULL); N, K multiples of 48. Deterministic (fixed-order chunk sums).
 * ob_dense_supported(K, N) / ob_dense_dw_workspace(M, N, K) == 0: the shape is not taken.
 * ------------------------------------------------------------------------------------ */
/* The property the int8 inference path's absmax launch relies on (round 6: max|silu| over a
 * lane's elements taken as silu(max y), csrc/tgemm_i8.hip): adds to *bad (a device uint32 the
 * caller zeroes) the count of fp32 bit patterns b in [lo_bits, hi_bits) with
 * fast_silu(float(b + 1)) < fast_silu(float(b)). Non-negative finite patterns only. */
OB_API int ob_silu_fast_monotone_check(uint32_t lo_bits, uint32_t hi_bits, uint32_t* bad,
                                       void* stream);
OB_API int ob_dense_supported(int64_t K, int64_t N);
OB_API int ob_dense_gemm(const float* X, int64_t M, int64_t K, const float* W, int w_trans,
                         const float* bias, int64_t N, float* Y, void* stream);
/* ob_dense_gemm (w_trans 0) with the residual tail of the conv module (conformer.py:160-167,
 * x + dropout(pw2(.))) in the epilogue: Y = R + dropout(X W^T + bias), R [M][N]; the dropout
 * is ob_residual_drop_fwd's (hash on the flat index row * N + col with rng / rng_offset, rscale
 * 1, no row mask), so Y equals ob_dense_gemm followed by ob_residual_drop_fwd bit for bit. */
OB_API int ob_dense_gemm_residual_drop(const float* X, int64_t M, int64_t K, const float* W,
                                       const float* bias, int64_t N, const float* R,
                                       float p_drop, const int64_t* rng, int64_t rng_offset,
                                       float* Y, void* stream);
OB_API size_t ob_dense_dw_workspace(int64_t M, int64_t N, int64_t K);
OB_API int ob_dense_dw(const float* dY, const float* X, int64_t M, int64_t N, int64_t K,
                       float* dW, float* db, void* ws, size_t ws_bytes, void* stream);
/* ob_dense_dw with the finish deferred to ob_dw_finish_table (same table and contract as
 * ob_bitlinear_bwd_dw_passes_defer; dense weights carry no STE mask / alpha). */
OB_API int ob_dense_dw_defer(const float* dY, const float* X, int64_t M, int64_t N, int64_t K,
                             float* dW, float* db, void* ws, size_t ws_bytes, void* table,
                             int64_t slot, int64_t start, int64_t* n_blocks, void* stream);

/* ------------------------------------------------------------------------------------
 * Conv module core (ConvModule, conformer.py:139-167; full precision), channels-last.
 * Rows = Bt*T frames (utterance b = rows [b*T, (b+1)*T)), channel fastest; P stacked
 * passes (Bt = P*B) keep per-pass BatchNorm statistics. pw1 / pw2 are plain GEMMs left to
 * the caller; between them:
 *   fwd: u [rows][2C] -> g = u[:, :C] * sigmoid(u[:, C:])      (GLU over channels, :156)
 *        z = depthwise_K(g) + b_dw   (zero padding K/2 at utterance edges, :157)
 *        stats[p][c] = {mean, rstd} of z over pass p's B*T frames (batch statistics,
 *        padded frames included, biased variance, eps; :158)
 *        v = swish(gamma * (z - mean) * rstd + beta)               (:159)
 *        g [rows][C] (the GLU output) is kept for the backward.
 *   bwd: from dv = dL/dv: du [rows][2C], dw_dw [C][K], db_dw [C], dgamma [C], dbeta [C]
 *        (weight gradients summed over passes). u, z, g, stats are the forward's.
 * K odd; ob_convmod_workspace() == 0 means the shape is not supported (C too wide for the
 * LDS tile). Deterministic (fixed-order reductions, fp64 statistics).
 * ------------------------------------------------------------------------------------ */
OB_API size_t ob_convmod_workspace(int64_t P, int64_t Bt, int64_t T, int64_t C, int64_t K);
OB_API int ob_convmod_fwd(const float* u, const float* w_dw, const float* b_dw,
                          const float* gamma, const float* beta, int64_t P, int64_t Bt,
                          int64_t T, int64_t C, int64_t K, float eps, float* z, float* g,
                          float* stats, float* v, void* ws, size_t ws_bytes, void* stream);
OB_API int ob_convmod_bwd(const float* dv, const float* u, const float* z, const float* g,
                          const float* stats, const float* w_dw, const float* gamma,
                          const float* beta, int64_t P, int64_t Bt, int64_t T, int64_t C,
                          int64_t K, float* du, float* dw_dw, float* db_dw, float* dgamma,
                          float* dbeta, void* ws, size_t ws_bytes, void* stream);
/* ob_convmod_bwd with the depthwise weight-gradient finish (dw_dw, db_dw: the fixed-order
 * sum of the per-tile partials) deferred when table != NULL and the shape runs on the
 * channel-split tiles: the backward launch writes the partials' descriptor into slot `slot`
 * of a caller-owned device table of ob_cm_wgrad_entry_bytes() entries, *deferred = 1, and
 * ob_cm_wgrad_table finishes entries 0 .. n-1 in one launch (nmax = the largest C * (K + 1))
 * with the same arithmetic. ws stays allocated until then. *deferred = 0: finished now. */
OB_API int ob_convmod_bwd_defer(const float* dv, const float* u, const float* z, const float* g,
                                const float* stats, const float* w_dw, const float* gamma,
                                const float* beta, int64_t P, int64_t Bt, int64_t T, int64_t C,
                                int64_t K, float* du, float* dw_dw, float* db_dw, float* dgamma,
                                float* dbeta, void* ws, size_t ws_bytes, void* table, int64_t slot,
                                int64_t* deferred, void* stream);
OB_API size_t ob_cm_wgrad_entry_bytes(void);
OB_API int ob_cm_wgrad_table(const void* table, int64_t n, int64_t nmax, void* stream);

/* ------------------------------------------------------------------------------------
 * Conv2dSubsampling's two convolutions (conformer.py:170-208: Conv2d(1, C, 3, 2) -> ReLU ->
 * Conv2d(C, C, 3, 2) -> ReLU; replaces the torch.nn.Conv2d / cuDNN calls the module makes),
 * channels-last so the flatten + Linear that follows needs no transpose:
 *   X  [B][T][F] feats;  W0 [C][1][3][3], b0 [C];  W2 [C][C][3][3], b2 [C] (torch layouts)
 *   Y1 [B][T1][F1][C] = relu(conv(X, W0) + b0),  T1 = (T-3)/2+1, F1 = (F-3)/2+1
 *   Y2 [B][T2][F2][C] = relu(conv(Y1, W2) + b2), T2 = (T1-3)/2+1, F2 = (F1-3)/2+1
 * ob_subsample_pack re-splits W2 into the bf16 hi/mid/lo images the fp32-exact MFMA
 * GEMMs read (call it whenever W2 changes; ob_subsample_image_bytes(C) bytes, 16-aligned).
 * bwd: from dY2 = dL/dY2 (before the ReLU mask) and the forward's X, W0, b0, Y1, Y2: dW0,
 * db0, dW2, db2 (overwritten; dX is not produced: the feats need no gradient). Deterministic; C in {48, 64, 96, 144},
 * T, F >= 7; ob_subsample_bwd_workspace() == 0 means unsupported.
 * ------------------------------------------------------------------------------------ */
OB_API size_t ob_subsample_image_bytes(int64_t C);
OB_API int ob_subsample_pack(const float* W2, int64_t C, void* img, void* stream);
OB_API int ob_subsample_fwd(const float* X, int64_t B, int64_t T, int64_t F, int64_t C,
                            const float* W0, const float* b0, const void* img,
                            const float* b2, float* Y1, float* Y2, void* stream);
OB_API size_t ob_subsample_bwd_workspace(int64_t B, int64_t T, int64_t F, int64_t C);
OB_API int ob_subsample_bwd(const float* X, const float* W0, const float* b0, const float* Y1,
                            const float* Y2, const float* dY2, int64_t B, int64_t T, int64_t F,
                            int64_t C, const void* img,
                            float* dW0, float* db0, float* dW2, float* db2, void* ws,
                            size_t ws_bytes, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* ONEBIT_HIP_H_ */
