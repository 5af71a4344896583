// ob_launch.h — internal (C++) launchers behind the C ABI in capi.hip.
// Arguments are validated by capi.hip before any of these is called.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/onebit_hip.h"

namespace ob {

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// quant.hip
// bits_dev (may be NULL): when set, the bitwidth is read on device (graph mode).
void launch_quant_pack(const float* W, const float* alpha, int alpha_raw, int bits,
                       const int* bits_dev, int64_t N, int64_t K, uint32_t* codes,
                       uint32_t* codes_t, hipStream_t s);
// Grouped pack (ob_pack_item from include/onebit_hip.h; table on device).
int64_t quant_pack_item_blocks(int64_t N, int64_t K);
int64_t quant_pack_item_blocks16(int64_t N, int64_t K);  // a bits == 16 (bf16 image) item
void launch_quant_pack_group(const ob_pack_item* items_dev, int n_items, int64_t total_blocks,
                             hipStream_t s);
void launch_quant_dequant(const float* W, const float* alpha, int alpha_raw, int bits, int64_t n,
                          float* W_hat, hipStream_t s);

// Split-reduction finish shared by both backward entries (one launch): sums `chunks` fp32
// slabs of length nk (+ an optional [chunks][n_db] bias slab), applies the STE mask, writes
// dW, and the last-arriving block sums the per-block alpha partials into dalpha.
// `apart` must hold ste_reduce_blocks(nk + n_db) floats; *ticket must be 0 on entry (it is
// 0 again on exit).
int64_t ste_reduce_blocks(int64_t total);
void launch_ste_reduce(const float* part, int chunks, int64_t nk, const float* part_db,
                       int64_t n_db, const float* W, const float* alpha, int alpha_raw, int bits,
                       const int* bits_dev, float* dW, float* db, float* apart, uint32_t* ticket,
                       float* dalpha, hipStream_t s);
// Stacked passes: chunks = P * cpp, chunk c of pass c / cpp; pass p's STE/alpha term uses
// bitwidth pass_bits[p] (DEVICE int32 [P], 1 or 2). P <= kMaxPasses.
constexpr int kMaxPasses = 4;
void launch_ste_reduce_passes(const float* part, int P, int cpp, int64_t nk, const float* part_db,
                              int64_t n_db, const float* W, const float* alpha, int alpha_raw,
                              const int* pass_bits, float* dW, float* db, float* apart,
                              uint32_t* ticket, float* dalpha, hipStream_t s);

// gemm.hip
// C[M][N] = a * (A[M][K] . Q^T) + bias, Q given as 2-bit codes [N][ceil(K/16)].
// the VALU sign-accumulate form of the forward (tgemm_va.hip; the north-star inner-product
// A/B, not on the product path): false for K % 4 != 0
bool launch_ternary_gemm_signacc(const float* A, int64_t M, int64_t K, const uint32_t* codes,
                                 int64_t N, const float* alpha, int alpha_raw, const float* bias,
                                 float* C, hipStream_t s);
void launch_ternary_gemm(const float* A, int64_t M, int64_t K, const uint32_t* codes, int64_t N,
                         const float* alpha, int alpha_raw, const float* bias, float* C,
                         hipStream_t s);

// P stacked passes of one layer (rows p*M .. p*M+M of A and C): pass p multiplies by the
// codes1 operand when pass_bits[p] (DEVICE int32 [P]) == 1, else by `codes`.
// `ep` (optional) fuses the elementwise ops that follow the GEMM at its call sites into
// the store; see TgemmEpi.
struct TgemmEpi;
void launch_ternary_gemm_passes(const float* A, int P, int64_t M, int64_t K,
                                const uint32_t* codes, const uint32_t* codes1,
                                const int* pass_bits, int64_t N, const float* alpha,
                                int alpha_raw, const float* bias, float* C, hipStream_t s,
                                const TgemmEpi* ep = nullptr);
// G <= 3 layers sharing A (same K, N) in one launch (each layer's codes / alpha / bias / C);
// false: shape refused
bool launch_ternary_gemm_passes_group(const float* A, int P, int64_t M, int64_t K, int G,
                                      const uint32_t* const* codes,
                                      const uint32_t* const* codes1, const int* pass_bits,
                                      int64_t N, const float* const* alpha, int alpha_raw,
                                      const float* const* bias, float* const* C, hipStream_t s);
// dX = sum_g alpha_g dY_g . Q_g^T over G = 3 sources of width N = 144 (the q / k / v input
// gradients of one LayerNorm output) in one launch; codes_t / codes_t1: the sources' dX code
// images (2-bit / 1-bit), per-pass bitwidths from pass_bits. false: shape not taken (the
// caller runs one dX launch per source).
bool launch_ternary_dx_sum(int G, const float* const* dY, int P, int64_t M, int64_t N,
                           const uint32_t* const* codes_t, const uint32_t* const* codes_t1,
                           const int* pass_bits, const float* const* alpha, int alpha_raw,
                           int64_t K, float* dX, hipStream_t s);

// Fused epilogues of the ternary GEMM, y = a * acc + bias; element (row, col) of the
// P*M x N output has dropout index row * N + col (ob_drop.h):
//   kEpiSwishDrop    C2 = y;  C = drop(silu(y))                 (FFN lin1 -> swish -> dropout,
//                                                                 conformer.py:36-38)
//   kEpiResidual     C = R + rscale * rowvalid * drop(y)          (lin2 -> dropout -> x + 0.5*h,
//                                                                 conformer.py:39-45; out_proj ->
//                                                                 dropout -> pad zero -> x + out,
//                                                                 :131-138)
//   kEpiSwishDropBwd C = y * keep * scale * silu'(R), R = the forward's pre-activation
//                                                                (dX of lin2 chained through the
//                                                                 dropout and swish backward)
// rowvalid = (lens == NULL) || (row % T < lens[row / T]).
enum { kEpiNone = 0, kEpiSwishDrop = 1, kEpiResidual = 2, kEpiSwishDropBwd = 3 };
struct TgemmEpi {
  int mode;
  const float* R;
  float* C2;
  float rscale;
  const int* lens;
  int T;
  float p_drop;
  const uint64_t* rng;  // device {seed, counter}; required when p_drop > 0
  uint64_t rng_off;     // added to the counter (per call site)
  // residual epilogue only (N == 144, K = 576 byte path): nln LayerNorms of the produced
  // rows, ln 1 normalising ln 0's output (the block-final LN and the next block's first)
  int nln;
  const float* lng[2];
  const float* lnb[2];
  float lneps[2];
  float* lny[2];
  float* lnmean[2];
  float* lnrstd[2];
};
// the residual epilogue can normalise its rows (TgemmEpi::nln): the byte-image K = 576 launch
bool ternary_residual_ln_supported(int64_t K, int64_t N, int alpha_raw);

// out = R + rscale * rowvalid * drop(Y) over [rows][N] (forward twin of drop_scale_bwd).
void launch_residual_drop_fwd(const float* R, const float* Y, int64_t rows, int64_t N,
                              float rscale, float p_drop, const uint64_t* rng, uint64_t rng_off,
                              const int* lens, int T, float* out, hipStream_t s);

// Subsampling conv tails (NCHW planes of hw elements): y = relu(y + b[c]) in place; and
// g' = g * (y > 0), db[c] = sum over planes of channel c (ws: relu_bias_bwd_workspace).
void launch_bias_relu_fwd(float* y, const float* bias, int64_t B, int64_t C, int64_t hw,
                          hipStream_t s);
size_t relu_bias_bwd_workspace(int64_t B, int64_t C);
void launch_relu_bias_bwd(const float* g, const float* y, int64_t B, int64_t C, int64_t hw,
                          float* gout, float* dbias, void* ws, hipStream_t s);
// p[0 .. n_words) = 0 as a kernel (graph-safe; see fused.hip).
void launch_zero_words(void* p, int64_t n_words, hipStream_t s);
// out[n] = sum over rows of x[rows][N] (fixed order; ws: colsum_workspace(N)).
size_t colsum_workspace(int64_t N);
void launch_colsum(const float* x, int64_t rows, int64_t N, float* out, void* ws, hipStream_t s);

// decattn.hip (the decoder's attention core; see the file header)
bool decattn_supported(int64_t Lq, int64_t Lk, int64_t dh);
void launch_decattn_fwd(const float* q, int64_t sq, const float* k, int64_t sk, const float* v,
                        int64_t sv, const uint8_t* kmask, int causal, int64_t B, int64_t H,
                        int64_t Lq, int64_t Lk, int64_t dh, float p_drop, const uint64_t* rng,
                        uint64_t rng_off, float* probs, float* ctx, hipStream_t s);
void launch_decattn_bwd(const float* dctx, const float* ctxo, const float* q, int64_t sq,
                        const float* k, int64_t sk, const float* v, int64_t sv, int64_t B, int64_t H, int64_t Lq, int64_t Lk,
                        int64_t dh, float p_drop, float* probs, float* dq, int64_t gq,
                        float* dk, int64_t gk, float* dv, int64_t gv, hipStream_t s);

// convmod.hip (conv module core, channels-last; see the file header)
bool convmod_supported(int64_t C, int64_t K);
size_t convmod_workspace(int64_t P, int64_t Bt, int64_t T, int64_t C, int64_t K);
void launch_convmod_fwd(const float* u, const float* wdw, const float* bdw, const float* gamma,
                        const float* beta, int64_t P, int64_t Bt, int64_t T, int64_t C, int64_t K,
                        float eps, float* z, float* g, float* stats, float* v, void* ws,
                        hipStream_t s);
// Deferred depthwise weight-gradient finish: the channel-tile backward (block 0) writes the
// partials' descriptor into table[slot]; launch_cm_wgrad_table finishes every entry in one
// launch (nmax = the largest C * (K + 1)).
struct CmWgradEntry {
  const float* wpart;
  float* dw;
  float* db;
  int nblk;
  int C;
  int K;
};
struct CmDefer {
  CmWgradEntry* table;  // nullptr: finish now
  int slot;
};
void launch_convmod_bwd(const float* dv, const float* u, const float* z, const float* g,
                        const float* stats, const float* wdw, const float* gamma,
                        const float* beta, int64_t P, int64_t Bt, int64_t T, int64_t C, int64_t K,
                        float* du, float* dwdw, float* dbdw, float* dgamma, float* dbeta, void* ws,
                        hipStream_t s, const CmDefer* defer = nullptr);
// true when launch_convmod_bwd can defer its weight-gradient finish at this shape
bool convmod_bwd_deferrable(int64_t C, int64_t K);
void launch_cm_wgrad_table(const CmWgradEntry* table, int n, int nmax, hipStream_t s);

// dY = rscale * rowvalid * drop(dOut) over [rows][N] (the backward of kEpiResidual's
// dropout / pad / scale, same keep mask).
void launch_drop_scale_bwd(const float* dout, int64_t rows, int64_t N, float rscale,
                           float p_drop, const uint64_t* rng, uint64_t rng_off, const int* lens,
                           int T, float* dy, hipStream_t s);

// Split-M partial of G = dY^T . X: part[c][N*K] for chunk c, part_db[c][N] (optional).
// With P stacked passes the chunks never straddle a pass: chunk c belongs to pass
// c / chunks_per_pass (so the reduction can weight each pass by its own bitwidth).
struct DwPlan {
  int64_t tiles_n, tiles_k, chunks, rows_per_chunk;
  int64_t passes, rows_per_pass, chunks_per_pass;
  int variant;  // 0: fp32 MFMA (OB_GEMM=f32); 4: bf16x6 with 64-wide tiles
};
DwPlan plan_dw(int64_t M, int64_t N, int64_t K);
DwPlan plan_dw_passes(int64_t P, int64_t M_per_pass, int64_t N, int64_t K);
// Alpha-gradient inputs of the LDS dW path (variant >= 9): each dW block writes its share
// of sum_e G[e] term[e] (at its pass's bitwidth) to apart[logical block].
struct DwAlpha {
  const float* W;
  const float* alpha;
  int alpha_raw;
  int bits;               // one pass: bitwidth, or read from bits_dev when set
  const int* bits_dev;
  const int* pass_bits;   // stacked passes: DEVICE int32 [P]
  float* apart;           // [tiles * chunks]
};
// Variants < 9 also zero *ticket (for the ste_reduce launch that follows on the same
// stream); variants >= 9 need `al` and are finished by launch_dw_finish.
void launch_dw_partial(const float* dY, const float* X, int64_t M, int64_t N, int64_t K,
                       const DwPlan& p, float* part, float* part_db, uint32_t* ticket,
                       hipStream_t s, const DwAlpha* al = nullptr);
// G layers sharing X (G <= kMaxDwGroup), LDS path only: p = plan_dw_passes(P, M, G * N, K)
// (its tiles_n counts all G layers' n-tiles); per layer i the single-layer outputs
// part[i] / part_db[i] / al[i].apart (alpha partial index chunk * tiles_of_one_layer + tile).
void launch_dw_partial_group(const float* const* dY, int G, const float* X, int64_t M,
                             int64_t N, int64_t K, const DwPlan& p, float* const* part,
                             float* const* part_db, const DwAlpha* al, hipStream_t s);
void launch_dw_finish(const float* part, int chunks, int64_t nk, const float* part_db,
                      int64_t n_db, const float* W, const float* alpha, int alpha_raw,
                      const float* apart, int n_apart, float* dW, float* db, float* dalpha,
                      hipStream_t s);

// The finish of one LDS-path dW (arguments of launch_dw_finish); a group of up to
// kMaxDwGroup of them runs as one launch (block ranges per layer, same arithmetic).
struct DwFinish {
  const float* part;
  int chunks;
  int64_t nk;
  const float* part_db;
  int64_t n_db;
  const float* W;
  const float* alpha;
  int alpha_raw;
  const float* apart;
  int n_apart;
  float* dW;
  float* db;
  float* dalpha;
};
constexpr int kMaxDwGroup = 3;
void launch_dw_finish_group(const DwFinish* a, int n, hipStream_t s);

// Deferred finishes (one launch for every layer of a backward): the dW partial launch writes
// its layers' finish descriptors into a device table (block 0, from its arguments); the table
// kernel later runs every entry's finish -- entry i owns finish blocks [start, next start).
struct DwFinishEntry {
  DwFinish f;
  int64_t start;
};
int64_t dw_finish_blocks(const DwFinish& a);
void launch_dw_table_entry(DwFinishEntry* table, int slot, const DwFinishEntry& ent, hipStream_t s);
void launch_dw_finish_table(const DwFinishEntry* table, int n, int64_t total_blocks, hipStream_t s);
// launch_dw_partial_group with the finish deferred: ent[i] (start filled in) is written to
// table[slot + i] by the partial launch itself
void launch_dw_partial_group_defer(const float* const* dY, int G, const float* X, int64_t M,
                                   int64_t N, int64_t K, const DwPlan& p, float* const* part,
                                   float* const* part_db, const DwAlpha* al,
                                   DwFinishEntry* table, int slot, const DwFinishEntry* ent,
                                   hipStream_t s);

// Grouped deferred dW (dw.hip, ob_dw_grouped): one descriptor per weight gradient; the host
// fills the work-space fields (work0 .. tile0) and the launcher copies the table to the device.
struct DwgDesc {
  const float* dY;
  const float* X;
  const float* W;  // nullptr: dense
  const float* alpha;
  const int* pass_bits;
  float* dW;
  float* db;
  float* dalpha;
  int64_t work0;  // first linear step (32 rows of one 144 x 144 tile) of this gemm
  int N, K, Mp, P, alpha_raw, bits;
  int spp;      // 32-row steps per pass
  int tiles_k;  // K / 144
  int tiles;    // (N / 144) * tiles_k
  int tile0;    // first tile index (tile tickets, tile alpha slots)
};
constexpr int kDwgTile = 144;
int dwg_blocks(int64_t total_steps);  // one block per CU (at most total_steps)
size_t dwg_slot_bytes();              // one partial slab (tile + db + alpha)
// table: device [G] descriptors; slots: 2 * blocks slabs; talpha: [total tiles] floats;
// tickets: [total tiles + G] zeroed words (left zero)
void launch_dw_grouped(const DwgDesc* host_descs, int G, int64_t total_steps, int blocks,
                       DwgDesc* table, float* slots, float* talpha, uint32_t* tickets,
                       int total_tiles, hipStream_t s);

// dgemm.hip (dense exact-fp32 GEMM of the pointwise convs): false = shape not taken
bool dense_gemm_supported(int64_t K, int64_t N);
// Optional residual epilogue: C = R + dropout(A W^T + b) (R [M][N], the flat index
// row * N + col keying the dropout hash: residual_drop_fwd's arithmetic, element for element)
struct DenseEpi {
  const float* R;  // nullptr: plain C = A W^T + b
  float p_drop;
  const uint64_t* rng;
  uint64_t rng_off;
};
bool launch_dense_gemm(const float* A, int64_t M, int64_t K, const float* W, int trans,
                       const float* bias, int64_t N, float* C, hipStream_t s,
                       const DenseEpi* epi = nullptr);

// tgemm_i8.hip (opt-in absmax-int8 activations x ternary codes on the i8 matrix cores)
bool ternary_gemm_i8_supported(int64_t K, int64_t N);
// violations of fast_silu(next float) >= fast_silu(x) over bit patterns [lo, hi), added to *bad
void launch_silu_monotone_check(uint32_t lo, uint32_t hi, uint32_t* bad, hipStream_t s);
size_t act_absmax_workspace(int P);
void launch_act_absmax(const float* X, int P, int64_t n_per_pass, float* amax, void* ws,
                       hipStream_t s);
void launch_act_dequant(const float* X, int P, int64_t n_per_pass, const float* amax, float* Xd,
                        hipStream_t s);
bool launch_ternary_gemm_i8(const float* A, int P, int64_t M, int64_t K, const uint32_t* codes,
                            const uint32_t* codes1, const int* pass_bits, int64_t N,
                            const float* alpha, int alpha_raw, const float* amax,
                            const float* bias, float* C, hipStream_t s);

// decode.hip (batched greedy CTC decode: argmax per frame, collapse per utterance)
void launch_ctc_greedy(const float* logits, const int64_t* lens, int64_t B, int64_t T, int64_t V,
                       int blank, int* ids, int* out, int* out_len, hipStream_t s);

// fused epilogue (mode 1: C = silu(y), per-pass max|C| into amax_out (zeroed here);
// mode 2: C = R + rscale * (valid ? y : 0*y) with lens / T row validity); N % 4 == 0
bool launch_ternary_gemm_i8_epi(const float* A, int P, int64_t M, int64_t K,
                                const uint32_t* codes, const uint32_t* codes1,
                                const int* pass_bits, int64_t N, const float* alpha,
                                int alpha_raw, const float* amax, const float* bias, float* C,
                                int mode, const float* R, float rscale, const int* lens, int64_t T,
                                float* amax_out, hipStream_t s);
// int8 operand Aq [P*M][K] (quantised by its producer at amax's scale); mode 0 plain / 2
// residual (C fp32), mode 3: silu(y) quantised to int8 at its own per-pass absmax (C int8,
// amax_out = that absmax; two launches)
bool launch_ternary_gemm_i8q(const int8_t* Aq, int P, int64_t M, int64_t K,
                             const uint32_t* codes, const uint32_t* codes1, const int* pass_bits,
                             int64_t N, const float* alpha, int alpha_raw, const float* amax,
                             const float* bias, void* C, int mode, const float* R, float rscale,
                             const int* lens, int64_t T, float* amax_out, hipStream_t s);

// layernorm.hip (LayerNorm over the last dim, d <= 512; deterministic dgamma/dbeta)
bool layernorm_supported(int64_t d);
size_t layernorm_bwd_workspace(int64_t rows, int64_t d);
void launch_layernorm_fwd(const float* x, const float* gamma, const float* beta, int64_t rows,
                          int64_t d, float eps, float* y, float* mean, float* rstd, hipStream_t s);
// y1 = LN1(x), y2 = LN2(y1) in one pass (bit-identical to two launch_layernorm_fwd)
void launch_layernorm_fwd_pair(const float* x, const float* g1, const float* b1, const float* g2,
                               const float* b2, int64_t rows, int64_t d, float eps1, float eps2,
                               float* y1, float* mean1, float* rstd1, float* y2, float* mean2,
                               float* rstd2, hipStream_t s);
// + per-pass max|y| into amax[P] (rows % P == 0, P <= 8; per-block partials in ws)
size_t layernorm_fwd_amax_workspace(int64_t P);
void launch_layernorm_fwd_amax(const float* x, const float* gamma, const float* beta,
                               int64_t rows, int64_t d, float eps, float* y, float* mean,
                               float* rstd, int P, float* amax, void* ws, hipStream_t s);
// the int8 image of LN(x) at its per-pass absmax scale (absmax pass, then LN again + quantise;
// ws as launch_layernorm_fwd_amax; yq 4-byte aligned)
void launch_layernorm_fwd_i8(const float* x, const float* gamma, const float* beta, int64_t rows,
                             int64_t d, float eps, int P, float* amax, int8_t* yq, void* ws,
                             hipStream_t s);
// Optional second output of the backward: dy2 = rscale * rowvalid * drop(dx) (the residual
// dropout backward of the module whose output this LN normalises; lens/T as TgemmEpi).
struct LnGradScale {
  float* dy2;
  float rscale;
  float p_drop;
  const uint64_t* rng;
  uint64_t rng_off;
  const int* lens;
  int T;
};
// Deferred LN parameter reduction: ln_bwd (block 0) writes its partials' descriptor into
// table[slot]; launch_ln_param_table reduces every entry in one launch (dmax = max d).
struct LnParamEntry {
  const float* part_g;
  const float* part_b;
  float* dgamma;
  float* dbeta;
  int nblk;
  int d;
};
struct LnDefer {
  LnParamEntry* table;  // nullptr: reduce now
  int slot;
};
void launch_ln_param_table(const LnParamEntry* table, int n, int dmax, hipStream_t s);
void launch_layernorm_bwd(const float* dy, const float* x, const float* gamma, const float* mean,
                          const float* rstd, int64_t rows, int64_t d, const float* dres, float* dx, float* dgamma,
                          float* dbeta, void* ws, hipStream_t s, const LnGradScale* gsc = nullptr,
                          const LnDefer* defer = nullptr);
// backward of y1 = LN1(x), y2 = LN2(y1) with y1's residual-branch gradient gres (may be null):
// dx = LN1_bwd(LN2_bwd(dy) + gres); ws = 2 * layernorm_bwd_workspace(rows, d) bytes (LN2's
// partials, then LN1's); gsc: the dy2 of the tail feeding x; defer2 / defer1 per layer.
void launch_layernorm_bwd_pair(const float* dy, const float* y1, const float* g2,
                               const float* mean2, const float* rstd2, const float* gres,
                               const float* x, const float* g1, const float* mean1,
                               const float* rstd1, int64_t rows, int64_t d, float* dx,
                               float* dg2, float* db2, float* dg1, float* db1, void* ws,
                               hipStream_t s, const LnGradScale* gsc, const LnDefer* defer2,
                               const LnDefer* defer1);

// dwconv.hip (depthwise Conv1d of the conv module, odd kernel width, 'same' padding)
bool dwconv_supported(int KT);
void launch_dwconv_fwd(const float* x, const float* w, const float* bias, int64_t B, int64_t C,
                       int64_t T, int64_t KT, float* y, hipStream_t s);
size_t dwconv_bwd_workspace(int64_t B, int64_t C, int64_t KT);
void launch_dwconv_bwd(const float* x, const float* dy, const float* w, int64_t B, int64_t C,
                       int64_t T, int64_t KT, float* dx, float* dw, float* db, float* part,
                       hipStream_t s);

// ctc.hip (CTC loss with device-side lengths; log_probs [B][T][V])
size_t ctc_workspace(int64_t B, int64_t T, int64_t S);
bool ctc_supported(int64_t S);
void launch_ctc_fwd(const float* lp, const int64_t* targets, const int64_t* in_len,
                    const int64_t* tg_len, int64_t B, int64_t T, int64_t V, int64_t S, int blank, int64_t G,
                    float* loss, float* ws, hipStream_t s);
void launch_ctc_bwd(const float* lp, const int64_t* targets, const int64_t* in_len,
                    const int64_t* tg_len, int64_t B, int64_t T, int64_t V, int64_t S, int blank, int64_t G,
                    const float* grad_out, float* grad, float* ws, hipStream_t s);
// CTC from the head's logits x [B][T][V] (no log_softmax tensor): forward = lse pass +
// alpha + reduce; backward = beta + reduce + dense softmax gradient with label fix-up.
size_t ctc_logits_workspace_bytes(int64_t B, int64_t T, int64_t S);
void launch_ctc_logits_fwd(const float* x, const int64_t* targets, const int64_t* in_len,
                           const int64_t* tg_len, int64_t B, int64_t T, int64_t V, int64_t S,
                           int blank, int64_t G, float* loss, void* ws, hipStream_t s);
void launch_ctc_logits_bwd(const float* x, const int64_t* targets, const int64_t* in_len,
                           const int64_t* tg_len, int64_t B, int64_t T, int64_t V, int64_t S,
                           int blank, int64_t G, const float* grad_out, float* grad, void* ws,
                           hipStream_t s);

// seqloss.hip: label-smoothed attention CE + KL(teacher || student) over the stacked decoder
// logits x [P*BU][V] (pass-major; the teacher's row of position q is row q).
bool att_kl_supported(int64_t V);
size_t att_kl_workspace(int64_t P, int64_t BU);
void launch_att_kl_fwd(const float* x, const int64_t* tgt, const uint8_t* pad, int64_t P,
                       int64_t BU, int64_t V, int pad_id, float ls, float* l_att, float* l_kl,
                       void* ws, hipStream_t s);
void launch_att_kl_bwd(const float* x, const int64_t* tgt, const uint8_t* pad, int64_t P,
                       int64_t BU, int64_t V, float ls, const float* g_att, const float* g_kl,
                       float* grad, const void* ws, hipStream_t s);
// the step's loss from its per-pass parts (P = 3): loss [1], parts [8]; and its backward
void launch_loss_combine_fwd(const float* l_att, const float* l_ctc, const float* l_kl,
                             float gamma, float lam1, float lam2, float* loss, float* parts,
                             hipStream_t s);
void launch_loss_combine_bwd(const float* gl, float gamma, float lam1, float lam2, float* d_att,
                             float* d_ctc, float* d_kl, hipStream_t s);

// adamw.hip (clip_grad_norm_ + AdamW over a tensor table; layout = ob_adamw_tensor)
struct AdamwTensor {
  float* param;
  const float* grad;
  float* exp_avg;
  float* exp_avg_sq;
  int64_t numel;
};
int64_t adamw_plan(const int64_t* numels, int64_t n, int64_t* map);
size_t adamw_workspace(int64_t n_blocks);
void launch_adamw(const AdamwTensor* tab, const int64_t* map, int64_t nb, const float* lr,
                  float* step, float grad_scale, double beta1, double beta2, double eps,
                  double weight_decay, double max_norm, float* total_norm_out, void* ws,
                  hipStream_t s);

// embed.hip (deterministic token-embedding backward; pad < 0: no padding row)
bool embed_supported(int64_t C);
void launch_embed_bwd(const int64_t* idx, int64_t N, const float* g, int64_t C, int64_t V,
                      int64_t pad, float* dW, hipStream_t s);

// relattn.hip (fused relative-position attention core of MHSA)
bool relattn_supported(int64_t T, int64_t d);
size_t relattn_bwd_workspace(int64_t Bt, int64_t T, int64_t H, int64_t d);
int64_t relattn_probs_elems(int64_t Bt, int64_t T, int64_t H);
int64_t relattn_saved_elems(int64_t Bt, int64_t T, int64_t H, int64_t d);
int relattn_set_flash(int on);  // 0 / 1 sets the process-wide backward mode; returns the previous
void launch_relattn_fwd(const float* q, const float* k, const float* v, const float* pos,
                        const float* u, const float* vb, const int* lens, int64_t Bt, int64_t P,
                        int64_t T, int64_t H, int64_t d, float p_drop, const uint64_t* rng,
                        uint64_t rng_off, float* saved, float* probs, float* ctx, hipStream_t s);
void launch_relattn_bwd(const float* dctx, const float* ctx, const float* q, const float* k,
                        const float* v, const float* pos, const float* u, const float* vb,
                        const int* lens, int64_t Bt, int64_t P, int64_t T, int64_t H, int64_t d,
                        float p_drop, const float* saved, float* dq, float* dk, float* dv,
                        float* dpos, float* du, float* dvb, void* ws, hipStream_t s);
void launch_relattn_dropout_mask(int64_t n, int64_t T, float p_drop, const uint64_t* rng,
                                 uint64_t rng_off, uint8_t* out, hipStream_t s);

// subsample.hip (Conv2dSubsampling, channels-last implicit GEMMs)
bool subsample_supported(int64_t T, int64_t F, int64_t C);
size_t subsample_image_bytes(int64_t C);
void launch_subsample_pack(const float* W2, int64_t C, void* img, hipStream_t s);
void launch_subsample_fwd(const float* X, int64_t B, int64_t T, int64_t F, int64_t C,
                          const float* W0, const float* b0, const void* img, const float* b2,
                          float* Y1, float* Y2, hipStream_t s);
size_t subsample_bwd_workspace(int64_t B, int64_t T, int64_t F, int64_t C);
void launch_subsample_bwd(const float* X, const float* W0, const float* b0, const float* Y1,
                          const float* Y2, const float* dY2, int64_t B, int64_t T, int64_t F,
                          int64_t C, const void* img,
                          float* dW0, float* db0, float* dW2, float* db2, void* ws,
                          hipStream_t s);

}  // namespace ob
