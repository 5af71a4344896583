// capi.hip — the C ABI declared in include/onebit_hip.h: argument validation, workspace
// carving and launch-error reporting around the launchers in quant.hip / gemm.hip.
#include <algorithm>
#include <vector>

#include "../../include/onebit_hip.h"
#include "ob_launch.h"
#include <stdint.h>

using namespace ob;

namespace {

constexpr int kAbiVersion = 4;  // 4 (round 6): ob_decattn_bwd consumes probs (dS' written there)

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline bool aligned4(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 3) == 0; }

inline int check_bits(int bits) { return (bits == 1 || bits == 2) ? OB_OK : OB_ERR_BITWIDTH; }

inline int launched() {
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? OB_OK : OB_ERR_HIP;
}

inline size_t align_up(size_t x) { return (x + 255) & ~size_t(255); }

struct DwWorkspace {
  size_t part, part_db, apart, total;
};

// G > 1: one layer's share of a grouped launch (plan of the G layers' N_total = G * N)
DwWorkspace dw_layout(int64_t P, int64_t M, int64_t N, int64_t K, int64_t G = 1) {
  const DwPlan p = plan_dw_passes(P, M, G * N, K);
  DwWorkspace w;
  w.part = align_up(sizeof(float) * (size_t)p.chunks * (size_t)N * (size_t)K);
  w.part_db = align_up(sizeof(float) * (size_t)p.chunks * (size_t)N);
  const int64_t napart = std::max<int64_t>(ste_reduce_blocks(N * K + N),
                                           p.tiles_n * p.tiles_k * p.chunks);
  w.apart = align_up(16 + sizeof(float) * (size_t)napart);
  w.total = w.part + w.part_db + w.apart;
  return w;
}

}  // namespace

extern "C" {

int ob_abi_version(void) { return kAbiVersion; }

const char* ob_status_string(int status) {
  switch (status) {
    case OB_OK: return "ok";
    case OB_ERR_NULL: return "null pointer argument";
    case OB_ERR_SHAPE: return "invalid shape";
    case OB_ERR_BITWIDTH: return "bitwidth must be one of {1,2,32}";
    case OB_ERR_WORKSPACE: return "workspace too small";
    case OB_ERR_ALIGN: return "pointer not 4-byte aligned";
    case OB_ERR_HIP: return "HIP launch error";
    default: return "unknown status";
  }
}

int ob_quant_pack(const float* W, const float* alpha, int alpha_raw, int bits, int64_t N,
                  int64_t K, uint32_t* codes, uint32_t* codes_t, void* stream) {
  if (int st = check_bits(bits)) return st;
  if (N < 0 || K < 0) return OB_ERR_SHAPE;
  if (!alpha || (N * K > 0 && !W)) return OB_ERR_NULL;
  if (!aligned4(W) || !aligned4(codes) || !aligned4(codes_t)) return OB_ERR_ALIGN;
  launch_quant_pack(W, alpha, alpha_raw, bits, nullptr, N, K, codes, codes_t, as_stream(stream));
  return launched();
}

int ob_quant_pack_dyn(const float* W, const float* alpha, int alpha_raw, const int32_t* bits_dev,
                      int64_t N, int64_t K, uint32_t* codes, uint32_t* codes_t, void* stream) {
  if (N < 0 || K < 0) return OB_ERR_SHAPE;
  if (!alpha || !bits_dev || (N * K > 0 && !W)) return OB_ERR_NULL;
  if (!aligned4(W) || !aligned4(codes) || !aligned4(codes_t) || !aligned4(bits_dev))
    return OB_ERR_ALIGN;
  launch_quant_pack(W, alpha, alpha_raw, 2, bits_dev, N, K, codes, codes_t, as_stream(stream));
  return launched();
}

int64_t ob_quant_pack_item_blocks(int64_t N, int64_t K) {
  if (N < 0 || K < 0) return OB_ERR_SHAPE;
  return quant_pack_item_blocks(N, K);
}

int64_t ob_weight_bf16_item_blocks(int64_t N, int64_t K) {
  if (N < 0 || K < 0) return OB_ERR_SHAPE;
  return quant_pack_item_blocks16(N, K);
}

int ob_quant_pack_group(const ob_pack_item* items, int n_items, int64_t total_blocks,
                        void* stream) {
  if (n_items < 0 || total_blocks < 0 || total_blocks > 0x7fffffff) return OB_ERR_SHAPE;
  if (n_items > 0 && !items) return OB_ERR_NULL;
  if (((uintptr_t)items & 7u) != 0) return OB_ERR_ALIGN;
  launch_quant_pack_group(items, n_items, total_blocks, as_stream(stream));
  return launched();
}

int ob_quant_dequant(const float* W, const float* alpha, int alpha_raw, int bits, int64_t n,
                     float* W_hat, void* stream) {
  if (int st = check_bits(bits)) return st;
  if (n < 0) return OB_ERR_SHAPE;
  if (!alpha || (n > 0 && (!W || !W_hat))) return OB_ERR_NULL;
  if (!aligned4(W) || !aligned4(W_hat)) return OB_ERR_ALIGN;
  launch_quant_dequant(W, alpha, alpha_raw, bits, n, W_hat, as_stream(stream));
  return launched();
}

size_t ob_quant_ste_bwd_workspace(int64_t n) {
  if (n < 0) return 0;
  return align_up(16 + sizeof(float) * (size_t)(ste_reduce_blocks(n) + 1));
}

int ob_quant_ste_bwd(const float* grad_W_hat, const float* W, const float* alpha, int alpha_raw,
                     int bits, int64_t n, float* grad_W, float* grad_alpha, void* ws,
                     size_t ws_bytes, void* stream) {
  if (int st = check_bits(bits)) return st;
  if (n < 0) return OB_ERR_SHAPE;
  if (!alpha || !grad_alpha || !ws || (n > 0 && (!grad_W_hat || !W || !grad_W)))
    return OB_ERR_NULL;
  if (ws_bytes < ob_quant_ste_bwd_workspace(n)) return OB_ERR_WORKSPACE;
  // ws: [ticket (16 B)][block partials]
  uint32_t* ticket = static_cast<uint32_t*>(ws);
  float* apart = reinterpret_cast<float*>(static_cast<char*>(ws) + 16);
  launch_zero_words(ticket, 1, as_stream(stream));
  launch_ste_reduce(grad_W_hat, 1, n, nullptr, 0, W, alpha, alpha_raw, bits, nullptr, grad_W,
                    nullptr, apart, ticket, grad_alpha, as_stream(stream));
  return launched();
}

int ob_bitlinear_fwd(const float* X, int64_t M, int64_t K, const uint32_t* codes,
                     const float* alpha, int alpha_raw, const float* bias, int64_t N, float* Y,
                     void* stream) {
  if (M < 0 || K < 0 || N < 0) return OB_ERR_SHAPE;
  if (!alpha || (M * N > 0 && !Y) || (M * K > 0 && !X) || (N * K > 0 && !codes))
    return OB_ERR_NULL;
  if (!aligned4(X) || !aligned4(Y) || !aligned4(bias)) return OB_ERR_ALIGN;
  launch_ternary_gemm(X, M, K, codes, N, alpha, alpha_raw, bias, Y, as_stream(stream));
  return launched();
}

int ob_bitlinear_fwd_signacc(const float* X, int64_t M, int64_t K, const uint32_t* codes,
                             const float* alpha, int alpha_raw, const float* bias, int64_t N,
                             float* Y, void* stream) {
  if (M < 0 || K < 0 || N < 0) return OB_ERR_SHAPE;
  if (!alpha || (M * N > 0 && !Y) || (M * K > 0 && !X) || (N * K > 0 && !codes))
    return OB_ERR_NULL;
  if ((reinterpret_cast<uintptr_t>(X) & 15) || !aligned4(Y) || !aligned4(bias)) return OB_ERR_ALIGN;
  if (!launch_ternary_gemm_signacc(X, M, K, codes, N, alpha, alpha_raw, bias, Y, as_stream(stream)))
    return OB_ERR_SHAPE;
  return launched();
}

int ob_bitlinear_bwd_dx(const float* dY, int64_t M, int64_t N, const uint32_t* codes_t,
                        const float* alpha, int alpha_raw, int64_t K, float* dX, void* stream) {
  if (M < 0 || K < 0 || N < 0) return OB_ERR_SHAPE;
  if (!alpha || (M * K > 0 && !dX) || (M * N > 0 && !dY) || (N * K > 0 && !codes_t))
    return OB_ERR_NULL;
  if (!aligned4(dY) || !aligned4(dX)) return OB_ERR_ALIGN;
  // dX = a * dY . Q: the same ternary GEMM with the roles of N and K exchanged.
  launch_ternary_gemm(dY, M, N, codes_t, K, alpha, alpha_raw, nullptr, dX, as_stream(stream));
  return launched();
}

size_t ob_bitlinear_bwd_dw_workspace(int64_t M, int64_t N, int64_t K) {
  if (M < 0 || N < 0 || K < 0) return 0;
  return dw_layout(1, M, N, K).total;
}

namespace {

// P stacked passes of M rows each (P = 1: the single-call entries). Pass bitwidths come
// from pass_bits (device [P]) when given, else from bits / bits_dev for the one pass.
int bwd_dw_impl(const float* dY, const float* X, int64_t P, int64_t M, int64_t N, int64_t K,
                const float* W, const float* alpha, int alpha_raw, int bits,
                const int32_t* bits_dev, const int32_t* pass_bits, float* dW, float* dalpha,
                float* db, void* ws, size_t ws_bytes, void* stream,
                DwFinish* defer = nullptr, DwFinishEntry* table = nullptr, int slot = 0,
                int64_t start = 0, int64_t* n_blocks = nullptr) {
  if (n_blocks) *n_blocks = 0;
  if (M < 0 || N < 0 || K < 0 || P < 1 || P > kMaxPasses) return OB_ERR_SHAPE;
  if (!alpha || !dalpha || !ws || (N * K > 0 && (!W || !dW)) || (M > 0 && (!dY || (K > 0 && !X))))
    return OB_ERR_NULL;
  if (!aligned4(dY) || !aligned4(X) || !aligned4(dW) || !aligned4(db) || !aligned4(bits_dev) ||
      !aligned4(pass_bits))
    return OB_ERR_ALIGN;
  const DwWorkspace L = dw_layout(P, M, N, K);
  if (ws_bytes < L.total) return OB_ERR_WORKSPACE;
  const DwPlan p = plan_dw_passes(P, M, N, K);
  char* base = static_cast<char*>(ws);
  float* part = reinterpret_cast<float*>(base);
  float* part_db = db ? reinterpret_cast<float*>(base + L.part) : nullptr;
  // apart region: [ticket (16 B)][block partials]
  uint32_t* ticket = reinterpret_cast<uint32_t*>(base + L.part + L.part_db);
  float* apart = reinterpret_cast<float*>(base + L.part + L.part_db + 16);
  hipStream_t s = as_stream(stream);
  int chunks = (int)p.chunks;
  int cpp = (int)p.chunks_per_pass;
  if (M == 0 || N == 0) {
    // No rows: every gradient is zero. Zero the first slab and reduce one chunk.
    launch_zero_words(part, N * K, s);
    if (db) launch_zero_words(part_db, N, s);
    launch_zero_words(ticket, 1, s);
    chunks = 1;
    cpp = 1;
    P = 1;
  } else if (p.variant >= 9) {  // LDS path: alpha partials in the GEMM, no ticket
    const DwAlpha al{W, alpha, alpha_raw, bits, reinterpret_cast<const int*>(bits_dev),
                     reinterpret_cast<const int*>(pass_bits), apart};
    const DwFinish fin{part, chunks, N * K, part_db, db ? N : 0, W, alpha, alpha_raw, apart,
                       (int)(p.tiles_n * p.tiles_k * p.chunks), dW, db, dalpha};
    if (table) {  // finish deferred to ob_dw_finish_table (entry written by the partial launch)
      const DwFinishEntry ent{fin, start};
      launch_dw_partial_group_defer(&dY, 1, X, P * M, N, K, p, &part, &part_db, &al, table, slot,
                                    &ent, s);
      if (n_blocks) *n_blocks = dw_finish_blocks(fin);
      return launched();
    }
    launch_dw_partial(dY, X, P * M, N, K, p, part, part_db, ticket, s, &al);
    if (defer) {  // the caller launches it (grouped with other layers' finishes)
      *defer = fin;
      return launched();
    }
    launch_dw_finish(fin.part, fin.chunks, fin.nk, fin.part_db, fin.n_db, fin.W, fin.alpha,
                     fin.alpha_raw, fin.apart, fin.n_apart, fin.dW, fin.db, fin.dalpha, s);
    return launched();
  } else {
    launch_dw_partial(dY, X, P * M, N, K, p, part, part_db, ticket, s);
  }
  if (pass_bits)
    launch_ste_reduce_passes(part, (int)P, cpp, N * K, part_db, db ? N : 0, W, alpha, alpha_raw,
                             reinterpret_cast<const int*>(pass_bits), dW, db, apart, ticket,
                             dalpha, s);
  else
    launch_ste_reduce(part, chunks, N * K, part_db, db ? N : 0, W, alpha, alpha_raw, bits,
                      reinterpret_cast<const int*>(bits_dev), dW, db, apart, ticket, dalpha, s);
  return launched();
}

}  // namespace

int ob_bitlinear_bwd_dw(const float* dY, const float* X, int64_t M, int64_t N, int64_t K,
                        const float* W, const float* alpha, int alpha_raw, int bits, float* dW,
                        float* dalpha, float* db, void* ws, size_t ws_bytes, void* stream) {
  if (int st = check_bits(bits)) return st;
  return bwd_dw_impl(dY, X, 1, M, N, K, W, alpha, alpha_raw, bits, nullptr, nullptr, dW, dalpha,
                     db, ws, ws_bytes, stream);
}

int ob_bitlinear_bwd_dw_dyn(const float* dY, const float* X, int64_t M, int64_t N, int64_t K,
                            const float* W, const float* alpha, int alpha_raw,
                            const int32_t* bits_dev, float* dW, float* dalpha, float* db, void* ws,
                            size_t ws_bytes, void* stream) {
  if (!bits_dev) return OB_ERR_NULL;
  return bwd_dw_impl(dY, X, 1, M, N, K, W, alpha, alpha_raw, 2, bits_dev, nullptr, dW, dalpha,
                     db, ws, ws_bytes, stream);
}

int ob_bitlinear_fwd_passes(const float* X, int64_t P, int64_t M, int64_t K,
                            const uint32_t* codes2, const uint32_t* codes1,
                            const int32_t* pass_bits, const float* alpha, int alpha_raw,
                            const float* bias, int64_t N, float* Y, void* stream) {
  if (M < 0 || K < 0 || N < 0 || P < 1 || P > 65535) return OB_ERR_SHAPE;
  if (!alpha || !pass_bits || (M * N > 0 && !Y) || (M * K > 0 && !X) ||
      (N * K > 0 && (!codes2 || !codes1)))
    return OB_ERR_NULL;
  if (!aligned4(X) || !aligned4(Y) || !aligned4(bias) || !aligned4(pass_bits)) return OB_ERR_ALIGN;
  launch_ternary_gemm_passes(X, (int)P, M, K, codes2, codes1, reinterpret_cast<const int*>(pass_bits),
                             N, alpha, alpha_raw, bias, Y, as_stream(stream));
  return launched();
}

int ob_bitlinear_fwd_passes_group(int64_t G, const float* X, int64_t P, int64_t M, int64_t K,
                                  const uint32_t* const* codes2, const uint32_t* const* codes1,
                                  const int32_t* pass_bits, const float* const* alpha,
                                  int alpha_raw, const float* const* bias, int64_t N,
                                  float* const* Y, void* stream) {
  if (G < 1 || G > 3 || M < 0 || K < 0 || N < 0 || P < 1 || P > 65535) return OB_ERR_SHAPE;
  if (!codes2 || !codes1 || !alpha || !bias || !Y || !pass_bits || (M * K > 0 && !X))
    return OB_ERR_NULL;
  for (int64_t i = 0; i < G; ++i) {
    if (!alpha[i] || (M * N > 0 && !Y[i]) || (N * K > 0 && (!codes2[i] || !codes1[i])))
      return OB_ERR_NULL;
    if (!aligned4(Y[i]) || !aligned4(bias[i])) return OB_ERR_ALIGN;
  }
  if (!aligned4(X) || !aligned4(pass_bits)) return OB_ERR_ALIGN;
  if (!launch_ternary_gemm_passes_group(X, (int)P, M, K, (int)G, codes2, codes1,
                                        reinterpret_cast<const int*>(pass_bits), N, alpha,
                                        alpha_raw, bias, Y, as_stream(stream)))
    return OB_ERR_SHAPE;
  return launched();
}

namespace {

// Shared argument checks of the fused-epilogue GEMM entries.
int fused_gemm_check(const float* A, int64_t P, int64_t M, int64_t K, const uint32_t* codes2,
                     const uint32_t* codes1, const int32_t* pass_bits, const float* alpha,
                     int64_t N, const float* out, float p_drop, const uint64_t* rng) {
  if (M < 0 || K < 0 || N < 0 || P < 1 || P > 65535) return OB_ERR_SHAPE;
  if (!(p_drop >= 0.0f && p_drop < 1.0f)) return OB_ERR_SHAPE;
  if (P > 1 && !pass_bits) return OB_ERR_NULL;
  if (!alpha || (M * N > 0 && !out) || (M * K > 0 && !A) ||
      (N * K > 0 && (!codes2 || (pass_bits && !codes1))) || (p_drop > 0.0f && !rng))
    return OB_ERR_NULL;
  if (!aligned4(A) || !aligned4(out) || !aligned4(pass_bits)) return OB_ERR_ALIGN;
  return OB_OK;
}

}  // namespace

int ob_bitlinear_fwd_swish_drop(const float* X, int64_t P, int64_t M, int64_t K,
                                const uint32_t* codes2, const uint32_t* codes1,
                                const int32_t* pass_bits, const float* alpha, int alpha_raw,
                                const float* bias, int64_t N, float p_drop, const uint64_t* rng,
                                int64_t rng_offset, float* Y_pre, float* Y_act, void* stream) {
  if (int st = fused_gemm_check(X, P, M, K, codes2, codes1, pass_bits, alpha, N, Y_act, p_drop, rng))
    return st;
  if (M * N > 0 && !Y_pre) return OB_ERR_NULL;
  if (!aligned4(Y_pre) || !aligned4(bias)) return OB_ERR_ALIGN;
  TgemmEpi ep{};
  ep.mode = kEpiSwishDrop;
  ep.C2 = Y_pre;
  ep.p_drop = p_drop;
  ep.rng = rng;
  ep.rng_off = (uint64_t)rng_offset;
  launch_ternary_gemm_passes(X, (int)P, M, K, codes2, pass_bits ? codes1 : codes2,
                             reinterpret_cast<const int*>(pass_bits), N, alpha, alpha_raw, bias,
                             Y_act, as_stream(stream), &ep);
  return launched();
}

int ob_bitlinear_fwd_residual(const float* X, int64_t P, int64_t M, int64_t K,
                              const uint32_t* codes2, const uint32_t* codes1,
                              const int32_t* pass_bits, const float* alpha, int alpha_raw,
                              const float* bias, int64_t N, const float* R, float rscale,
                              float p_drop, const uint64_t* rng, int64_t rng_offset,
                              const int32_t* lens, int64_t T, float* Y, void* stream) {
  if (int st = fused_gemm_check(X, P, M, K, codes2, codes1, pass_bits, alpha, N, Y, p_drop, rng))
    return st;
  if (M * N > 0 && !R) return OB_ERR_NULL;
  if (lens && (T < 1 || (P * M) % T)) return OB_ERR_SHAPE;
  if (T > 0x7fffffff) return OB_ERR_SHAPE;
  if (!aligned4(R) || !aligned4(bias) || !aligned4(lens)) return OB_ERR_ALIGN;
  TgemmEpi ep{};
  ep.mode = kEpiResidual;
  ep.R = R;
  ep.rscale = rscale;
  ep.lens = reinterpret_cast<const int*>(lens);
  ep.T = (int)T;
  ep.p_drop = p_drop;
  ep.rng = rng;
  ep.rng_off = (uint64_t)rng_offset;
  launch_ternary_gemm_passes(X, (int)P, M, K, codes2, pass_bits ? codes1 : codes2,
                             reinterpret_cast<const int*>(pass_bits), N, alpha, alpha_raw, bias, Y,
                             as_stream(stream), &ep);
  return launched();
}

int ob_bitlinear_fwd_residual_ln(const float* X, int64_t P, int64_t M, int64_t K,
                                 const uint32_t* codes2, const uint32_t* codes1,
                                 const int32_t* pass_bits, const float* alpha, int alpha_raw,
                                 const float* bias, int64_t N, const float* R, float rscale,
                                 float p_drop, const uint64_t* rng, int64_t rng_offset,
                                 const int32_t* lens, int64_t T, float* Y, int nln,
                                 const float* ln_w0, const float* ln_b0, float eps0, float* ln_y0,
                                 float* ln_mean0, float* ln_rstd0, const float* ln_w1,
                                 const float* ln_b1, float eps1, float* ln_y1, float* ln_mean1,
                                 float* ln_rstd1, void* stream) {
  if (int st = fused_gemm_check(X, P, M, K, codes2, codes1, pass_bits, alpha, N, Y, p_drop, rng))
    return st;
  if (nln < 1 || nln > 2) return OB_ERR_SHAPE;
  if (!ternary_residual_ln_supported(K, N, alpha_raw)) return OB_ERR_SHAPE;  // caller falls back
  if (M * N > 0 && (!R || !ln_y0 || !ln_mean0 || !ln_rstd0 ||
                    (nln > 1 && (!ln_y1 || !ln_mean1 || !ln_rstd1))))
    return OB_ERR_NULL;
  if (lens && (T < 1 || (P * M) % T)) return OB_ERR_SHAPE;
  if (T > 0x7fffffff) return OB_ERR_SHAPE;
  auto a16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  if (!a16(X) || !a16(R) || !a16(Y) || !a16(ln_y0) || !a16(ln_w0) || !a16(ln_b0) ||
      (nln > 1 && (!a16(ln_y1) || !a16(ln_w1) || !a16(ln_b1))) || !aligned4(bias) ||
      !aligned4(lens) || !aligned4(ln_mean0) || !aligned4(ln_rstd0) || !aligned4(ln_mean1) ||
      !aligned4(ln_rstd1))
    return OB_ERR_ALIGN;
  TgemmEpi ep{};
  ep.mode = kEpiResidual;
  ep.R = R;
  ep.rscale = rscale;
  ep.lens = reinterpret_cast<const int*>(lens);
  ep.T = (int)T;
  ep.p_drop = p_drop;
  ep.rng = rng;
  ep.rng_off = (uint64_t)rng_offset;
  ep.nln = nln;
  ep.lng[0] = ln_w0;
  ep.lnb[0] = ln_b0;
  ep.lneps[0] = eps0;
  ep.lny[0] = ln_y0;
  ep.lnmean[0] = ln_mean0;
  ep.lnrstd[0] = ln_rstd0;
  ep.lng[1] = ln_w1;
  ep.lnb[1] = ln_b1;
  ep.lneps[1] = eps1;
  ep.lny[1] = ln_y1;
  ep.lnmean[1] = ln_mean1;
  ep.lnrstd[1] = ln_rstd1;
  launch_ternary_gemm_passes(X, (int)P, M, K, codes2, pass_bits ? codes1 : codes2,
                             reinterpret_cast<const int*>(pass_bits), N, alpha, alpha_raw, bias, Y,
                             as_stream(stream), &ep);
  return launched();
}

int ob_bitlinear_bwd_dx_swish_drop(const float* dY, int64_t P, int64_t M, int64_t N,
                                   const uint32_t* codes2_t, const uint32_t* codes1_t,
                                   const int32_t* pass_bits, const float* alpha, int alpha_raw,
                                   int64_t K, const float* pre, float p_drop, const uint64_t* rng,
                                   int64_t rng_offset, float* dPre, void* stream) {
  if (int st = fused_gemm_check(dY, P, M, N, codes2_t, codes1_t, pass_bits, alpha, K, dPre, p_drop,
                                rng))
    return st;
  if (M * K > 0 && !pre) return OB_ERR_NULL;
  if (!aligned4(pre)) return OB_ERR_ALIGN;
  TgemmEpi ep{};
  ep.mode = kEpiSwishDropBwd;
  ep.R = pre;
  ep.p_drop = p_drop;
  ep.rng = rng;
  ep.rng_off = (uint64_t)rng_offset;
  launch_ternary_gemm_passes(dY, (int)P, M, N, codes2_t, pass_bits ? codes1_t : codes2_t,
                             reinterpret_cast<const int*>(pass_bits), K, alpha, alpha_raw, nullptr,
                             dPre, as_stream(stream), &ep);
  return launched();
}

int ob_drop_scale_bwd(const float* dOut, int64_t rows, int64_t N, float rscale, float p_drop,
                      const uint64_t* rng, int64_t rng_offset, const int32_t* lens, int64_t T,
                      float* dY, void* stream) {
  if (rows < 0 || N < 0 || !(p_drop >= 0.0f && p_drop < 1.0f)) return OB_ERR_SHAPE;
  if (lens && (T < 1 || T > 0x7fffffff || rows % T)) return OB_ERR_SHAPE;
  if ((rows * N > 0 && (!dOut || !dY)) || (p_drop > 0.0f && !rng)) return OB_ERR_NULL;
  if ((reinterpret_cast<uintptr_t>(dOut) & 15) || (reinterpret_cast<uintptr_t>(dY) & 15) ||
      !aligned4(lens))
    return OB_ERR_ALIGN;
  launch_drop_scale_bwd(dOut, rows, N, rscale, p_drop, rng, (uint64_t)rng_offset,
                        reinterpret_cast<const int*>(lens), (int)T, dY, as_stream(stream));
  return launched();
}

int ob_residual_drop_fwd(const float* R, const float* Y, int64_t rows, int64_t N, float rscale,
                         float p_drop, const uint64_t* rng, int64_t rng_offset,
                         const int32_t* lens, int64_t T, float* out, void* stream) {
  if (rows < 0 || N < 0 || !(p_drop >= 0.0f && p_drop < 1.0f)) return OB_ERR_SHAPE;
  if (lens && (T < 1 || T > 0x7fffffff || rows % T)) return OB_ERR_SHAPE;
  if ((rows * N > 0 && (!R || !Y || !out)) || (p_drop > 0.0f && !rng)) return OB_ERR_NULL;
  if (!aligned4(R) || !aligned4(Y) || !aligned4(out) || !aligned4(lens)) return OB_ERR_ALIGN;
  launch_residual_drop_fwd(R, Y, rows, N, rscale, p_drop, rng, (uint64_t)rng_offset,
                           reinterpret_cast<const int*>(lens), (int)T, out, as_stream(stream));
  return launched();
}

int ob_bias_relu_fwd(float* y, const float* bias, int64_t B, int64_t C, int64_t hw,
                     void* stream) {
  if (B < 0 || C < 0 || hw < 0) return OB_ERR_SHAPE;
  if (B * C * hw > 0 && (!y || !bias)) return OB_ERR_NULL;
  if (!aligned4(y) || !aligned4(bias)) return OB_ERR_ALIGN;
  if (hw % 4 == 0 && (reinterpret_cast<uintptr_t>(y) & 15)) return OB_ERR_ALIGN;
  launch_bias_relu_fwd(y, bias, B, C, hw, as_stream(stream));
  return launched();
}

size_t ob_relu_bias_bwd_workspace(int64_t B, int64_t C) {
  return (B < 0 || C < 0) ? 0 : relu_bias_bwd_workspace(B, C);
}

int ob_relu_bias_bwd(const float* g, const float* y, int64_t B, int64_t C, int64_t hw,
                     float* gout, float* dbias, void* ws, size_t ws_bytes, void* stream) {
  if (B < 0 || C < 0 || hw < 0 || B * C > 0x7fffffff) return OB_ERR_SHAPE;
  if (B * C * hw > 0 && (!g || !y || !gout)) return OB_ERR_NULL;
  if (B * C > 0 && !ws) return OB_ERR_NULL;
  if (ws_bytes < relu_bias_bwd_workspace(B, C)) return OB_ERR_WORKSPACE;
  if (!aligned4(g) || !aligned4(y) || !aligned4(gout) || !aligned4(dbias)) return OB_ERR_ALIGN;
  launch_relu_bias_bwd(g, y, B, C, hw, gout, dbias, ws, as_stream(stream));
  return launched();
}

size_t ob_colsum_workspace(int64_t N) { return N < 0 ? 0 : colsum_workspace(N); }

int ob_colsum(const float* x, int64_t rows, int64_t N, float* out, void* ws, size_t ws_bytes,
              void* stream) {
  if (rows < 0 || N < 0 || N > 0x7fffffff) return OB_ERR_SHAPE;
  if (N > 0 && (!out || !ws || (rows > 0 && !x))) return OB_ERR_NULL;
  if (ws_bytes < colsum_workspace(N)) return OB_ERR_WORKSPACE;
  if (!aligned4(x) || !aligned4(out)) return OB_ERR_ALIGN;
  launch_colsum(x, rows, N, out, ws, as_stream(stream));
  return launched();
}

namespace {
inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }
}  // namespace

int ob_dense_supported(int64_t K, int64_t N) { return dense_gemm_supported(K, N) ? 1 : 0; }

int ob_silu_fast_monotone_check(uint32_t lo_bits, uint32_t hi_bits, uint32_t* bad, void* stream) {
  if (!bad) return OB_ERR_NULL;
  if (lo_bits > hi_bits || hi_bits >= 0x7F800000u) return OB_ERR_SHAPE;  // finite, >= +0
  launch_silu_monotone_check(lo_bits, hi_bits, bad, as_stream(stream));
  return launched();
}

int ob_dense_gemm(const float* X, int64_t M, int64_t K, const float* W, int w_trans,
                  const float* bias, int64_t N, float* Y, void* stream) {
  if (M < 0 || M > ((int64_t)1 << 40) || !dense_gemm_supported(K, N)) return OB_ERR_SHAPE;
  if (!W || (M > 0 && (!X || !Y))) return OB_ERR_NULL;
  if (!aligned16(X) || !aligned16(W) || !aligned16(Y) || !aligned4(bias)) return OB_ERR_ALIGN;
  if (!launch_dense_gemm(X, M, K, W, w_trans, bias, N, Y, as_stream(stream))) return OB_ERR_SHAPE;
  return launched();
}

int ob_dense_gemm_residual_drop(const float* X, int64_t M, int64_t K, const float* W,
                                const float* bias, int64_t N, const float* R, float p_drop,
                                const int64_t* rng, int64_t rng_offset, float* Y, void* stream) {
  if (M < 0 || M > ((int64_t)1 << 40) || !dense_gemm_supported(K, N)) return OB_ERR_SHAPE;
  if (!(p_drop >= 0.0f && p_drop < 1.0f)) return OB_ERR_SHAPE;
  if (!W || (M > 0 && (!X || !Y || !R)) || (p_drop > 0.0f && !rng)) return OB_ERR_NULL;
  if (!aligned16(X) || !aligned16(W) || !aligned16(Y) || !aligned4(bias) || !aligned4(R))
    return OB_ERR_ALIGN;
  const DenseEpi epi{R, p_drop, reinterpret_cast<const uint64_t*>(rng), (uint64_t)rng_offset};
  if (!launch_dense_gemm(X, M, K, W, 0, bias, N, Y, as_stream(stream), &epi)) return OB_ERR_SHAPE;
  return launched();
}

size_t ob_dense_dw_workspace(int64_t M, int64_t N, int64_t K) {
  if (M < 0 || N <= 0 || K <= 0 || N % 4 != 0 || K % 4 != 0) return 0;
  const int v = plan_dw(M, N, K).variant;
  if (v != 4 && v < 9) return 0;  // the bf16x6 tiles (LDS: widths % 48; register: % 4)
  return dw_layout(1, M, N, K).total;
}

int ob_dense_dw(const float* dY, const float* X, int64_t M, int64_t N, int64_t K, float* dW,
                float* db, void* ws, size_t ws_bytes, void* stream) {
  return ob_dense_dw_defer(dY, X, M, N, K, dW, db, ws, ws_bytes, nullptr, 0, 0, nullptr, stream);
}

int ob_dense_dw_defer(const float* dY, const float* X, int64_t M, int64_t N, int64_t K,
                      float* dW, float* db, void* ws, size_t ws_bytes, void* table, int64_t slot,
                      int64_t start, int64_t* n_blocks, void* stream) {
  if (n_blocks) *n_blocks = 0;
  if (table && (!n_blocks || slot < 0 || start < 0)) return OB_ERR_NULL;
  const size_t need = ob_dense_dw_workspace(M, N, K);
  if (need == 0) return OB_ERR_SHAPE;
  if (!dW || !ws || (M > 0 && (!dY || !X))) return OB_ERR_NULL;
  if (ws_bytes < need) return OB_ERR_WORKSPACE;
  if (!aligned16(dY) || !aligned16(X) || !aligned4(dW) || !aligned4(db)) return OB_ERR_ALIGN;
  hipStream_t s = as_stream(stream);
  if (M == 0) {
    launch_zero_words(dW, N * K, s);
    if (db) launch_zero_words(db, N, s);
    return launched();
  }
  const DwWorkspace L = dw_layout(1, M, N, K);
  const DwPlan p = plan_dw(M, N, K);
  char* base = static_cast<char*>(ws);
  float* part = reinterpret_cast<float*>(base);
  float* part_db = db ? reinterpret_cast<float*>(base + L.part) : nullptr;
  const DwAlpha al{nullptr, nullptr, 0, 2, nullptr, nullptr, nullptr};  // no alpha: dense
  if (p.variant < 9) {  // register bf16x6 tiles (64-wide): the same chunk partials + finish
    uint32_t* ticket = reinterpret_cast<uint32_t*>(base + L.part + L.part_db);
    launch_dw_partial(dY, X, M, N, K, p, part, part_db, ticket, s);
    const DwFinish fin{part, (int)p.chunks, N * K, part_db, db ? N : 0, nullptr, nullptr, 0,
                       nullptr, 0, dW, db, nullptr};
    if (table) {
      // (no entry written by the register kernel: a 1-block launch writes it)
      const DwFinishEntry ent{fin, start};
      launch_dw_table_entry(static_cast<DwFinishEntry*>(table), (int)slot, ent, s);
      *n_blocks = dw_finish_blocks(fin);
      return launched();
    }
    launch_dw_finish(part, (int)p.chunks, N * K, part_db, db ? N : 0, nullptr, nullptr, 0,
                     nullptr, 0, dW, db, nullptr, s);
    return launched();
  }
  if (table) {  // finish deferred to ob_dw_finish_table
    const DwFinish fin{part, (int)p.chunks, N * K, part_db, db ? N : 0, nullptr, nullptr, 0,
                       nullptr, 0, dW, db, nullptr};
    const DwFinishEntry ent{fin, start};
    launch_dw_partial_group_defer(&dY, 1, X, M, N, K, p, &part, &part_db, &al,
                                  static_cast<DwFinishEntry*>(table), (int)slot, &ent, s);
    *n_blocks = dw_finish_blocks(fin);
    return launched();
  }
  launch_dw_partial(dY, X, M, N, K, p, part, part_db, nullptr, s, &al);
  launch_dw_finish(part, (int)p.chunks, N * K, part_db, db ? N : 0, nullptr, nullptr, 0, nullptr,
                   0, dW, db, nullptr, s);
  return launched();
}

namespace {
int subsample_check(int64_t B, int64_t T, int64_t F, int64_t C) {
  if (B < 1 || B > 65535 || T > (1 << 20) || F > (1 << 16)) return OB_ERR_SHAPE;
  if (B * ((T - 3) / 2 + 1) * ((F - 3) / 2 + 1) * C >= ((int64_t)1 << 30)) return OB_ERR_SHAPE;
  if (!subsample_supported(T, F, C)) return OB_ERR_SHAPE;
  return OB_OK;
}
}  // namespace

size_t ob_subsample_image_bytes(int64_t C) {
  return subsample_supported(7, 7, C) ? subsample_image_bytes(C) : 0;
}

int ob_subsample_pack(const float* W2, int64_t C, void* img, void* stream) {
  if (!subsample_supported(7, 7, C)) return OB_ERR_SHAPE;
  if (!W2 || !img) return OB_ERR_NULL;
  if (!aligned4(W2) || !aligned16(img)) return OB_ERR_ALIGN;
  launch_subsample_pack(W2, C, img, as_stream(stream));
  return launched();
}

int ob_subsample_fwd(const float* X, int64_t B, int64_t T, int64_t F, int64_t C,
                     const float* W0, const float* b0, const void* img, const float* b2,
                     float* Y1, float* Y2, void* stream) {
  if (const int st = subsample_check(B, T, F, C)) return st;
  if (!X || !W0 || !b0 || !img || !b2 || !Y1 || !Y2) return OB_ERR_NULL;
  if (!aligned4(X) || !aligned4(W0) || !aligned4(b0) || !aligned4(b2) || !aligned16(img) ||
      !aligned16(Y1) || !aligned16(Y2))
    return OB_ERR_ALIGN;
  launch_subsample_fwd(X, B, T, F, C, W0, b0, img, b2, Y1, Y2, as_stream(stream));
  return launched();
}

size_t ob_subsample_bwd_workspace(int64_t B, int64_t T, int64_t F, int64_t C) {
  return subsample_check(B, T, F, C) ? 0 : subsample_bwd_workspace(B, T, F, C);
}

int ob_subsample_bwd(const float* X, const float* W0, const float* b0, const float* Y1,
                     const float* Y2, const float* dY2, int64_t B, int64_t T, int64_t F, int64_t C,
                     const void* img, float* dW0,
                     float* db0, float* dW2, float* db2, void* ws, size_t ws_bytes,
                     void* stream) {
  if (const int st = subsample_check(B, T, F, C)) return st;
  if (!X || !W0 || !b0 || !Y1 || !Y2 || !dY2 || !img || !dW0 || !db0 || !dW2 || !db2 || !ws)
    return OB_ERR_NULL;
  if (ws_bytes < subsample_bwd_workspace(B, T, F, C)) return OB_ERR_WORKSPACE;
  if (!aligned4(X) || !aligned4(W0) || !aligned4(b0) || !aligned16(Y1) || !aligned16(Y2) ||
      !aligned16(dY2) || !aligned16(img) ||
      !aligned16(ws) || !aligned4(dW0) || !aligned4(db0) || !aligned4(dW2) || !aligned4(db2))
    return OB_ERR_ALIGN;
  if (B * ((T - 3) / 2 + 1) * ((F - 3) / 2 + 1) * C * 4 >= ((int64_t)1 << 31)) return OB_ERR_SHAPE;
  launch_subsample_bwd(X, W0, b0, Y1, Y2, dY2, B, T, F, C, img, dW0, db0, dW2, db2, ws,
                       as_stream(stream));
  return launched();
}

namespace {
int convmod_check(int64_t P, int64_t Bt, int64_t T, int64_t C, int64_t K) {
  if (P < 1 || Bt < 0 || T < 0 || C < 1 || K < 1 || Bt % P || Bt > 65535) return OB_ERR_SHAPE;
  if (!convmod_supported(C, K) || Bt * T * 2 * C > ((int64_t)1 << 40)) return OB_ERR_SHAPE;
  return OB_OK;
}
}  // namespace

size_t ob_convmod_workspace(int64_t P, int64_t Bt, int64_t T, int64_t C, int64_t K) {
  if (convmod_check(P, Bt, T, C, K)) return 0;
  return convmod_workspace(P, Bt, T, C, K);
}

int ob_convmod_fwd(const float* u, const float* w_dw, const float* b_dw, const float* gamma,
                   const float* beta, int64_t P, int64_t Bt, int64_t T, int64_t C, int64_t K,
                   float eps, float* z, float* g, float* stats, float* v, void* ws,
                   size_t ws_bytes, void* stream) {
  if (int st = convmod_check(P, Bt, T, C, K)) return st;
  if (Bt * T == 0) return OB_OK;
  if (!u || !w_dw || !gamma || !beta || !z || !g || !stats || !v || !ws) return OB_ERR_NULL;
  if (ws_bytes < convmod_workspace(P, Bt, T, C, K)) return OB_ERR_WORKSPACE;
  if (((uintptr_t)ws & 7u) || !aligned4(u) || !aligned4(z) || !aligned4(v) || !aligned4(stats) ||
      !aligned4(w_dw) || !aligned4(b_dw))
    return OB_ERR_ALIGN;
  if (!aligned4(g)) return OB_ERR_ALIGN;
  launch_convmod_fwd(u, w_dw, b_dw, gamma, beta, P, Bt, T, C, K, eps, z, g, stats, v, ws,
                     as_stream(stream));
  return launched();
}

int ob_convmod_bwd(const float* dv, const float* u, const float* z, const float* g,
                   const float* stats, const float* w_dw, const float* gamma, const float* beta,
                   int64_t P, int64_t Bt, int64_t T, int64_t C, int64_t K, float* du,
                   float* dw_dw, float* db_dw, float* dgamma, float* dbeta, void* ws,
                   size_t ws_bytes, void* stream) {
  if (int st = convmod_check(P, Bt, T, C, K)) return st;
  if (!dw_dw || !dgamma || !dbeta || !w_dw || !gamma || !beta) return OB_ERR_NULL;
  if (Bt * T > 0 && (!dv || !u || !z || !g || !stats || !du || !ws)) return OB_ERR_NULL;
  if (ws_bytes < convmod_workspace(P, Bt, T, C, K)) return OB_ERR_WORKSPACE;
  if (((uintptr_t)ws & 7u) || !aligned4(dv) || !aligned4(u) || !aligned4(z) || !aligned4(g) ||
      !aligned4(du))
    return OB_ERR_ALIGN;
  launch_convmod_bwd(dv, u, z, g, stats, w_dw, gamma, beta, P, Bt, T, C, K, du, dw_dw, db_dw,
                     dgamma, dbeta, ws, as_stream(stream));
  return launched();
}

int ob_convmod_bwd_defer(const float* dv, const float* u, const float* z, const float* g,
                         const float* stats, const float* w_dw, const float* gamma,
                         const float* beta, int64_t P, int64_t Bt, int64_t T, int64_t C, int64_t K,
                         float* du, float* dw_dw, float* db_dw, float* dgamma, float* dbeta,
                         void* ws, size_t ws_bytes, void* table, int64_t slot, int64_t* deferred,
                         void* stream) {
  if (int st = convmod_check(P, Bt, T, C, K)) return st;
  if (!dw_dw || !dgamma || !dbeta || !w_dw || !gamma || !beta) return OB_ERR_NULL;
  if (Bt * T > 0 && (!dv || !u || !z || !g || !stats || !du || !ws)) return OB_ERR_NULL;
  if (ws_bytes < convmod_workspace(P, Bt, T, C, K)) return OB_ERR_WORKSPACE;
  if (((uintptr_t)ws & 7u) || !aligned4(dv) || !aligned4(u) || !aligned4(z) || !aligned4(g) ||
      !aligned4(du))
    return OB_ERR_ALIGN;
  if (slot < 0) return OB_ERR_SHAPE;
  const bool dfr = table && Bt * T > 0 && convmod_bwd_deferrable(C, K);
  const CmDefer df{dfr ? static_cast<CmWgradEntry*>(table) : nullptr, (int)slot};
  launch_convmod_bwd(dv, u, z, g, stats, w_dw, gamma, beta, P, Bt, T, C, K, du, dw_dw, db_dw,
                     dgamma, dbeta, ws, as_stream(stream), &df);
  if (deferred) *deferred = dfr ? 1 : 0;
  return launched();
}

size_t ob_cm_wgrad_entry_bytes(void) { return sizeof(CmWgradEntry); }

int ob_cm_wgrad_table(const void* table, int64_t n, int64_t nmax, void* stream) {
  if (n < 0 || nmax < 0 || nmax > (1 << 24)) return OB_ERR_SHAPE;
  if (n > 0 && !table) return OB_ERR_NULL;
  launch_cm_wgrad_table(static_cast<const CmWgradEntry*>(table), (int)n, (int)nmax,
                        as_stream(stream));
  return launched();
}

size_t ob_act_absmax_workspace(int64_t P) {
  return (P < 1 || P > 65535) ? 0 : act_absmax_workspace((int)P);
}

int ob_act_absmax(const float* X, int64_t P, int64_t n_per_pass, float* amax, void* ws,
                  size_t ws_bytes, void* stream) {
  if (P < 1 || P > 65535 || n_per_pass < 0) return OB_ERR_SHAPE;
  if (!amax || !ws || (n_per_pass > 0 && !X)) return OB_ERR_NULL;
  if (ws_bytes < act_absmax_workspace((int)P)) return OB_ERR_WORKSPACE;
  if ((reinterpret_cast<uintptr_t>(X) & 15) || (n_per_pass % 4) || !aligned4(amax) ||
      !aligned4(ws))
    return OB_ERR_ALIGN;
  launch_act_absmax(X, (int)P, n_per_pass, amax, ws, as_stream(stream));
  return launched();
}

int ob_act_dequant_i8(const float* X, int64_t P, int64_t n_per_pass, const float* amax,
                      float* X_deq, void* stream) {
  if (P < 1 || P > 65535 || n_per_pass < 0) return OB_ERR_SHAPE;
  if (!amax || (n_per_pass > 0 && (!X || !X_deq))) return OB_ERR_NULL;
  if (!aligned4(X) || !aligned4(X_deq) || !aligned4(amax)) return OB_ERR_ALIGN;
  launch_act_dequant(X, (int)P, n_per_pass, amax, X_deq, as_stream(stream));
  return launched();
}

int ob_bitlinear_fwd_i8(const float* X, int64_t P, int64_t M, int64_t K, const uint32_t* codes,
                        const uint32_t* codes1, const int32_t* pass_bits, const float* alpha,
                        int alpha_raw, const float* amax, const float* bias, int64_t N, float* Y,
                        void* stream) {
  if (M < 0 || K < 0 || N < 0 || P < 1 || P > 65535) return OB_ERR_SHAPE;
  if (P > 1 && !pass_bits) return OB_ERR_NULL;
  if (!alpha || !amax || (M * N > 0 && !Y) || (M * K > 0 && !X) || (N * K > 0 && !codes) ||
      (pass_bits && N * K > 0 && !codes1))
    return OB_ERR_NULL;
  if (M * N > 0 && !ternary_gemm_i8_supported(K, N)) return OB_ERR_SHAPE;
  if ((reinterpret_cast<uintptr_t>(X) & 15) || !aligned4(Y) || !aligned4(bias) ||
      !aligned4(amax) || !aligned4(pass_bits))
    return OB_ERR_ALIGN;
  if (!launch_ternary_gemm_i8(X, (int)P, M, K, codes, pass_bits ? codes1 : codes,
                              reinterpret_cast<const int*>(pass_bits), N, alpha, alpha_raw, amax,
                              bias, Y, as_stream(stream)))
    return OB_ERR_SHAPE;
  return launched();
}

int ob_bitlinear_fwd_i8_epi(const float* X, int64_t P, int64_t M, int64_t K,
                            const uint32_t* codes, const uint32_t* codes1,
                            const int32_t* pass_bits, const float* alpha, int alpha_raw,
                            const float* amax, const float* bias, int64_t N, int mode,
                            const float* R, float rscale, const int32_t* lens, int64_t T,
                            float* amax_out, float* Y, void* stream) {
  if (M < 0 || K < 0 || N < 0 || P < 1 || P > 65535 || (mode != 1 && mode != 2) || N % 4)
    return OB_ERR_SHAPE;
  if (P > 1 && !pass_bits) return OB_ERR_NULL;
  if (!alpha || !amax || (M * N > 0 && !Y) || (M * K > 0 && !X) || (N * K > 0 && !codes) ||
      (pass_bits && N * K > 0 && !codes1) || (mode == 1 && !amax_out) ||
      (mode == 2 && M * N > 0 && !R) || (lens && T < 1))
    return OB_ERR_NULL;
  if (M * N > 0 && !ternary_gemm_i8_supported(K, N)) return OB_ERR_SHAPE;
  if ((reinterpret_cast<uintptr_t>(X) & 15) || (reinterpret_cast<uintptr_t>(Y) & 15) ||
      (reinterpret_cast<uintptr_t>(R) & 15) || !aligned4(bias) || !aligned4(amax) ||
      !aligned4(pass_bits) || !aligned4(amax_out) || !aligned4(lens))
    return OB_ERR_ALIGN;
  if (!launch_ternary_gemm_i8_epi(X, (int)P, M, K, codes, pass_bits ? codes1 : codes,
                                  reinterpret_cast<const int*>(pass_bits), N, alpha, alpha_raw,
                                  amax, bias, Y, mode, R, rscale,
                                  reinterpret_cast<const int*>(lens), T, amax_out,
                                  as_stream(stream)))
    return OB_ERR_SHAPE;
  return launched();
}

int ob_bitlinear_fwd_i8q(const int8_t* Xq, int64_t P, int64_t M, int64_t K,
                         const uint32_t* codes, const uint32_t* codes1, const int32_t* pass_bits,
                         const float* alpha, int alpha_raw, const float* amax, const float* bias,
                         int64_t N, int mode, const float* R, float rscale, const int32_t* lens,
                         int64_t T, float* amax_out, void* Y, void* stream) {
  if (M < 0 || K < 0 || N < 0 || P < 1 || P > 65535 || (mode != 0 && mode != 2 && mode != 3) ||
      N % 4 || (mode == 3 && N % 16))
    return OB_ERR_SHAPE;
  if (P > 1 && !pass_bits) return OB_ERR_NULL;
  if (!alpha || !amax || (M * N > 0 && !Y) || (M * K > 0 && !Xq) || (N * K > 0 && !codes) ||
      (pass_bits && N * K > 0 && !codes1) || (mode == 3 && !amax_out) ||
      (mode == 2 && M * N > 0 && !R) || (lens && T < 1))
    return OB_ERR_NULL;
  if (M * N > 0 && !ternary_gemm_i8_supported(K, N)) return OB_ERR_SHAPE;
  if ((reinterpret_cast<uintptr_t>(Xq) & 15) || (reinterpret_cast<uintptr_t>(Y) & 15) ||
      (reinterpret_cast<uintptr_t>(R) & 15) || !aligned4(bias) || !aligned4(amax) ||
      !aligned4(pass_bits) || !aligned4(amax_out) || !aligned4(lens))
    return OB_ERR_ALIGN;
  if (!launch_ternary_gemm_i8q(Xq, (int)P, M, K, codes, pass_bits ? codes1 : codes,
                               reinterpret_cast<const int*>(pass_bits), N, alpha, alpha_raw, amax,
                               bias, Y, mode, R, rscale, reinterpret_cast<const int*>(lens), T,
                               amax_out, as_stream(stream)))
    return OB_ERR_SHAPE;
  return launched();
}

int ob_bitlinear_bwd_dx_passes(const float* dY, int64_t P, int64_t M, int64_t N,
                               const uint32_t* codes2_t, const uint32_t* codes1_t,
                               const int32_t* pass_bits, const float* alpha, int alpha_raw,
                               int64_t K, float* dX, void* stream) {
  if (M < 0 || K < 0 || N < 0 || P < 1 || P > 65535) return OB_ERR_SHAPE;
  if (!alpha || !pass_bits || (M * K > 0 && !dX) || (M * N > 0 && !dY) ||
      (N * K > 0 && (!codes2_t || !codes1_t)))
    return OB_ERR_NULL;
  if (!aligned4(dY) || !aligned4(dX) || !aligned4(pass_bits)) return OB_ERR_ALIGN;
  launch_ternary_gemm_passes(dY, (int)P, M, N, codes2_t, codes1_t,
                             reinterpret_cast<const int*>(pass_bits), K, alpha, alpha_raw, nullptr,
                             dX, as_stream(stream));
  return launched();
}

int ob_bitlinear_bwd_dx_passes_sum(int64_t G, const float* const* dY, int64_t P, int64_t M,
                                   int64_t N, const uint32_t* const* codes2_t,
                                   const uint32_t* const* codes1_t, const int32_t* pass_bits,
                                   const float* const* alpha, int alpha_raw, int64_t K, float* dX,
                                   void* stream) {
  if (G < 1 || G > 3 || M < 0 || K < 0 || N < 0 || P < 1 || P > 65535) return OB_ERR_SHAPE;
  if (!dY || !codes2_t || !codes1_t || !alpha || !pass_bits || !dX) return OB_ERR_NULL;
  for (int64_t i = 0; i < G; ++i)
    if (!dY[i] || !codes2_t[i] || !codes1_t[i] || !alpha[i]) return OB_ERR_NULL;
  if (!aligned4(pass_bits)) return OB_ERR_ALIGN;
  if (!launch_ternary_dx_sum((int)G, dY, (int)P, M, N, codes2_t, codes1_t,
                             reinterpret_cast<const int*>(pass_bits), alpha, alpha_raw, K, dX,
                             as_stream(stream)))
    return OB_ERR_SHAPE;  // not this kernel's shape: one ob_bitlinear_bwd_dx_passes per source
  return launched();
}

size_t ob_bitlinear_bwd_dw_passes_workspace(int64_t P, int64_t M, int64_t N, int64_t K) {
  if (M < 0 || N < 0 || K < 0 || P < 1 || P > kMaxPasses) return 0;
  return dw_layout(P, M, N, K).total;
}

int ob_bitlinear_bwd_dw_passes(const float* dY, const float* X, int64_t P, int64_t M, int64_t N,
                               int64_t K, const float* W, const float* alpha, int alpha_raw,
                               const int32_t* pass_bits, float* dW, float* dalpha, float* db,
                               void* ws, size_t ws_bytes, void* stream) {
  if (!pass_bits) return OB_ERR_NULL;
  return bwd_dw_impl(dY, X, P, M, N, K, W, alpha, alpha_raw, 2, nullptr, pass_bits, dW, dalpha,
                     db, ws, ws_bytes, stream);
}

size_t ob_bitlinear_bwd_dw_passes_group_workspace(int64_t G, int64_t P, int64_t M, int64_t N,
                                                  int64_t K) {
  if (G < 1 || G > kMaxDwGroup) return 0;
  const size_t one = ob_bitlinear_bwd_dw_passes_workspace(P, M, N, K);
  if (!one) return 0;
  return (size_t)G * std::max(align_up(one), dw_layout(P, M, N, K, G).total);
}

namespace {
int dw_group_impl(int64_t G, const float* const* dY, const float* X, int64_t P, int64_t M,
                  int64_t N, int64_t K, const float* const* W, const float* const* alpha,
                  int alpha_raw, const int32_t* pass_bits, float* const* dW,
                  float* const* dalpha, float* const* db, void* ws, size_t ws_bytes,
                  void* stream, DwFinishEntry* table, int slot, int64_t start,
                  int64_t* n_blocks);
}  // namespace

int ob_bitlinear_bwd_dw_passes_group(int64_t G, const float* const* dY, const float* X,
                                     int64_t P, int64_t M, int64_t N, int64_t K,
                                     const float* const* W, const float* const* alpha,
                                     int alpha_raw, const int32_t* pass_bits, float* const* dW,
                                     float* const* dalpha, float* const* db, void* ws,
                                     size_t ws_bytes, void* stream) {
  return dw_group_impl(G, dY, X, P, M, N, K, W, alpha, alpha_raw, pass_bits, dW, dalpha, db, ws,
                       ws_bytes, stream, nullptr, 0, 0, nullptr);
}

int ob_bitlinear_bwd_dw_passes_group_defer(int64_t G, const float* const* dY, const float* X,
                                           int64_t P, int64_t M, int64_t N, int64_t K,
                                           const float* const* W, const float* const* alpha,
                                           int alpha_raw, const int32_t* pass_bits,
                                           float* const* dW, float* const* dalpha,
                                           float* const* db, void* ws, size_t ws_bytes,
                                           void* table, int64_t slot, int64_t start,
                                           int64_t* n_blocks, void* stream) {
  if (!table || !n_blocks || slot < 0 || start < 0) return OB_ERR_NULL;
  return dw_group_impl(G, dY, X, P, M, N, K, W, alpha, alpha_raw, pass_bits, dW, dalpha, db, ws,
                       ws_bytes, stream, static_cast<DwFinishEntry*>(table), (int)slot, start,
                       n_blocks);
}

namespace {
int dw_group_impl(int64_t G, const float* const* dY, const float* X, int64_t P, int64_t M,
                  int64_t N, int64_t K, const float* const* W, const float* const* alpha,
                  int alpha_raw, const int32_t* pass_bits, float* const* dW,
                  float* const* dalpha, float* const* db, void* ws, size_t ws_bytes,
                  void* stream, DwFinishEntry* table, int slot, int64_t start,
                  int64_t* n_blocks) {
  if (n_blocks) *n_blocks = 0;
  if (G < 1 || G > kMaxDwGroup) return OB_ERR_SHAPE;
  if (!dY || !W || !alpha || !dW || !dalpha || !db || !pass_bits || !ws) return OB_ERR_NULL;
  const size_t need = ob_bitlinear_bwd_dw_passes_group_workspace(G, P, M, N, K);
  if (need == 0) return OB_ERR_SHAPE;
  if (ws_bytes < need) return OB_ERR_WORKSPACE;
  const size_t one = need / (size_t)G;
  const DwPlan pg = plan_dw_passes(P, M, G * N, K);
  if (pg.variant >= 9 && M > 0 && N > 0 && K > 0 && P <= kMaxPasses) {
    // one partial launch for the G layers (they share X), then one grouped finish
    for (int64_t i = 0; i < G; ++i)
      if (!dY[i] || !W[i] || !alpha[i] || !dW[i] || !dalpha[i]) return OB_ERR_NULL;
    if (!X) return OB_ERR_NULL;
    if (!aligned4(X) || !aligned4(pass_bits)) return OB_ERR_ALIGN;
    const DwWorkspace Lg = dw_layout(P, M, N, K, G);
    float* part[kMaxDwGroup];
    float* part_db[kMaxDwGroup];
    DwAlpha al[kMaxDwGroup];
    DwFinish fin[kMaxDwGroup];
    for (int64_t i = 0; i < G; ++i) {
      if (!aligned4(dY[i]) || !aligned4(dW[i]) || !aligned4(db[i])) return OB_ERR_ALIGN;
      char* base = static_cast<char*>(ws) + i * one;
      part[i] = reinterpret_cast<float*>(base);
      part_db[i] = db[i] ? reinterpret_cast<float*>(base + Lg.part) : nullptr;
      float* apart = reinterpret_cast<float*>(base + Lg.part + Lg.part_db + 16);
      al[i] = DwAlpha{W[i], alpha[i], alpha_raw, 2, nullptr,
                      reinterpret_cast<const int*>(pass_bits), apart};
      fin[i] = DwFinish{part[i], (int)pg.chunks, N * K, part_db[i], db[i] ? N : 0, W[i],
                        alpha[i], alpha_raw, apart, (int)(pg.tiles_n / G * pg.tiles_k * pg.chunks),
                        dW[i], db[i], dalpha[i]};
    }
    hipStream_t s = as_stream(stream);
    if (table) {  // finishes deferred to ob_dw_finish_table
      DwFinishEntry ent[kMaxDwGroup];
      int64_t at = start;
      for (int64_t i = 0; i < G; ++i) {
        ent[i] = DwFinishEntry{fin[i], at};
        at += dw_finish_blocks(fin[i]);
      }
      launch_dw_partial_group_defer(dY, (int)G, X, P * M, N, K, pg, part, part_db, al, table,
                                    slot, ent, s);
      *n_blocks = at - start;
      return launched();
    }
    launch_dw_partial_group(dY, (int)G, X, P * M, N, K, pg, part, part_db, al, s);
    launch_dw_finish_group(fin, (int)G, s);
    return launched();
  }
  DwFinish fin[kMaxDwGroup];
  bool deferred[kMaxDwGroup] = {false, false, false};
  for (int64_t i = 0; i < G; ++i) {
    fin[i].part = nullptr;
    const int st = bwd_dw_impl(dY[i], X, P, M, N, K, W[i], alpha[i], alpha_raw, 2, nullptr,
                               pass_bits, dW[i], dalpha[i], db[i],
                               static_cast<char*>(ws) + i * one, one, stream, &fin[i]);
    if (st != OB_OK) return st;
    deferred[i] = fin[i].part != nullptr;
  }
  // the LDS path deferred its finish (every layer, at one shape); others finished already
  int nd = 0;
  DwFinish grp[kMaxDwGroup];
  for (int64_t i = 0; i < G; ++i)
    if (deferred[i]) grp[nd++] = fin[i];
  if (nd) launch_dw_finish_group(grp, nd, as_stream(stream));
  return launched();
}
}  // namespace

int ob_bitlinear_bwd_dw_passes_defer(const float* dY, const float* X, int64_t P, int64_t M,
                                     int64_t N, int64_t K, const float* W, const float* alpha,
                                     int alpha_raw, const int32_t* pass_bits, float* dW,
                                     float* dalpha, float* db, void* ws, size_t ws_bytes,
                                     void* table, int64_t slot, int64_t start, int64_t* n_blocks,
                                     void* stream) {
  if (!pass_bits || !table || !n_blocks || slot < 0 || start < 0) return OB_ERR_NULL;
  return bwd_dw_impl(dY, X, P, M, N, K, W, alpha, alpha_raw, 2, nullptr, pass_bits, dW, dalpha,
                     db, ws, ws_bytes, stream, nullptr, static_cast<DwFinishEntry*>(table),
                     (int)slot, start, n_blocks);
}

size_t ob_dw_finish_entry_bytes(void) { return sizeof(DwFinishEntry); }

int ob_dw_finish_table(const void* table, int64_t n, int64_t total_blocks, void* stream) {
  if (n < 0 || total_blocks < 0 || total_blocks > 0x7fffffff) return OB_ERR_SHAPE;
  if (n > 0 && !table) return OB_ERR_NULL;
  launch_dw_finish_table(static_cast<const DwFinishEntry*>(table), (int)n, total_blocks,
                         as_stream(stream));
  return launched();
}

int ob_dw_grouped_supported(int64_t N, int64_t K) {
  return N > 0 && K > 0 && N % kDwgTile == 0 && K % kDwgTile == 0 && N <= (1 << 20) &&
         K <= (1 << 20);
}

namespace {
struct DwgPlan {
  std::vector<DwgDesc> d;
  int64_t steps = 0;
  int tiles = 0, blocks = 0;
  size_t table = 0, slots = 0, talpha = 0, total = 0;
};

// validates the descriptors and lays out the linear work space (gemm-major, tile, pass, step)
int dwg_plan(const ob_dwg_gemm* g, int64_t G, DwgPlan& pl) {
  if (G < 1 || G > (1 << 16)) return OB_ERR_SHAPE;
  if (!g) return OB_ERR_NULL;
  pl.d.resize((size_t)G);
  int64_t tiles = 0;
  for (int64_t i = 0; i < G; ++i) {
    const ob_dwg_gemm& e = g[i];
    // 32-bit offsets in the kernel: one pass of an operand, the weight, the step count
    if (!ob_dw_grouped_supported(e.N, e.K) || e.M < 1 || e.P < 1 || e.P > kMaxPasses ||
        e.M * e.P >= ((int64_t)1 << 30) || e.M * std::max(e.N, e.K) * 4 >= ((int64_t)1 << 31) ||
        e.N * e.K * 4 >= ((int64_t)1 << 31))
      return OB_ERR_SHAPE;
    if (!e.dY || !e.X || !e.dW) return OB_ERR_NULL;
    if (e.W && (!e.alpha || !e.dalpha)) return OB_ERR_NULL;
    if (e.W && !e.pass_bits && check_bits(e.bits) != OB_OK) return OB_ERR_BITWIDTH;
    if (!aligned4(e.dY) || !aligned4(e.X) || ((reinterpret_cast<uintptr_t>(e.dY) |
                                               reinterpret_cast<uintptr_t>(e.X)) & 15))
      return OB_ERR_ALIGN;
    DwgDesc& d = pl.d[(size_t)i];
    d.dY = e.dY;
    d.X = e.X;
    d.W = e.W;
    d.alpha = e.alpha;
    d.pass_bits = e.pass_bits;
    d.dW = e.dW;
    d.db = e.db;
    d.dalpha = e.dalpha;
    d.N = (int)e.N;
    d.K = (int)e.K;
    d.Mp = (int)e.M;
    d.P = (int)e.P;
    d.alpha_raw = e.alpha_raw;
    d.bits = e.bits;
    d.spp = (int)ceil_div(e.M, 32);
    d.tiles_k = (int)(e.K / kDwgTile);
    d.tiles = (int)((e.N / kDwgTile) * d.tiles_k);
    d.tile0 = (int)tiles;
    d.work0 = pl.steps;
    tiles += d.tiles;
    pl.steps += (int64_t)d.tiles * d.P * d.spp;
  }
  if (tiles > (1 << 24) || pl.steps >= ((int64_t)1 << 31)) return OB_ERR_SHAPE;
  pl.tiles = (int)tiles;
  pl.blocks = dwg_blocks(pl.steps);
  pl.table = align_up(sizeof(DwgDesc) * (size_t)G);
  pl.slots = align_up(dwg_slot_bytes() * 2 * (size_t)pl.blocks);
  pl.talpha = align_up(sizeof(float) * (size_t)tiles);
  pl.total = pl.table + pl.slots + pl.talpha;
  return OB_OK;
}
}  // namespace

size_t ob_dw_grouped_workspace(const ob_dwg_gemm* gemms, int64_t G) {
  DwgPlan pl;
  return dwg_plan(gemms, G, pl) == OB_OK ? pl.total : 0;
}

size_t ob_dw_grouped_tickets(const ob_dwg_gemm* gemms, int64_t G) {
  DwgPlan pl;
  return dwg_plan(gemms, G, pl) == OB_OK ? (size_t)pl.tiles + (size_t)G : 0;
}

int ob_dw_grouped(const ob_dwg_gemm* gemms, int64_t G, void* ws, size_t ws_bytes, void* tickets,
                  size_t ticket_words, void* stream) {
  DwgPlan pl;
  const int st = dwg_plan(gemms, G, pl);
  if (st != OB_OK) return st;
  if (!ws || !tickets) return OB_ERR_NULL;
  if (ws_bytes < pl.total || ticket_words < (size_t)pl.tiles + (size_t)G) return OB_ERR_WORKSPACE;
  unsigned char* base = static_cast<unsigned char*>(ws);
  launch_dw_grouped(pl.d.data(), (int)G, pl.steps, pl.blocks, reinterpret_cast<DwgDesc*>(base),
                    reinterpret_cast<float*>(base + pl.table),
                    reinterpret_cast<float*>(base + pl.table + pl.slots),
                    static_cast<uint32_t*>(tickets), pl.tiles, as_stream(stream));
  return launched();
}

int ob_dwconv1d_fwd(const float* x, const float* w, const float* bias, int64_t B, int64_t C,
                    int64_t T, int64_t KT, float* y, void* stream) {
  if (B < 0 || C < 0 || T < 0 || KT < 1 || KT % 2 == 0 || !dwconv_supported((int)KT))
    return OB_ERR_SHAPE;
  if (B * C * T > 0 && (!x || !y || !w)) return OB_ERR_NULL;
  if (!aligned4(x) || !aligned4(y) || !aligned4(w) || !aligned4(bias)) return OB_ERR_ALIGN;
  launch_dwconv_fwd(x, w, bias, B, C, T, KT, y, as_stream(stream));
  return launched();
}

size_t ob_dwconv1d_bwd_workspace(int64_t B, int64_t C, int64_t KT) {
  if (B < 0 || C < 0 || KT < 1) return 0;
  return align_up(dwconv_bwd_workspace(B, C, KT));
}

int ob_dwconv1d_bwd(const float* x, const float* dy, const float* w, int64_t B, int64_t C,
                    int64_t T, int64_t KT, float* dx, float* dw, float* db, void* ws,
                    size_t ws_bytes, void* stream) {
  if (B < 0 || C < 0 || T < 0 || KT < 1 || KT % 2 == 0 || !dwconv_supported((int)KT))
    return OB_ERR_SHAPE;
  if (!dw || !w || !ws || (B * C * T > 0 && (!x || !dy))) return OB_ERR_NULL;
  if (!aligned4(x) || !aligned4(dy) || !aligned4(dx) || !aligned4(dw) || !aligned4(db))
    return OB_ERR_ALIGN;
  if (ws_bytes < ob_dwconv1d_bwd_workspace(B, C, KT)) return OB_ERR_WORKSPACE;
  launch_dwconv_bwd(x, dy, w, B, C, T, KT, dx, dw, db, static_cast<float*>(ws),
                    as_stream(stream));
  return launched();
}

size_t ob_ctc_loss_workspace(int64_t B, int64_t T, int64_t S) {
  if (B < 0 || T < 0 || S < 0) return 0;
  return align_up(ctc_workspace(B, T, S));
}

int ob_ctc_loss_fwd(const float* log_probs, const int64_t* targets, const int64_t* input_lengths,
                    const int64_t* target_lengths, int64_t B, int64_t T, int64_t V, int64_t S,
                    int blank, float* loss, void* ws, size_t ws_bytes, void* stream) {
  if (B < 1 || T < 0 || V < 1 || S < 0 || blank < 0 || blank >= V || !ctc_supported(S))
    return OB_ERR_SHAPE;
  if (!log_probs || !input_lengths || !target_lengths || !loss || !ws || (S > 0 && !targets))
    return OB_ERR_NULL;
  if (ws_bytes < ob_ctc_loss_workspace(B, T, S)) return OB_ERR_WORKSPACE;
  launch_ctc_fwd(log_probs, targets, input_lengths, target_lengths, B, T, V, S, blank, 1, loss,
                 static_cast<float*>(ws), as_stream(stream));
  return launched();
}

int ob_ctc_loss_fwd_groups(const float* log_probs, const int64_t* targets,
                           const int64_t* input_lengths, const int64_t* target_lengths, int64_t G,
                           int64_t B, int64_t T, int64_t V, int64_t S, int blank, float* loss,
                           void* ws, size_t ws_bytes, void* stream) {
  if (G < 1 || G > 64 || B < 1 || B % G || T < 0 || V < 1 || S < 0 || blank < 0 || blank >= V ||
      !ctc_supported(S))
    return OB_ERR_SHAPE;
  if (!log_probs || !input_lengths || !target_lengths || !loss || !ws || (S > 0 && !targets))
    return OB_ERR_NULL;
  if (ws_bytes < ob_ctc_loss_workspace(B, T, S)) return OB_ERR_WORKSPACE;
  launch_ctc_fwd(log_probs, targets, input_lengths, target_lengths, B, T, V, S, blank, G, loss,
                 static_cast<float*>(ws), as_stream(stream));
  return launched();
}

int ob_ctc_loss_bwd(const float* log_probs, const int64_t* targets, const int64_t* input_lengths,
                    const int64_t* target_lengths, int64_t B, int64_t T, int64_t V, int64_t S,
                    int blank, const float* grad_out, float* grad, void* ws, size_t ws_bytes,
                    void* stream) {
  if (B < 1 || T < 0 || V < 1 || S < 0 || blank < 0 || blank >= V || !ctc_supported(S))
    return OB_ERR_SHAPE;
  if (!log_probs || !input_lengths || !target_lengths || !grad || !ws || (S > 0 && !targets))
    return OB_ERR_NULL;
  if (ws_bytes < ob_ctc_loss_workspace(B, T, S)) return OB_ERR_WORKSPACE;
  launch_ctc_bwd(log_probs, targets, input_lengths, target_lengths, B, T, V, S, blank, 1,
                 grad_out, grad, static_cast<float*>(ws), as_stream(stream));
  return launched();
}

int ob_ctc_loss_bwd_groups(const float* log_probs, const int64_t* targets,
                           const int64_t* input_lengths, const int64_t* target_lengths, int64_t G,
                           int64_t B, int64_t T, int64_t V, int64_t S, int blank,
                           const float* grad_out, float* grad, void* ws, size_t ws_bytes,
                           void* stream) {
  if (G < 1 || G > 64 || B < 1 || B % G || T < 0 || V < 1 || S < 0 || blank < 0 || blank >= V ||
      !ctc_supported(S))
    return OB_ERR_SHAPE;
  if (!log_probs || !input_lengths || !target_lengths || !grad || !ws || (S > 0 && !targets))
    return OB_ERR_NULL;
  if (ws_bytes < ob_ctc_loss_workspace(B, T, S)) return OB_ERR_WORKSPACE;
  launch_ctc_bwd(log_probs, targets, input_lengths, target_lengths, B, T, V, S, blank, G,
                 grad_out, grad, static_cast<float*>(ws), as_stream(stream));
  return launched();
}

size_t ob_ctc_logits_workspace(int64_t B, int64_t T, int64_t S) {
  if (B < 0 || T < 0 || S < 0) return 0;
  return align_up(ctc_logits_workspace_bytes(B, T, S));
}

namespace {
int ctc_logits_check(const float* x, const int64_t* targets, const int64_t* input_lengths,
                     const int64_t* target_lengths, int64_t G, int64_t B, int64_t T, int64_t V,
                     int64_t S, int blank, const void* out, void* ws, size_t ws_bytes) {
  if (G < 1 || G > 64 || B < 1 || B % G || T < 0 || V < 1 || V > INT32_MAX || S < 0 ||
      blank < 0 || blank >= V || !ctc_supported(S) || B * T > INT32_MAX)
    return OB_ERR_SHAPE;
  if (!x || !input_lengths || !target_lengths || !out || !ws || (S > 0 && !targets))
    return OB_ERR_NULL;
  if (ws_bytes < ob_ctc_logits_workspace(B, T, S)) return OB_ERR_WORKSPACE;
  if ((V & 3) == 0 && (reinterpret_cast<uintptr_t>(x) & 15)) return OB_ERR_ALIGN;
  return OB_OK;
}
}  // namespace

int ob_ctc_loss_logits_fwd_groups(const float* logits, const int64_t* targets,
                                  const int64_t* input_lengths, const int64_t* target_lengths,
                                  int64_t G, int64_t B, int64_t T, int64_t V, int64_t S, int blank,
                                  float* loss, void* ws, size_t ws_bytes, void* stream) {
  if (int st = ctc_logits_check(logits, targets, input_lengths, target_lengths, G, B, T, V, S,
                                blank, loss, ws, ws_bytes))
    return st;
  launch_ctc_logits_fwd(logits, targets, input_lengths, target_lengths, B, T, V, S, blank, G,
                        loss, ws, as_stream(stream));
  return launched();
}

int ob_ctc_loss_logits_bwd_groups(const float* logits, const int64_t* targets,
                                  const int64_t* input_lengths, const int64_t* target_lengths,
                                  int64_t G, int64_t B, int64_t T, int64_t V, int64_t S, int blank,
                                  const float* grad_out, float* grad, void* ws, size_t ws_bytes,
                                  void* stream) {
  if (int st = ctc_logits_check(logits, targets, input_lengths, target_lengths, G, B, T, V, S,
                                blank, grad, ws, ws_bytes))
    return st;
  if ((V & 3) == 0 && (reinterpret_cast<uintptr_t>(grad) & 15)) return OB_ERR_ALIGN;
  launch_ctc_logits_bwd(logits, targets, input_lengths, target_lengths, B, T, V, S, blank, G,
                        grad_out, grad, ws, as_stream(stream));
  return launched();
}

size_t ob_att_kl_workspace(int64_t P, int64_t BU) {
  if (P < 1 || BU < 0) return 0;
  return align_up(att_kl_workspace(P, BU));
}

namespace {
int att_kl_check(const float* x, const int64_t* tgt, const uint8_t* pad, int64_t P, int64_t BU,
                 int64_t V, float ls, const void* out, size_t ws_bytes, const void* ws) {
  if (P < 1 || P > 64 || BU < 1 || !att_kl_supported(V) || P * BU > INT32_MAX ||
      !(ls > 0.0f && ls < 1.0f))
    return OB_ERR_SHAPE;
  if (!x || !tgt || !pad || !out || !ws) return OB_ERR_NULL;
  if (ws_bytes < ob_att_kl_workspace(P, BU)) return OB_ERR_WORKSPACE;
  if (reinterpret_cast<uintptr_t>(x) & 15) return OB_ERR_ALIGN;
  return OB_OK;
}
}  // namespace

int ob_att_kl_loss_fwd(const float* logits, const int64_t* tgt_out, const uint8_t* tgt_pad,
                       int64_t P, int64_t BU, int64_t V, int pad_id, float label_smoothing,
                       float* l_att, float* l_kl, void* ws, size_t ws_bytes, void* stream) {
  if (int st = att_kl_check(logits, tgt_out, tgt_pad, P, BU, V, label_smoothing, l_att, ws_bytes,
                            ws))
    return st;
  if (P > 1 && !l_kl) return OB_ERR_NULL;
  launch_att_kl_fwd(logits, tgt_out, tgt_pad, P, BU, V, pad_id, label_smoothing, l_att, l_kl, ws,
                    as_stream(stream));
  return launched();
}

int ob_att_kl_loss_bwd(const float* logits, const int64_t* tgt_out, const uint8_t* tgt_pad,
                       int64_t P, int64_t BU, int64_t V, float label_smoothing,
                       const float* g_att, const float* g_kl, float* grad, const void* ws,
                       size_t ws_bytes, void* stream) {
  if (int st = att_kl_check(logits, tgt_out, tgt_pad, P, BU, V, label_smoothing, grad, ws_bytes,
                            ws))
    return st;
  if (!g_att || (P > 1 && !g_kl)) return OB_ERR_NULL;
  if (reinterpret_cast<uintptr_t>(grad) & 15) return OB_ERR_ALIGN;
  launch_att_kl_bwd(logits, tgt_out, tgt_pad, P, BU, V, label_smoothing, g_att, g_kl, grad, ws,
                    as_stream(stream));
  return launched();
}

int ob_loss_combine_fwd(const float* l_att, const float* l_ctc, const float* l_kl, float gamma,
                        float lambda1, float lambda2, float* loss, float* parts, void* stream) {
  if (!l_att || !l_ctc || !l_kl || !loss || !parts) return OB_ERR_NULL;
  launch_loss_combine_fwd(l_att, l_ctc, l_kl, gamma, lambda1, lambda2, loss, parts,
                          as_stream(stream));
  return launched();
}

int ob_loss_combine_bwd(const float* g_loss, float gamma, float lambda1, float lambda2,
                        float* d_att, float* d_ctc, float* d_kl, void* stream) {
  if (!g_loss || !d_att || !d_ctc || !d_kl) return OB_ERR_NULL;
  launch_loss_combine_bwd(g_loss, gamma, lambda1, lambda2, d_att, d_ctc, d_kl, as_stream(stream));
  return launched();
}

int ob_ctc_greedy_decode(const float* logits, const int64_t* lens, int64_t B, int64_t T,
                         int64_t V, int blank, int32_t* ids, int32_t* out, int32_t* out_len,
                         void* stream) {
  if (B < 0 || T < 0 || V < 1 || V > INT32_MAX || blank < 0 || blank >= V) return OB_ERR_SHAPE;
  if (B > 0 && (!lens || !out_len || (T > 0 && (!logits || !ids || !out)))) return OB_ERR_NULL;
  if (!aligned4(logits) || !aligned4(ids) || !aligned4(out) || !aligned4(out_len))
    return OB_ERR_ALIGN;
  launch_ctc_greedy(logits, lens, B, T, V, blank, reinterpret_cast<int*>(ids),
                    reinterpret_cast<int*>(out), reinterpret_cast<int*>(out_len),
                    as_stream(stream));
  return launched();
}

int ob_layernorm_fwd(const float* x, const float* gamma, const float* beta, int64_t rows,
                     int64_t d, float eps, float* y, float* mean, float* rstd, void* stream) {
  if (rows < 0 || !layernorm_supported(d) || !(eps >= 0.0f)) return OB_ERR_SHAPE;
  if (rows > 0 && (!x || !y)) return OB_ERR_NULL;
  if (!aligned4(x) || !aligned4(y) || !aligned4(gamma) || !aligned4(beta)) return OB_ERR_ALIGN;
  launch_layernorm_fwd(x, gamma, beta, rows, d, eps, y, mean, rstd, as_stream(stream));
  return launched();
}

int ob_layernorm_fwd_pair(const float* x, const float* g1, const float* b1, const float* g2,
                          const float* b2, int64_t rows, int64_t d, float eps1, float eps2,
                          float* y1, float* mean1, float* rstd1, float* y2, float* mean2,
                          float* rstd2, void* stream) {
  if (rows < 0 || !layernorm_supported(d) || !(eps1 >= 0.0f) || !(eps2 >= 0.0f))
    return OB_ERR_SHAPE;
  if (rows > 0 && (!x || !y1 || !y2)) return OB_ERR_NULL;
  if (!aligned4(x) || !aligned4(y1) || !aligned4(y2) || !aligned4(g1) || !aligned4(b1) ||
      !aligned4(g2) || !aligned4(b2))
    return OB_ERR_ALIGN;
  launch_layernorm_fwd_pair(x, g1, b1, g2, b2, rows, d, eps1, eps2, y1, mean1, rstd1, y2, mean2,
                            rstd2, as_stream(stream));
  return launched();
}

size_t ob_layernorm_fwd_amax_workspace(int64_t P) {
  return (P < 1 || P > 8) ? 0 : layernorm_fwd_amax_workspace(P);
}

int ob_layernorm_fwd_amax(const float* x, const float* gamma, const float* beta, int64_t rows,
                          int64_t d, float eps, float* y, float* mean, float* rstd, int64_t P,
                          float* amax, void* ws, size_t ws_bytes, void* stream) {
  if (rows < 0 || !layernorm_supported(d) || !(eps >= 0.0f) || P < 1 || P > 8 || rows % P)
    return OB_ERR_SHAPE;
  if ((rows > 0 && (!x || !y)) || !amax || !ws) return OB_ERR_NULL;
  if (ws_bytes < layernorm_fwd_amax_workspace(P)) return OB_ERR_WORKSPACE;
  if (!aligned4(x) || !aligned4(y) || !aligned4(gamma) || !aligned4(beta) || !aligned4(amax))
    return OB_ERR_ALIGN;
  launch_layernorm_fwd_amax(x, gamma, beta, rows, d, eps, y, mean, rstd, (int)P, amax, ws,
                            as_stream(stream));
  return launched();
}

int ob_layernorm_fwd_i8(const float* x, const float* gamma, const float* beta, int64_t rows,
                        int64_t d, float eps, int64_t P, float* amax, int8_t* yq, void* ws,
                        size_t ws_bytes, void* stream) {
  if (rows < 0 || !layernorm_supported(d) || !(eps >= 0.0f) || P < 1 || P > 8 || rows % P)
    return OB_ERR_SHAPE;
  if ((rows > 0 && (!x || !yq)) || !amax || !ws) return OB_ERR_NULL;
  if (ws_bytes < layernorm_fwd_amax_workspace(P)) return OB_ERR_WORKSPACE;
  if (!aligned4(x) || !aligned4(yq) || !aligned4(gamma) || !aligned4(beta) || !aligned4(amax))
    return OB_ERR_ALIGN;
  launch_layernorm_fwd_i8(x, gamma, beta, rows, d, eps, (int)P, amax, yq, ws, as_stream(stream));
  return launched();
}

size_t ob_layernorm_bwd_workspace(int64_t rows, int64_t d) {
  if (rows < 0 || !layernorm_supported(d)) return 0;
  return layernorm_bwd_workspace(rows, d);
}

int ob_layernorm_bwd(const float* dy, const float* x, const float* gamma, const float* mean,
                     const float* rstd, int64_t rows, int64_t d, float* dx, float* dgamma,
                     float* dbeta, void* ws, size_t ws_bytes, void* stream) {
  if (rows < 0 || !layernorm_supported(d)) return OB_ERR_SHAPE;
  if (rows > 0 && (!dy || !x || !mean || !rstd || !dx)) return OB_ERR_NULL;
  if ((dgamma || dbeta) && !ws) return OB_ERR_NULL;
  if ((dgamma || dbeta) && ws_bytes < layernorm_bwd_workspace(rows, d)) return OB_ERR_WORKSPACE;
  if (!aligned4(dy) || !aligned4(x) || !aligned4(dx)) return OB_ERR_ALIGN;
  launch_layernorm_bwd(dy, x, gamma, mean, rstd, rows, d, nullptr, dx, dgamma, dbeta, ws,
                       as_stream(stream));
  return launched();
}

int ob_layernorm_bwd_res(const float* dy, const float* x, const float* gamma, const float* mean,
                         const float* rstd, int64_t rows, int64_t d, const float* dres, float* dx,
                         float* dgamma, float* dbeta, void* ws, size_t ws_bytes, void* stream) {
  if (rows < 0 || !layernorm_supported(d)) return OB_ERR_SHAPE;
  if (rows > 0 && (!dy || !x || !mean || !rstd || !dx || !dres)) return OB_ERR_NULL;
  if ((dgamma || dbeta) && !ws) return OB_ERR_NULL;
  if ((dgamma || dbeta) && ws_bytes < layernorm_bwd_workspace(rows, d)) return OB_ERR_WORKSPACE;
  if (!aligned4(dy) || !aligned4(x) || !aligned4(dx) || !aligned4(dres)) return OB_ERR_ALIGN;
  launch_layernorm_bwd(dy, x, gamma, mean, rstd, rows, d, dres, dx, dgamma, dbeta, ws,
                       as_stream(stream));
  return launched();
}

int ob_layernorm_bwd_ex(const float* dy, const float* x, const float* gamma, const float* mean,
                        const float* rstd, int64_t rows, int64_t d, const float* dres, float* dx,
                        float* dgamma, float* dbeta, void* ws, size_t ws_bytes, float* dy2,
                        float rscale, float p_drop, const uint64_t* rng, int64_t rng_offset,
                        const int32_t* lens, int64_t T, void* stream) {
  return ob_layernorm_bwd_defer(dy, x, gamma, mean, rstd, rows, d, dres, dx, dgamma, dbeta, ws,
                                ws_bytes, dy2, rscale, p_drop, rng, rng_offset, lens, T, nullptr,
                                0, stream);
}

size_t ob_ln_param_entry_bytes(void) { return sizeof(LnParamEntry); }

int ob_ln_param_table(const void* table, int64_t n, int64_t dmax, void* stream) {
  if (n < 0 || dmax < 0 || dmax > 512) return OB_ERR_SHAPE;
  if (n > 0 && !table) return OB_ERR_NULL;
  launch_ln_param_table(static_cast<const LnParamEntry*>(table), (int)n, (int)dmax,
                        as_stream(stream));
  return launched();
}

size_t ob_layernorm_bwd_pair_workspace(int64_t rows, int64_t d) {
  if (rows < 0 || !layernorm_supported(d)) return 0;
  return 2 * layernorm_bwd_workspace(rows, d);
}

int ob_layernorm_bwd_pair(const float* dy, const float* y1, const float* g2, const float* mean2,
                          const float* rstd2, const float* gres, const float* x, const float* g1,
                          const float* mean1, const float* rstd1, int64_t rows, int64_t d,
                          float* dx, float* dg2, float* db2, float* dg1, float* db1, void* ws,
                          size_t ws_bytes, float* dy2, float rscale, float p_drop,
                          const uint64_t* rng, int64_t rng_offset, const int32_t* lens, int64_t T,
                          void* table, int64_t slot2, int64_t slot1, void* stream) {
  if (rows < 0 || !layernorm_supported(d) || !(p_drop >= 0.0f && p_drop < 1.0f))
    return OB_ERR_SHAPE;
  if (rows > 0 && (!dy || !y1 || !mean2 || !rstd2 || !x || !mean1 || !rstd1 || !dx || !ws))
    return OB_ERR_NULL;
  if (dy2 && p_drop > 0.0f && !rng) return OB_ERR_NULL;
  if (ws_bytes < 2 * layernorm_bwd_workspace(rows, d)) return OB_ERR_WORKSPACE;
  if (!aligned4(dy) || !aligned4(y1) || !aligned4(gres) || !aligned4(x) || !aligned4(dx) ||
      !aligned4(dy2) || !aligned4(g1) || !aligned4(g2) || ((uintptr_t)ws & 15))
    return OB_ERR_ALIGN;
  LnGradScale gsc{dy2, rscale, p_drop, rng, (uint64_t)rng_offset, lens, (int)T};
  LnParamEntry* tab = static_cast<LnParamEntry*>(table);
  const LnDefer f2{tab && slot2 >= 0 ? tab : nullptr, (int)slot2};
  const LnDefer f1{tab && slot1 >= 0 ? tab : nullptr, (int)slot1};
  launch_layernorm_bwd_pair(dy, y1, g2, mean2, rstd2, gres, x, g1, mean1, rstd1, rows, d, dx, dg2,
                            db2, dg1, db1, ws, as_stream(stream), dy2 ? &gsc : nullptr, &f2, &f1);
  return launched();
}

int ob_layernorm_bwd_defer(const float* dy, const float* x, const float* gamma, const float* mean,
                           const float* rstd, int64_t rows, int64_t d, const float* dres,
                           float* dx, float* dgamma, float* dbeta, void* ws, size_t ws_bytes,
                           float* dy2, float rscale, float p_drop, const uint64_t* rng,
                           int64_t rng_offset, const int32_t* lens, int64_t T, void* table,
                           int64_t slot, void* stream) {
  if (table && slot < 0) return OB_ERR_SHAPE;
  if (rows < 0 || !layernorm_supported(d)) return OB_ERR_SHAPE;
  if (rows > 0 && (!dy || !x || !mean || !rstd || !dx)) return OB_ERR_NULL;
  if ((dgamma || dbeta) && !ws) return OB_ERR_NULL;
  if ((dgamma || dbeta) && ws_bytes < layernorm_bwd_workspace(rows, d)) return OB_ERR_WORKSPACE;
  if (!aligned4(dy) || !aligned4(x) || !aligned4(dx) || !aligned4(dres) || !aligned4(dy2) ||
      !aligned4(lens))
    return OB_ERR_ALIGN;
  if (dy2) {
    if (!(p_drop >= 0.0f && p_drop < 1.0f)) return OB_ERR_SHAPE;
    if (lens && (T < 1 || T > 0x7fffffff || rows % T)) return OB_ERR_SHAPE;
    if (p_drop > 0.0f && !rng) return OB_ERR_NULL;
  }
  LnGradScale gs{dy2, rscale, p_drop, rng, (uint64_t)rng_offset,
                 reinterpret_cast<const int*>(lens), (int)T};
  const LnDefer df{static_cast<LnParamEntry*>(table), (int)slot};
  launch_layernorm_bwd(dy, x, gamma, mean, rstd, rows, d, dres, dx, dgamma, dbeta, ws,
                       as_stream(stream), &gs, &df);
  return launched();
}

namespace {
int relattn_check(int64_t Bt, int64_t P, int64_t T, int64_t H, int64_t d, float p_drop) {
  if (Bt < 1 || P < 1 || Bt % P != 0 || H < 1 || !relattn_supported(T, d)) return OB_ERR_SHAPE;
  if (Bt > 65535 || H > 65535 || !(p_drop >= 0.0f && p_drop < 1.0f)) return OB_ERR_SHAPE;
  return OB_OK;
}
}  // namespace

int ob_relattn_fwd(const float* q, const float* k, const float* v, const float* pos,
                   const float* u, const float* vb, const int32_t* lens, int64_t Bt, int64_t P,
                   int64_t T, int64_t H, int64_t d, float p_drop, const int64_t* rng,
                   int64_t rng_offset, float* saved, float* probs, float* ctx, void* stream) {
  if (int st = relattn_check(Bt, P, T, H, d, p_drop)) return st;
  if (!q || !k || !v || !pos || !u || !vb || !lens || !ctx || (p_drop > 0.0f && !rng))
    return OB_ERR_NULL;
  if (((uintptr_t)saved & 15) || ((uintptr_t)probs & 15)) return OB_ERR_ALIGN;
  launch_relattn_fwd(q, k, v, pos, u, vb, lens, Bt, P, T, H, d, p_drop,
                     reinterpret_cast<const uint64_t*>(rng), (uint64_t)rng_offset, saved, probs,
                     ctx, as_stream(stream));
  return launched();
}

int64_t ob_relattn_saved_elems(int64_t Bt, int64_t T, int64_t H, int64_t d) {
  if (Bt < 1 || H < 1 || !relattn_supported(T, d)) return 0;
  return relattn_saved_elems(Bt, T, H, d);
}

size_t ob_relattn_bwd_workspace(int64_t Bt, int64_t T, int64_t H, int64_t d) {
  if (Bt < 1 || H < 1 || !relattn_supported(T, d)) return 0;
  return align_up(relattn_bwd_workspace(Bt, T, H, d));
}

int ob_relattn_set_bwd_mode(int mode) { return relattn_set_flash(mode); }

int64_t ob_relattn_probs_elems(int64_t Bt, int64_t T, int64_t H) {
  if (Bt < 1 || H < 1 || T < 1) return 0;
  return relattn_probs_elems(Bt, T, H);
}

int ob_relattn_bwd(const float* dctx, const float* ctx, const float* q, const float* k,
                   const float* v, const float* pos, const float* u, const float* vb,
                   const int32_t* lens, int64_t Bt, int64_t P, int64_t T, int64_t H, int64_t d,
                   float p_drop, const int64_t* rng, int64_t rng_offset, const float* saved,
                   int64_t saved_elems, float* dq, float* dk, float* dv, float* dpos, float* du,
                   float* dvb, void* ws, size_t ws_bytes, void* stream) {
  if (int st = relattn_check(Bt, P, T, H, d, p_drop)) return st;
  if (!dctx || !ctx || !q || !k || !v || !pos || !u || !vb || !lens || !saved || !dq || !dk ||
      !dv || !dpos || !du || !dvb || !ws)
    return OB_ERR_NULL;
  // `saved` laid out under the other backward mode (ob_relattn_set_bwd_mode in between)
  if (saved_elems != relattn_saved_elems(Bt, T, H, d)) return OB_ERR_SHAPE;
  (void)rng;  // the forward's keep decisions are in the saved state
  (void)rng_offset;
  if ((uintptr_t)saved & 15) return OB_ERR_ALIGN;
  if (ws_bytes < ob_relattn_bwd_workspace(Bt, T, H, d)) return OB_ERR_WORKSPACE;
  launch_relattn_bwd(dctx, ctx, q, k, v, pos, u, vb, lens, Bt, P, T, H, d, p_drop, saved, dq, dk,
                     dv, dpos, du, dvb, ws, as_stream(stream));
  return launched();
}

int ob_decattn_supported(int64_t Lq, int64_t Lk, int64_t dh) {
  return decattn_supported(Lq, Lk, dh) ? 1 : 0;
}

static int decattn_check(int64_t B, int64_t H, int64_t Lq, int64_t Lk, int64_t dh, int64_t sq,
                         int64_t sk, int64_t sv, float p_drop) {
  if (B < 0 || H < 1 || !decattn_supported(Lq, Lk, dh) || !(p_drop >= 0.0f && p_drop < 1.0f))
    return OB_ERR_SHAPE;
  if (sq < H * dh || sk < H * dh || sv < H * dh) return OB_ERR_SHAPE;
  if (B * H * Lq > INT32_MAX) return OB_ERR_SHAPE;
  return OB_OK;
}

int ob_decattn_fwd(const float* q, int64_t sq, const float* k, int64_t sk, const float* v,
                   int64_t sv, const uint8_t* kmask, int64_t causal, int64_t B, int64_t H,
                   int64_t Lq, int64_t Lk, int64_t dh, float p_drop, const int64_t* rng,
                   int64_t rng_offset, float* probs, float* ctx, void* stream) {
  if (int st = decattn_check(B, H, Lq, Lk, dh, sq, sk, sv, p_drop)) return st;
  if (B > 0 && (!q || !k || !v || !probs || !ctx || (p_drop > 0.0f && !rng))) return OB_ERR_NULL;
  if (!aligned4(q) || !aligned4(k) || !aligned4(v) || !aligned4(probs) ||
      (reinterpret_cast<uintptr_t>(ctx) & 15))
    return OB_ERR_ALIGN;
  launch_decattn_fwd(q, sq, k, sk, v, sv, kmask, causal ? 1 : 0, B, H, Lq, Lk, dh, p_drop,
                     reinterpret_cast<const uint64_t*>(rng), (uint64_t)rng_offset, probs, ctx,
                     as_stream(stream));
  return launched();
}

int ob_decattn_bwd(const float* dctx, const float* ctx, const float* q, int64_t sq, const float* k,
                   int64_t sk, const float* v, int64_t sv, int64_t B, int64_t H, int64_t Lq, int64_t Lk,
                   int64_t dh, float p_drop, float* probs, float* dq, int64_t gq, float* dk,
                   int64_t gk, float* dv, int64_t gv, void* stream) {
  if (int st = decattn_check(B, H, Lq, Lk, dh, sq, sk, sv, p_drop)) return st;
  if (gq < H * dh || gk < H * dh || gv < H * dh) return OB_ERR_SHAPE;
  if (B > 0 && (!dctx || !ctx || !q || !k || !v || !probs || !dq || !dk || !dv)) return OB_ERR_NULL;
  if (!aligned4(ctx) || !aligned4(dctx) || !aligned4(q) || !aligned4(k) || !aligned4(v) || !aligned4(probs) ||
      !aligned4(dq) || !aligned4(dk) || !aligned4(dv))
    return OB_ERR_ALIGN;
  launch_decattn_bwd(dctx, ctx, q, sq, k, sk, v, sv, B, H, Lq, Lk, dh, p_drop, probs, dq, gq, dk, gk,
                     dv, gv, as_stream(stream));
  return launched();
}

int ob_relattn_dropout_mask(int64_t n, int64_t row_len, float p_drop, const int64_t* rng,
                            int64_t rng_offset, uint8_t* out, void* stream) {
  if (n < 0 || row_len < 1 || !(p_drop >= 0.0f && p_drop < 1.0f)) return OB_ERR_SHAPE;
  if ((n > 0 && !out) || (p_drop > 0.0f && !rng)) return OB_ERR_NULL;
  launch_relattn_dropout_mask(n, row_len, p_drop, reinterpret_cast<const uint64_t*>(rng),
                              (uint64_t)rng_offset, out, as_stream(stream));
  return launched();
}

int ob_embedding_bwd(const int64_t* indices, int64_t N, const float* grad, int64_t C,
                     int64_t V, int64_t padding_idx, float* grad_weight, void* stream) {
  if (N < 0 || V < 0 || !embed_supported(C) || padding_idx >= V) return OB_ERR_SHAPE;
  if ((N > 0 && (!indices || !grad)) || (V > 0 && !grad_weight)) return OB_ERR_NULL;
  if (!aligned4(grad) || !aligned4(grad_weight)) return OB_ERR_ALIGN;
  launch_embed_bwd(indices, N, grad, C, V, padding_idx, grad_weight, as_stream(stream));
  return launched();
}

int64_t ob_adamw_plan(const int64_t* numels, int64_t n_tensors, int64_t* chunk_map) {
  if (!numels || n_tensors < 1) return OB_ERR_SHAPE;
  for (int64_t t = 0; t < n_tensors; ++t)
    if (numels[t] < 1) return OB_ERR_SHAPE;
  return adamw_plan(numels, n_tensors, chunk_map);
}

size_t ob_adamw_workspace(int64_t n_blocks) {
  if (n_blocks < 1) return 0;
  return align_up(adamw_workspace(n_blocks));
}

int ob_adamw_clip_step(const ob_adamw_tensor* table, int64_t n_tensors, const int64_t* chunk_map,
                       int64_t n_blocks, const float* lr, float* step, float grad_scale,
                       double beta1, double beta2, double eps, double weight_decay,
                       double max_norm, float* total_norm,
                       void* ws, size_t ws_bytes, void* stream) {
  static_assert(sizeof(ob_adamw_tensor) == sizeof(AdamwTensor), "table layout");
  if (n_tensors < 1 || n_blocks < 1 || n_blocks > 0x7fffffff) return OB_ERR_SHAPE;
  if (!table || !chunk_map || !lr || !step || !ws) return OB_ERR_NULL;
  if (ws_bytes < ob_adamw_workspace(n_blocks)) return OB_ERR_WORKSPACE;
  launch_adamw(reinterpret_cast<const AdamwTensor*>(table), chunk_map, n_blocks, lr, step,
               grad_scale, beta1, beta2, eps, weight_decay, max_norm, total_norm, ws,
               as_stream(stream));
  return launched();
}

}  // extern "C"
