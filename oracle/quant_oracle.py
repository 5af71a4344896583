"""CPU oracle for the BitLinear hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg import this
module. It is the checker, never the product: the product path is libonebit_hip.so.

Three restatements of y00njaekim/CMU-11785-IDL-1.58bit-ASR ``onebit_asr/quant.py``:

* ``np_*``   numpy, vectorised, fp32 operation order of quant.py:49-91;
* ``c_*``    the C twin in quant_oracle.c (built by ``make -C oracle``);
* ``TorchRefQuantizedLinear`` / ``ref_quantize_weight``: plain-PyTorch fp32 autograd
  restatement (quant.py:38-127) — the fp32 reference for the float kernels.

Parity anchor: the reference ships no golden vectors or known-answer tests for this path
(SURVEY.md §4, §8c), and importing/running it here was denied. The
restatements are pinned by hand-derived known answers in tests/golden/quant_kat.json and by
agreeing with each other (tests/test_oracle.py); the model-level restatement
(conformer_oracle.py) is pinned by tests/golden/model_kat.json (tests/test_model_kat.py).
"""
from __future__ import annotations

import ctypes
import math
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
C_LIB_PATH = HERE / "build" / "liborc_quant.so"

EPS = np.float32(1e-8)


# ----------------------------------------------------------------------------- numpy
def np_effective_alpha(alpha: float, alpha_raw: bool = True) -> np.float32:
    a = np.float32(alpha)
    return np.float32(np.abs(a) + EPS) if alpha_raw else a  # quant.py:124


def np_quant_q(W: np.ndarray, alpha: float, bits: int, alpha_raw: bool = True) -> np.ndarray:
    """Q in {-1,0,+1} as float32 (quant.py:49-60)."""
    if bits not in (1, 2):
        raise ValueError("bitwidth must be one of {1,2,32}")
    a = np_effective_alpha(alpha, alpha_raw)
    wa = (np.asarray(W, np.float32) / a).astype(np.float32)
    c = np.clip(wa, np.float32(-1), np.float32(1))
    if bits == 1:
        q = np.sign(c)
        q[q == 0] = 1.0
        return q.astype(np.float32)
    return np.where(np.abs(c) < np.float32(0.5), np.float32(0), np.sign(c)).astype(np.float32)


def np_codes(W: np.ndarray, alpha: float, bits: int, alpha_raw: bool = True):
    """Device code words (include/onebit_hip.h): codes [N][ceil(K/16)], codes_t [K][ceil(N/16)]."""
    q = np_quant_q(W, alpha, bits, alpha_raw)
    n, k = q.shape
    c = np.where(q > 0, 1, np.where(q < 0, 3, 0)).astype(np.uint64)

    def pack_rows(cm: np.ndarray) -> np.ndarray:
        rows, cols = cm.shape
        words = (cols + 15) // 16
        padded = np.zeros((rows, words * 16), np.uint64)
        padded[:, :cols] = cm
        shifts = (2 * np.arange(16, dtype=np.uint64))[None, None, :]
        return (padded.reshape(rows, words, 16) << shifts).sum(-1).astype(np.uint32)

    return pack_rows(c), pack_rows(c.T.copy())


def np_term(wa: np.ndarray, bits: int) -> np.ndarray:
    """quant.py:86-90."""
    awa = np.abs(wa)
    s = np.sign(wa).astype(np.float32)
    piece = np.where(awa >= np.float32(0.5), s, np.float32(0)) if bits == 2 else s
    inner = (-wa + piece).astype(np.float32)
    return np.where(awa < np.float32(1), inner, s).astype(np.float32)


def np_ste_bwd(g: np.ndarray, W: np.ndarray, alpha: float, bits: int, alpha_raw: bool = True):
    """(grad_W fp32, grad_alpha as float64 sum of the fp32 products) — quant.py:80-91,
    chained through alpha.abs() when alpha_raw."""
    a = np_effective_alpha(alpha, alpha_raw)
    wa = (np.asarray(W, np.float32) / a).astype(np.float32)
    g = np.asarray(g, np.float32)
    ind = (np.abs(wa) <= np.float32(1)).astype(np.float32)
    gw = (g * ind).astype(np.float32)
    prod = (g * np_term(wa, bits)).astype(np.float32)
    ga = float(prod.astype(np.float64).sum())
    if alpha_raw:
        ga *= float(np.sign(np.float32(alpha)))
    return gw, ga


def np_bitlinear_fwd(X: np.ndarray, W: np.ndarray, alpha: float, bias, bits: int,
                     alpha_raw: bool = True) -> np.ndarray:
    """Y = X . (a*Q)^T + b in float64 (summation-order-free reference)."""
    a = np_effective_alpha(alpha, alpha_raw)
    w_hat = (a * np_quant_q(W, alpha, bits, alpha_raw)).astype(np.float32)
    y = np.asarray(X, np.float64) @ w_hat.astype(np.float64).T
    if bias is not None:
        y = y + np.asarray(bias, np.float64)
    return y


# ----------------------------------------------------------------------------- C twin
_clib = None


# ------------------------------------------------------ opt-in int8 activation mode
# NOT reference arithmetic (the reference keeps activations fp32, quant.py:126; SURVEY.md
# §0 F3). This restates the north-star mode the HIP path implements
# (cmu-11785-idl-1.58bit-asr_amd/csrc/tgemm_i8.hip) so it can be checked bit-exactly:
# BitNet-b1.58 per-tensor absmax activations, then the reference's F.linear with W_hat.
def np_act_quant_i8(X: np.ndarray):
    """(xq int32, gamma f32): gamma = max(max|X|, 1e-5), xq = clamp(rint(X * (127/gamma)))."""
    X = np.asarray(X, np.float32)
    gam = np.float32(max(np.float32(np.abs(X).max()) if X.size else np.float32(0), np.float32(1e-5)))
    sx = np.float32(np.float32(127.0) / gam)
    xq = np.clip(np.rint((X * sx).astype(np.float32)), -127, 127).astype(np.int32)
    return xq, gam


def np_act_dequant_i8(X: np.ndarray) -> np.ndarray:
    xq, gam = np_act_quant_i8(X)
    return (xq.astype(np.float32) * np.float32(gam / np.float32(127.0))).astype(np.float32)


def np_bitlinear_fwd_i8(X: np.ndarray, W: np.ndarray, alpha: float, bias, bits: int,
                        alpha_raw: bool = True) -> np.ndarray:
    """Y = float(xq . Q^T) * (a * (gamma/127)) + b, each op rounded once in fp32."""
    xq, gam = np_act_quant_i8(X)
    q = np_quant_q(W, alpha, bits, alpha_raw).astype(np.int64)
    acc = (xq.astype(np.int64) @ q.T).astype(np.float32)  # exact integers (< 2^24)
    osc = np.float32(np_effective_alpha(alpha, alpha_raw) * np.float32(gam / np.float32(127.0)))
    y = (acc * osc).astype(np.float32)
    if bias is not None:
        y = (y + np.asarray(bias, np.float32)).astype(np.float32)
    return y


def c_lib() -> ctypes.CDLL:
    global _clib
    if _clib is None:
        if not C_LIB_PATH.is_file():
            raise RuntimeError(f"{C_LIB_PATH} missing: run `make -C oracle`")
        lib = ctypes.CDLL(str(C_LIB_PATH))
        P = ctypes.c_void_p
        I64, F, I = ctypes.c_int64, ctypes.c_float, ctypes.c_int
        lib.orc_quant_q.argtypes = [P, I64, F, I, I, P]
        lib.orc_quant_dequant.argtypes = [P, I64, F, I, I, P]
        lib.orc_quant_pack.argtypes = [P, I64, I64, F, I, I, P, P]
        lib.orc_ste_bwd.argtypes = [P, P, I64, F, I, I, P, P, P]
        lib.orc_bitlinear_fwd.argtypes = [P, I64, I64, P, I64, F, I, I, P, P]
        for fn in (lib.orc_quant_q, lib.orc_quant_dequant, lib.orc_quant_pack, lib.orc_ste_bwd,
                   lib.orc_bitlinear_fwd):
            fn.restype = I
        _clib = lib
    return _clib


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def c_quant_q(W, alpha, bits, alpha_raw=True) -> np.ndarray:
    W = np.ascontiguousarray(W, np.float32)
    q = np.empty(W.shape, np.int8)
    st = c_lib().orc_quant_q(_p(W), W.size, float(alpha), int(alpha_raw), bits, _p(q))
    if st:
        raise ValueError("bitwidth must be one of {1,2,32}")
    return q


def c_codes(W, alpha, bits, alpha_raw=True):
    W = np.ascontiguousarray(W, np.float32)
    n, k = W.shape
    codes = np.empty((n, (k + 15) // 16), np.uint32)
    codes_t = np.empty((k, (n + 15) // 16), np.uint32)
    st = c_lib().orc_quant_pack(_p(W), n, k, float(alpha), int(alpha_raw), bits, _p(codes), _p(codes_t))
    if st:
        raise ValueError("bitwidth must be one of {1,2,32}")
    return codes, codes_t


def c_ste_bwd(g, W, alpha, bits, alpha_raw=True):
    g = np.ascontiguousarray(g, np.float32)
    W = np.ascontiguousarray(W, np.float32)
    gw = np.empty_like(W)
    ga64 = ctypes.c_double(0.0)
    ga32 = ctypes.c_float(0.0)
    st = c_lib().orc_ste_bwd(_p(g), _p(W), W.size, float(alpha), int(alpha_raw), bits, _p(gw),
                             ctypes.byref(ga64), ctypes.byref(ga32))
    if st:
        raise ValueError("bitwidth must be one of {1,2,32}")
    return gw, ga64.value, ga32.value


def c_bitlinear_fwd(X, W, alpha, bias, bits, alpha_raw=True) -> np.ndarray:
    X = np.ascontiguousarray(X, np.float32)
    W = np.ascontiguousarray(W, np.float32)
    m, k = X.shape
    n = W.shape[0]
    y = np.empty((m, n), np.float64)
    b = None if bias is None else np.ascontiguousarray(bias, np.float32)
    st = c_lib().orc_bitlinear_fwd(_p(X), m, k, _p(W), n, float(alpha), int(alpha_raw), bits,
                                   None if b is None else _p(b), _p(y))
    if st:
        raise ValueError("bitwidth must be one of {1,2,32}")
    return y


# ----------------------------------------------------------------------------- torch fp32
# Test hook (tests/test_conformer_s_oracle_gpu.py): when a dict, every backward adds the
# float64 sum of |grad_out * term| -- the magnitude of the terms the alpha gradient sums,
# the natural scale of its rounding error -- under id(W) of the layer's weight.
TERM_SCALE = None


class _RefQuantizeSTE(torch.autograd.Function):
    """quant.py:38-92 in plain torch fp32 ops (CPU)."""

    @staticmethod
    def forward(ctx, W, alpha, bitwidth: int):
        ctx.key = id(W)
        if bitwidth == 32:
            ctx.bits = 32
            return W
        if bitwidth not in (1, 2):
            raise ValueError("bitwidth must be one of {1,2,32}")
        wa = W / alpha
        clipped = wa.clamp(-1.0, 1.0)
        if bitwidth == 1:
            q = clipped.sign()
            q = torch.where(q == 0, torch.ones_like(q), q)
        else:
            q = torch.where(clipped.abs() < 0.5, torch.zeros_like(clipped), clipped.sign())
        ctx.bits = bitwidth
        ctx.save_for_backward(wa)
        return alpha * q

    @staticmethod
    def backward(ctx, grad_out):
        if ctx.bits == 32:
            return grad_out, grad_out.new_zeros(()), None
        (wa,) = ctx.saved_tensors
        awa = wa.abs()
        grad_w = grad_out * (awa <= 1.0).to(grad_out.dtype)
        s = wa.sign()
        piece = torch.where(awa >= 0.5, s, torch.zeros_like(wa)) if ctx.bits == 2 else s
        term = torch.where(awa < 1.0, -wa + piece, s)
        prod = grad_out * term
        if TERM_SCALE is not None:
            TERM_SCALE[ctx.key] = TERM_SCALE.get(ctx.key, 0.0) + prod.abs().double().sum().item()
        return grad_w, prod.sum(), None


def ref_quantize_weight(W, alpha, bitwidth):
    return _RefQuantizeSTE.apply(W, alpha, bitwidth)


def ref_quantized_linear(x, weight, alpha, bias, bitwidth):
    """QuantizedLinear.forward (quant.py:120-127) in torch fp32 on whatever device x is."""
    if bitwidth == 32:
        return torch.nn.functional.linear(x, weight, bias)
    w_used = ref_quantize_weight(weight, alpha.abs() + 1e-8, bitwidth)
    return torch.nn.functional.linear(x, w_used, bias)


def ref_layer_init(in_features: int, out_features: int, generator: torch.Generator):
    """Parameters distributed as QuantizedLinear.__init__ (quant.py:100-118): W ~ U(-2/sqrt(in),
    2/sqrt(in)) (kaiming_uniform a=sqrt(5), then x2), alpha = mean|W|, bias zeros."""
    bound = 2.0 / math.sqrt(in_features)
    w = (torch.rand(out_features, in_features, generator=generator) * 2 - 1) * bound
    return w, w.abs().mean(), torch.zeros(out_features)
