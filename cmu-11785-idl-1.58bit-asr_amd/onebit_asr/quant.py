"""BitLinear / QuantizedLinear on MI355X: the reference's layer surface over HIP kernels.

Reference surface kept verbatim (onebit_asr/quant.py of y00njaekim/CMU-11785-IDL-1.58bit-ASR):

* ``QuantizedLinear(in_features, out_features, bias=True)`` with parameters ``weight``
  ``[out, in]``, ``alpha`` (0-dim) and ``bias`` ``[out]`` -- the checkpoint keys
  (quant.py:99-118, eval.py:282);
* ``QuantizedLinear.forward(x, bitwidth)`` with ``bitwidth`` in {1, 2, 32}
  (quant.py:120-127);
* ``quantize_weight(W, alpha, bitwidth)`` and ``_QuantizeSTE`` (quant.py:38-96);
* ``ValueError("bitwidth must be one of {1,2,32}")`` for any other bitwidth (quant.py:65-66).

What changes is the execution: for bitwidth 1/2 the layer never materialises
``W_hat = alpha * Q``. One launch packs W into 2-bit codes (cached per weight version,
so the three passes of a training step share it), one launch runs the ternary GEMM
with the scale and bias in its epilogue, and the backward is one dX GEMM plus one
split-M dW GEMM whose reduction applies the STE mask and the alpha gradient
(quant.py:72-92) in the same pass. The bitwidth is a Python int: there is no
``torch.tensor(bitwidth)`` H2D copy per call and no ``.item()`` sync in backward
(quant.py:69,75).

bitwidth 32 stays ``F.linear`` on the weight, as in the reference (quant.py:121-122).
There is no CPU path for bitwidth 1/2: the oracle under ``oracle/`` is the checker.
"""
from __future__ import annotations

import ctypes
import math
from typing import Optional

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib, deferred
from .linear import linear

__all__ = ["QuantizedLinear", "BitLinear", "quantize_weight", "pack_codes", "set_quant_off", "DeviceBits",
           "DynamicBitwidth", "PassBits", "StackedBits", "set_act_quant", "ACT_QUANT_MODES",
           "act_absmax", "PackGroup"]

_VALID = (1, 2, 32)


class DynamicBitwidth:
    """A BitLinear bitwidth (1 or 2) that lives on the device: slot `index` of an int32
    tensor. Used for the stochastic-precision pass under HIP-graph capture, where the
    per-block bitwidths change every step but the captured graph must not
    (reference train.py:102-103, conformer.py:265-269)."""

    __slots__ = ("tensor", "index")

    def __init__(self, tensor: torch.Tensor, index: int):
        self.tensor = tensor
        self.index = index

    def ptr(self) -> int:
        return self.tensor.data_ptr() + 4 * self.index


class DeviceBits:
    """Per-block SP bitwidths on device. ``set(sp_mask)`` stages a new mask (1 -> 1-bit,
    else 2-bit, as conformer.py:268) with an async H2D copy; ``[i]`` is block i's
    DynamicBitwidth. It stands in for the reference's ``sp_mask`` list."""

    def __init__(self, n_layers: int, device):
        self.n_layers = n_layers
        self.tensor = torch.full((n_layers,), 2, dtype=torch.int32, device=device)

    def set(self, sp_mask) -> None:
        host = torch.tensor([1 if m == 1 else 2 for m in sp_mask], dtype=torch.int32)
        if self.tensor.is_cuda:
            host = host.pin_memory()
        self.tensor.copy_(host, non_blocking=True)

    def __getitem__(self, i: int) -> DynamicBitwidth:
        return DynamicBitwidth(self.tensor, i)

    def __len__(self) -> int:
        return self.n_layers


class PassBits:
    """Bitwidths of P stacked passes of one layer call: the reference's teacher (2-bit),
    student (1-bit) and stochastic-precision passes (train.py:82-105) run as ONE call on
    inputs stacked along the batch, pass p at bitwidth ``tensor[p]`` (DEVICE int32 [P],
    1 or 2). The layer then needs one launch per kernel instead of one per pass, and its
    parameter gradients are summed inside the kernels rather than by autograd."""

    __slots__ = ("tensor",)

    def __init__(self, tensor: torch.Tensor):
        if tensor.dtype != torch.int32 or tensor.dim() != 1:
            raise TypeError("PassBits wants a 1-D int32 device tensor")
        self.tensor = tensor

    @property
    def passes(self) -> int:
        return self.tensor.numel()


class StackedBits:
    """Per-block ``PassBits`` of the training step's three stacked passes: column 0 the
    2-bit teacher, column 1 the 1-bit student, column 2 the SP pass (1 where sp_mask[i]
    == 1, else 2; conformer.py:265-269, train.py:102-103). ``set(sp_mask)`` rewrites the
    device table with one async copy, so a captured step replays with the new mask."""

    passes = 3

    def __init__(self, n_layers: int, device):
        self.n_layers = n_layers
        self.tensor = torch.tensor([[2, 1, 2]] * n_layers, dtype=torch.int32, device=device)

    def set(self, sp_mask) -> None:
        if len(sp_mask) != self.n_layers:
            raise ValueError(f"sp_mask has {len(sp_mask)} entries for {self.n_layers} blocks")
        host = torch.tensor([[2, 1, 1 if m == 1 else 2] for m in sp_mask], dtype=torch.int32)
        if self.tensor.is_cuda:
            host = host.pin_memory()
        self.tensor.copy_(host, non_blocking=True)

    def __getitem__(self, i: int) -> "PassBits":
        return PassBits(self.tensor[i])

    def __len__(self) -> int:
        return self.n_layers


def _check_bitwidth(bitwidth) -> int:
    if isinstance(bitwidth, DynamicBitwidth):
        return 0
    if bitwidth not in _VALID:
        raise ValueError("bitwidth must be one of {1,2,32}")
    return int(bitwidth)


ACT_QUANT_MODES = (None, "absmax_int8")


def _check_act_quant(mode):
    if mode not in ACT_QUANT_MODES:
        raise ValueError(f"act_quant must be one of {ACT_QUANT_MODES}, got {mode!r}")
    return mode


def set_act_quant(module: nn.Module, mode: Optional[str]) -> nn.Module:
    """Switch every QuantizedLinear under ``module`` to activation mode ``mode``."""
    _check_act_quant(mode)
    for m in module.modules():
        if isinstance(m, QuantizedLinear):
            m.act_quant = mode
        if getattr(m, "int8_ln", False) and hasattr(getattr(m, "ln", None), "emit_amax"):
            m.ln.emit_amax = mode == "absmax_int8"
    return module


def set_quant_off(module: nn.Module, dtype=torch.bfloat16) -> nn.Module:
    """BASELINE configs[3]: every QuantizedLinear under ``module`` becomes a plain linear
    layer whatever the bitwidth; ``alpha`` then receives no gradient. ``None`` restores the
    BitLinear path. The reference has no such mode (its bitwidth 32 is fp32 F.linear,
    quant.py:121-122); this is the measurement ceiling for the ternary kernels, not a
    parity path.
    * a torch dtype (bf16): ``F.linear`` in that dtype on the library GEMMs (hipBLASLt);
    * ``"bf16w"``: the SAME fused call sites and kernels as the ternary path with the weight
      operand bf16(W) instead of the 2-bit codes (alpha_raw 2/3 of include/onebit_hip.h;
      activations exact fp32) and a plain dense dW -- only the weight format differs, so
      the comparison with the 1.58-bit step isolates it."""
    if dtype is not None and dtype != "bf16w" and not isinstance(dtype, torch.dtype):
        raise ValueError(f"quant_off must be None, a torch dtype or 'bf16w', got {dtype!r}")
    for m in module.modules():
        if isinstance(m, QuantizedLinear):
            m.quant_off = dtype
    return module


_ONE_PASS = {}  # device index -> int32 [1] pass_bits of a one-pass quant-off call


def _require_device(*tensors: torch.Tensor) -> None:
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise RuntimeError(
                "BitLinear bitwidth 1/2 runs only on a ROCm device (HIP kernels, no CPU "
                "fallback); move the module and inputs to 'cuda'"
            )
        if t is not None and t.dtype != torch.float32:
            raise TypeError(f"BitLinear parity path computes in fp32, got {t.dtype}")


def pack_codes(weight: torch.Tensor, alpha: torch.Tensor, bits, alpha_raw: bool = True):
    """2-bit codes of Q(W / a): ``codes [N, ceil(K/16)]`` and ``codes_t [K, ceil(N/16)]``
    (int32 views of the uint32 words described in include/onebit_hip.h). ``bits`` is 1, 2 or
    a DynamicBitwidth (read on device)."""
    _require_device(weight, alpha)
    n, k = weight.shape
    w = weight.detach().contiguous()
    codes = torch.empty((n, (k + 15) // 16), dtype=torch.int32, device=w.device)
    codes_t = torch.empty((k, (n + 15) // 16), dtype=torch.int32, device=w.device)
    lib = _lib.load()
    if isinstance(bits, DynamicBitwidth):
        st = lib.ob_quant_pack_dyn(w.data_ptr(), alpha.data_ptr(), int(alpha_raw), bits.ptr(), n, k,
                                   codes.data_ptr(), codes_t.data_ptr(), _lib.stream_of(w))
    else:
        st = lib.ob_quant_pack(w.data_ptr(), alpha.data_ptr(), int(alpha_raw), bits, n, k,
                               codes.data_ptr(), codes_t.data_ptr(), _lib.stream_of(w))
    _lib.check(st, "ob_quant_pack")
    return codes, codes_t


class _BitLinearFn(torch.autograd.Function):
    """y = |alpha|_eps * (x . Q^T) + b with STE backward (quant.py:44-92 + F.linear)."""

    @staticmethod
    def forward(ctx, x2d, weight, alpha, bias, bits, codes, codes_t):
        m, k = x2d.shape
        n = weight.shape[0]
        y = torch.empty((m, n), dtype=torch.float32, device=x2d.device)
        lib = _lib.load()
        _lib.check(
            lib.ob_bitlinear_fwd(x2d.data_ptr(), m, k, codes.data_ptr(), alpha.data_ptr(), 1,
                                 _lib.ptr(bias), n, y.data_ptr(), _lib.stream_of(x2d)),
            "ob_bitlinear_fwd",
        )
        ctx.bits = bits
        ctx.has_bias = bias is not None
        ctx.save_for_backward(x2d, weight, alpha, codes_t)
        return y

    @staticmethod
    def backward(ctx, gy):
        x2d, weight, alpha, codes_t = ctx.saved_tensors
        gy = gy.contiguous()
        m, k = x2d.shape
        n = weight.shape[0]
        lib = _lib.load()
        stream = _lib.stream_of(gy)
        gx = gw = galpha = gb = None
        if ctx.needs_input_grad[0]:
            gx = torch.empty((m, k), dtype=torch.float32, device=gy.device)
            _lib.check(
                lib.ob_bitlinear_bwd_dx(gy.data_ptr(), m, n, codes_t.data_ptr(),
                                        alpha.data_ptr(), 1, k, gx.data_ptr(), stream),
                "ob_bitlinear_bwd_dx",
            )
        if ctx.needs_input_grad[1] or ctx.needs_input_grad[2] or ctx.needs_input_grad[3]:
            gw = torch.empty_like(weight)
            galpha = torch.empty((), dtype=torch.float32, device=gy.device)
            gb = torch.empty((n,), dtype=torch.float32, device=gy.device) if ctx.has_bias else None
            ws_bytes = lib.ob_bitlinear_bwd_dw_workspace(m, n, k)
            ws = torch.empty((max(ws_bytes, 1),), dtype=torch.uint8, device=gy.device)
            if isinstance(ctx.bits, DynamicBitwidth):
                st = lib.ob_bitlinear_bwd_dw_dyn(gy.data_ptr(), x2d.data_ptr(), m, n, k,
                                                 weight.data_ptr(), alpha.data_ptr(), 1,
                                                 ctx.bits.ptr(), gw.data_ptr(), galpha.data_ptr(),
                                                 _lib.ptr(gb), ws.data_ptr(), ws_bytes, stream)
            else:
                st = lib.ob_bitlinear_bwd_dw(gy.data_ptr(), x2d.data_ptr(), m, n, k,
                                             weight.data_ptr(), alpha.data_ptr(), 1, ctx.bits,
                                             gw.data_ptr(), galpha.data_ptr(), _lib.ptr(gb),
                                             ws.data_ptr(), ws_bytes, stream)
            _lib.check(st, "ob_bitlinear_bwd_dw")
            if not ctx.needs_input_grad[1]:
                gw = None
            if not ctx.needs_input_grad[2]:
                galpha = None
        return gx, gw, galpha, gb, None, None, None


class _BitLinearPassesFn(torch.autograd.Function):
    """P stacked passes (rows p*M .. p*M+M at bitwidth pass_bits[p]) in one call each for
    fwd, dX and dW (include/onebit_hip.h, "Stacked passes")."""

    @staticmethod
    def forward(ctx, x2d, weight, alpha, bias, pass_bits, P, codes2, codes2_t, codes1, codes1_t):
        rows, k = x2d.shape
        m = rows // P
        n = weight.shape[0]
        y = torch.empty((rows, n), dtype=torch.float32, device=x2d.device)
        lib = _lib.load()
        # int16 "codes" = bf16 weight images: the quant-off ceiling (alpha_raw 2, dense dW)
        ctx.dense = codes2.dtype == torch.int16
        _lib.check(
            lib.ob_bitlinear_fwd_passes(x2d.data_ptr(), P, m, k, codes2.data_ptr(), codes1.data_ptr(),
                                        pass_bits.data_ptr(), alpha.data_ptr(),
                                        2 if ctx.dense else 1, _lib.ptr(bias), n, y.data_ptr(),
                                        _lib.stream_of(x2d)),
            "ob_bitlinear_fwd_passes",
        )
        ctx.P = P
        ctx.has_bias = bias is not None
        ctx.bias = bias
        deferred.note(weight, alpha, bias)
        ctx.save_for_backward(x2d, weight, alpha, pass_bits, codes2_t, codes1_t)
        return y

    @staticmethod
    def backward(ctx, gy):
        x2d, weight, alpha, pass_bits, codes2_t, codes1_t = ctx.saved_tensors
        gy = gy.contiguous()
        rows, k = x2d.shape
        P = ctx.P
        m = rows // P
        n = weight.shape[0]
        lib = _lib.load()
        stream = _lib.stream_of(gy)
        gx = gw = galpha = gb = None
        if ctx.needs_input_grad[0]:
            gx = torch.empty((rows, k), dtype=torch.float32, device=gy.device)
            _lib.check(
                lib.ob_bitlinear_bwd_dx_passes(gy.data_ptr(), P, m, n, codes2_t.data_ptr(),
                                               codes1_t.data_ptr(), pass_bits.data_ptr(),
                                               alpha.data_ptr(), 2 if ctx.dense else 1, k,
                                               gx.data_ptr(), stream),
                "ob_bitlinear_bwd_dx_passes",
            )
        if ctx.dense and (ctx.needs_input_grad[1] or ctx.needs_input_grad[3]):
            wsb = lib.ob_dense_dw_workspace(rows, n, k)
            if wsb and gy.data_ptr() % 16 == 0 and x2d.data_ptr() % 16 == 0:
                gw = deferred.grad_buf(weight)
                gb = deferred.grad_buf(ctx.bias, (n,), gy.device) if ctx.has_bias else None
                ws = torch.empty((wsb,), dtype=torch.uint8, device=gy.device)
                deferred.dense_dw(gy, x2d, rows, n, k, gw, gb, ws, wsb, stream, weight, ctx.bias)
            else:  # shapes off the dW kernels (N or K not a multiple of 48): library fp32
                from .linear import colsum

                gw = gy.t() @ x2d
                gb = colsum(gy) if ctx.has_bias else None
            return gx, gw, None, gb, None, None, None, None, None, None
        if ctx.needs_input_grad[1] or ctx.needs_input_grad[2] or ctx.needs_input_grad[3]:
            gw = deferred.grad_buf(weight)
            galpha = deferred.grad_buf(alpha, (), gy.device)
            gb = deferred.grad_buf(ctx.bias, (n,), gy.device) if ctx.has_bias else None
            if deferred.dwg_take(gy, x2d, P, m, n, k, gw, gb, stream, weight, ctx.bias,
                                 alpha=alpha, ga=galpha, pass_bits=pass_bits):
                return gx, gw, galpha, gb, None, None, None, None, None, None
            ws_bytes = lib.ob_bitlinear_bwd_dw_passes_workspace(P, m, n, k)
            ws = torch.empty((max(ws_bytes, 1),), dtype=torch.uint8, device=gy.device)
            slot = (deferred.dw_slot(gy.device, stream)
                    if deferred.can_defer(weight, alpha, ctx.bias) else None)
            if slot is not None:  # finish at the end of the backward (deferred.py)
                nb = ctypes.c_int64(0)
                _lib.check(lib.ob_bitlinear_bwd_dw_passes_defer(
                    gy.data_ptr(), x2d.data_ptr(), P, m, n, k, weight.data_ptr(),
                    alpha.data_ptr(), 1, pass_bits.data_ptr(), gw.data_ptr(), galpha.data_ptr(),
                    _lib.ptr(gb), ws.data_ptr(), ws_bytes, slot[0], slot[1], slot[2],
                    ctypes.addressof(nb), stream), "ob_bitlinear_bwd_dw_passes_defer")
                deferred.dw_done(1, nb.value)
                deferred.keep(ws)
            else:
                _lib.check(
                    lib.ob_bitlinear_bwd_dw_passes(gy.data_ptr(), x2d.data_ptr(), P, m, n, k,
                                                   weight.data_ptr(), alpha.data_ptr(), 1,
                                                   pass_bits.data_ptr(), gw.data_ptr(),
                                                   galpha.data_ptr(), _lib.ptr(gb), ws.data_ptr(),
                                                   ws_bytes, stream),
                    "ob_bitlinear_bwd_dw_passes",
                )
        return gx, gw, galpha, gb, None, None, None, None, None, None


def act_absmax(x: torch.Tensor, passes: int = 1) -> torch.Tensor:
    """Per-pass max|x| (device fp32 [passes]) of a contiguous fp32 tensor whose leading
    rows split into ``passes`` equal passes (the int8 mode's per-tensor scale)."""
    lib = _lib.load()
    n = x.numel() // passes
    amax = torch.empty((passes,), dtype=torch.float32, device=x.device)
    wsb = lib.ob_act_absmax_workspace(passes)
    ws = torch.empty((max(wsb, 1),), dtype=torch.uint8, device=x.device)
    _lib.check(lib.ob_act_absmax(x.data_ptr(), passes, n, amax.data_ptr(), ws.data_ptr(), wsb,
                                 _lib.stream_of(x)), "ob_act_absmax")
    return amax


class _BitLinearI8Fn(torch.autograd.Function):
    """Opt-in north-star mode (act_quant="absmax_int8"; not the reference's arithmetic,
    which keeps activations fp32 -- quant.py:126): per-pass absmax int8
    activations x ternary codes on the int8 matrix cores (csrc/tgemm_i8.hip). Backward is
    the straight-through estimator on both quantizers: dX = dY . W_hat (the fp32-path dX
    kernel), dW / dalpha / db from dY and the dequantized activations the forward used."""

    @staticmethod
    def forward(ctx, x2d, weight, alpha, bias, bits, P, codes, codes_t, codes1, codes1_t,
                amax=None):
        rows, k = x2d.shape
        m = rows // P
        n = weight.shape[0]
        lib = _lib.load()
        stream = _lib.stream_of(x2d)
        if amax is None:  # (else the producer's: LN / swish epilogue, x._ob_amax)
            amax = act_absmax(x2d, P)
        y = torch.empty((rows, n), dtype=torch.float32, device=x2d.device)
        pb = bits.tensor if isinstance(bits, PassBits) else None
        _lib.check(
            lib.ob_bitlinear_fwd_i8(x2d.data_ptr(), P, m, k, codes.data_ptr(), _lib.ptr(codes1),
                                    _lib.ptr(pb), alpha.data_ptr(), 1, amax.data_ptr(),
                                    _lib.ptr(bias), n, y.data_ptr(), stream),
            "ob_bitlinear_fwd_i8",
        )
        ctx.bits = bits
        ctx.P = P
        ctx.has_bias = bias is not None
        ctx.save_for_backward(x2d, weight, alpha, amax, codes_t, codes1_t)
        return y

    @staticmethod
    def backward(ctx, gy):
        x2d, weight, alpha, amax, codes_t, codes1_t = ctx.saved_tensors
        gy = gy.contiguous()
        rows, k = x2d.shape
        P = ctx.P
        m = rows // P
        n = weight.shape[0]
        lib = _lib.load()
        stream = _lib.stream_of(gy)
        stacked = isinstance(ctx.bits, PassBits)
        gx = gw = galpha = gb = None
        if ctx.needs_input_grad[0]:
            gx = torch.empty((rows, k), dtype=torch.float32, device=gy.device)
            if stacked:
                st = lib.ob_bitlinear_bwd_dx_passes(gy.data_ptr(), P, m, n, codes_t.data_ptr(),
                                                    codes1_t.data_ptr(), ctx.bits.tensor.data_ptr(),
                                                    alpha.data_ptr(), 1, k, gx.data_ptr(), stream)
            else:
                st = lib.ob_bitlinear_bwd_dx(gy.data_ptr(), m, n, codes_t.data_ptr(),
                                             alpha.data_ptr(), 1, k, gx.data_ptr(), stream)
            _lib.check(st, "ob_bitlinear_bwd_dx")
        if ctx.needs_input_grad[1] or ctx.needs_input_grad[2] or ctx.needs_input_grad[3]:
            xd = torch.empty_like(x2d)
            _lib.check(lib.ob_act_dequant_i8(x2d.data_ptr(), P, m * k, amax.data_ptr(),
                                             xd.data_ptr(), stream), "ob_act_dequant_i8")
            gw = torch.empty_like(weight)
            galpha = torch.empty((), dtype=torch.float32, device=gy.device)
            gb = torch.empty((n,), dtype=torch.float32, device=gy.device) if ctx.has_bias else None
            if stacked:
                ws_bytes = lib.ob_bitlinear_bwd_dw_passes_workspace(P, m, n, k)
                ws = torch.empty((max(ws_bytes, 1),), dtype=torch.uint8, device=gy.device)
                st = lib.ob_bitlinear_bwd_dw_passes(gy.data_ptr(), xd.data_ptr(), P, m, n, k,
                                                    weight.data_ptr(), alpha.data_ptr(), 1,
                                                    ctx.bits.tensor.data_ptr(), gw.data_ptr(),
                                                    galpha.data_ptr(), _lib.ptr(gb), ws.data_ptr(),
                                                    ws_bytes, stream)
            else:
                ws_bytes = lib.ob_bitlinear_bwd_dw_workspace(m, n, k)
                ws = torch.empty((max(ws_bytes, 1),), dtype=torch.uint8, device=gy.device)
                st = lib.ob_bitlinear_bwd_dw(gy.data_ptr(), xd.data_ptr(), m, n, k,
                                             weight.data_ptr(), alpha.data_ptr(), 1, ctx.bits,
                                             gw.data_ptr(), galpha.data_ptr(), _lib.ptr(gb),
                                             ws.data_ptr(), ws_bytes, stream)
            _lib.check(st, "ob_bitlinear_bwd_dw")
        return gx, gw, galpha, gb, None, None, None, None, None, None, None


class _QuantizeSTE(torch.autograd.Function):
    """quantize_weight's autograd function (quant.py:38-92): W_hat = a * Q(W/a) with the
    STE / LSQ-style alpha gradient. ``alpha`` is used as given (no abs/eps), as in the
    reference, where QuantizedLinear applies ``|alpha| + 1e-8`` before calling it."""

    @staticmethod
    def forward(ctx, W, alpha, bitwidth: int):
        bitwidth = _check_bitwidth(bitwidth)
        ctx.bits = bitwidth
        if bitwidth == 32:  # quant.py:61-64 passthrough
            return W
        _require_device(W, alpha)
        w = W.contiguous()
        out = torch.empty_like(w)
        lib = _lib.load()
        _lib.check(
            lib.ob_quant_dequant(w.data_ptr(), alpha.data_ptr(), 0, bitwidth, w.numel(),
                                 out.data_ptr(), _lib.stream_of(w)),
            "ob_quant_dequant",
        )
        ctx.save_for_backward(w, alpha)
        return out

    @staticmethod
    def backward(ctx, grad_out):
        if ctx.bits == 32:  # quant.py:76-78
            return grad_out, grad_out.new_zeros(()), None
        w, alpha = ctx.saved_tensors
        g = grad_out.contiguous()
        gw = torch.empty_like(w)
        galpha = torch.empty((), dtype=torch.float32, device=w.device)
        lib = _lib.load()
        ws_bytes = lib.ob_quant_ste_bwd_workspace(w.numel())
        ws = torch.empty((max(ws_bytes, 1),), dtype=torch.uint8, device=w.device)
        _lib.check(
            lib.ob_quant_ste_bwd(g.data_ptr(), w.data_ptr(), alpha.data_ptr(), 0, ctx.bits,
                                 w.numel(), gw.data_ptr(), galpha.data_ptr(), ws.data_ptr(),
                                 ws_bytes, _lib.stream_of(w)),
            "ob_quant_ste_bwd",
        )
        return gw, galpha.reshape(alpha.shape), None


def quantize_weight(W: torch.Tensor, alpha: torch.Tensor, bitwidth: int) -> torch.Tensor:
    """quant.py:95-96."""
    return _QuantizeSTE.apply(W, alpha, bitwidth)


class QuantizedLinear(nn.Module):
    """quant.py:99-127, same constructor, parameters, init and forward signature."""

    def __init__(self, in_features: int, out_features: int, bias: bool = True,
                 act_quant: Optional[str] = None):
        super().__init__()
        self.in_features = in_features
        self.out_features = out_features
        # None: the reference's fp32 activations. "absmax_int8": the opt-in north-star mode
        # (per-tensor absmax int8 activations on the int8 matrix cores; own tolerance).
        self.act_quant = _check_act_quant(act_quant)
        # BASELINE configs[3] ("quant off: BitLinear -> bf16 nn.Linear"): a torch dtype here
        # makes forward a plain F.linear in that dtype at every bitwidth (set_quant_off).
        self.quant_off: Optional[torch.dtype] = None
        self.weight = nn.Parameter(torch.empty(out_features, in_features))
        # quant.py:104-108: kaiming_uniform(a=sqrt(5)) then x2, i.e. U(-2/sqrt(in), 2/sqrt(in)).
        nn.init.kaiming_uniform_(self.weight, a=math.sqrt(5))
        with torch.no_grad():
            self.weight.mul_(2.0)
            init_alpha = self.weight.abs().mean()  # quant.py:111-113
        self.alpha = nn.Parameter(init_alpha)
        if bias:
            self.bias = nn.Parameter(torch.zeros(out_features))  # quant.py:115-116
        else:
            self.register_parameter("bias", None)
        self._codes_cache: dict = {}
        # packed-ternary checkpoint (checkpoint.py): {bits: (codes, codes_t)} used as they are;
        # the fp32 weight is then not meaningful (inference at bitwidth 1 / 2 only)
        self._packed: Optional[dict] = None

    def extra_repr(self) -> str:
        extra = f", act_quant={self.act_quant!r}" if self.act_quant else ""
        return (f"in_features={self.in_features}, out_features={self.out_features}, "
                f"bias={self.bias is not None}{extra}")

    def _codes(self, bits: int):
        """Codes for the current (weight, alpha) values: repacked only when either
        parameter was modified in place (optimizer step, load_state_dict, DDP broadcast)."""
        if self._packed is not None:
            if bits not in self._packed:
                raise KeyError(f"packed layer has no {bits}-bit codes "
                               f"(checkpoint holds {sorted(self._packed)})")
            return self._packed[bits]
        key = (self.weight.data_ptr(), self.weight._version, self.alpha.data_ptr(),
               self.alpha._version)
        hit = self._codes_cache.get(bits)
        if hit is not None and hit[0] == key:
            return hit[1], hit[2]
        codes, codes_t = pack_codes(self.weight, self.alpha, bits, alpha_raw=True)
        self._codes_cache[bits] = (key, codes, codes_t)
        return codes, codes_t

    def forward(self, x: torch.Tensor, bitwidth: int) -> torch.Tensor:
        if self.quant_off == "bf16w":  # configs[3] ceiling on the fused kernels (bf16 W)
            return self._forward_bf16w(x)
        if self.quant_off is not None:  # configs[3] ceiling: no quantizer, library GEMM
            return linear(x, self.weight, self.bias, dtype=self.quant_off)
        if self._packed is not None:
            self._check_packed_use(bitwidth)
        if isinstance(bitwidth, PassBits):
            return self._forward_passes(x, bitwidth)
        bits = _check_bitwidth(bitwidth)
        if bits == 32:  # quant.py:121-122 (F.linear; graph-safe bias gradient)
            return linear(x, self.weight, self.bias)
        _require_device(x, self.weight)
        lead = x.shape[:-1]
        x2d = x.reshape(-1, self.in_features)
        if not x2d.is_contiguous():
            x2d = x2d.contiguous()
        if bits == 0:  # DynamicBitwidth: codes depend on a device value, never cached
            if self.act_quant is not None:
                raise NotImplementedError("act_quant with a DynamicBitwidth: use StackedBits")
            codes, codes_t = pack_codes(self.weight, self.alpha, bitwidth, alpha_raw=True)
            bits = bitwidth
        else:
            codes, codes_t = self._codes(bits)
        if self.act_quant == "absmax_int8":
            amax = getattr(x, "_ob_amax", None)  # the producer's (LN / swish epilogue) scale
            if amax is not None and amax.numel() != 1:
                amax = None
            y = _BitLinearI8Fn.apply(x2d, self.weight, self.alpha, self.bias, bits, 1, codes,
                                     codes_t, None, None, amax)
            return y.view(*lead, self.out_features)
        y = _BitLinearFn.apply(x2d, self.weight, self.alpha, self.bias, bits, codes, codes_t)
        return y.view(*lead, self.out_features)

    def _forward_bf16w(self, x: torch.Tensor) -> torch.Tensor:
        """Quant-off (set_quant_off "bf16w") on the stacked-pass GEMM entries with B =
        bf16(W): one pass, the weight itself in every codes slot (alpha_raw 2 / 3)."""
        _require_device(x, self.weight)
        lead = x.shape[:-1]
        x2d = x.reshape(-1, self.in_features)
        if not x2d.is_contiguous():
            x2d = x2d.contiguous()
        key = x.device.index
        one = _ONE_PASS.get(key)
        if one is None:
            one = torch.full((1,), 2, dtype=torch.int32, device=x.device)
            _ONE_PASS[key] = one
        img, img_t = self._bf16_images()
        y = _BitLinearPassesFn.apply(x2d, self.weight, self.alpha, self.bias, one, 1, img, img_t,
                                     img, img_t)
        return y.view(*lead, self.out_features)

    def _bf16_images(self):
        """(bf16(W) [N][K], bf16(W^T) [K][N]) as int16 tensors, the quant-off GEMM operand;
        packed once per step for every layer by PackGroup, else here (one-item group)."""
        key = (self.weight.data_ptr(), self.weight._version)
        hit = self._codes_cache.get(16)
        if hit is not None and hit[0] == key:
            return hit[1], hit[2]
        n, k = self.weight.shape
        img = torch.empty((n, k), dtype=torch.int16, device=self.weight.device)
        img_t = torch.empty((k, n), dtype=torch.int16, device=self.weight.device)
        lib = _lib.load()
        items = np.zeros(1, dtype=PackGroup.ITEM)
        items[0] = (self.weight.data_ptr(), self.alpha.data_ptr(), img.data_ptr(),
                    img_t.data_ptr(), n, k, 0, 16, 1)
        table = torch.from_numpy(items.view(np.uint8).copy()).to(self.weight.device)
        _lib.check(lib.ob_quant_pack_group(table.data_ptr(), 1, lib.ob_weight_bf16_item_blocks(n, k),
                                           _lib.stream_of(self.weight)), "ob_quant_pack_group")
        self._codes_cache[16] = (key, img, img_t)
        return img, img_t

    def _forward_passes(self, x: torch.Tensor, pb: PassBits) -> torch.Tensor:
        """x: the P passes stacked on the leading dim ([P*B, ..., K] or [P*M, K])."""
        _require_device(x, self.weight)
        P = pb.passes
        lead = x.shape[:-1]
        x2d = x.reshape(-1, self.in_features)
        if x2d.shape[0] % P:
            raise ValueError(f"{x2d.shape[0]} rows do not split into {P} passes")
        if not x2d.is_contiguous():
            x2d = x2d.contiguous()
        codes2, codes2_t = self._codes(2)
        codes1, codes1_t = self._codes(1)
        if self.act_quant == "absmax_int8":
            y = _BitLinearI8Fn.apply(x2d, self.weight, self.alpha, self.bias, pb, P, codes2,
                                     codes2_t, codes1, codes1_t)
            return y.view(*lead, self.out_features)
        y = _BitLinearPassesFn.apply(x2d, self.weight, self.alpha, self.bias, pb.tensor, P,
                                     codes2, codes2_t, codes1, codes1_t)
        return y.view(*lead, self.out_features)

    def install_packed(self, packed: dict) -> None:
        """Use the given {bits: (codes, codes_t)} (a packed-ternary checkpoint,
        checkpoint.load_packed) for every forward at those bitwidths: inference only."""
        for b, (c, ct) in packed.items():
            n, k = self.weight.shape
            if b not in (1, 2) or tuple(c.shape) != (n, (k + 15) // 16) or \
                    tuple(ct.shape) != (k, (n + 15) // 16):
                raise ValueError(f"bad packed codes for bitwidth {b}")
        self._packed = dict(packed)
        self._codes_cache = {}

    def _check_packed_use(self, bitwidth) -> None:
        if isinstance(bitwidth, int) and bitwidth == 32:
            raise RuntimeError("packed-ternary layer: the checkpoint holds no fp32 weights "
                               "(bitwidth 32 needs an fp32 checkpoint)")
        if torch.is_grad_enabled() and (self.alpha.requires_grad or self.weight.requires_grad):
            raise RuntimeError("packed-ternary layers are inference-only: run under "
                               "torch.no_grad() / torch.inference_mode()")

    def invalidate_codes(self) -> None:
        """Drop the cached 2-bit codes. Needed after writing ``weight`` / ``alpha`` through
        ``.data`` (such writes do not bump the version counter the cache is keyed on);
        optimizer steps, ``load_state_dict`` and in-place ops on the parameters do not need it."""
        self._codes_cache = {}

    def _save_to_state_dict(self, destination, prefix, keep_vars):
        """A packed layer's ``weight`` is a placeholder (the codes came from a packed
        checkpoint): it is left out, so that the state dict cannot be mistaken for an fp32
        checkpoint (a strict load of it reports the missing weight; a packed model is
        saved with checkpoint.save_packed's source model or re-exported from its file)."""
        super()._save_to_state_dict(destination, prefix, keep_vars)
        if self._packed is not None:
            destination.pop(prefix + "weight", None)

    def _load_from_state_dict(self, state_dict, prefix, *args, **kwargs):
        self._codes_cache = {}
        if prefix + "weight" in state_dict:  # an fp32 weight replaces packed codes
            self._packed = None
        return super()._load_from_state_dict(state_dict, prefix, *args, **kwargs)

    def _apply(self, fn, *args, **kwargs):  # .to()/.cuda() invalidate cached codes
        self._codes_cache = {}
        if self._packed is not None:  # packed codes follow the module (int: no dtype cast)
            self._packed = {b: (fn(c), fn(ct)) for b, (c, ct) in self._packed.items()}
        return super()._apply(fn, *args, **kwargs)


class PackGroup:
    """Packs every QuantizedLinear under ``module`` for bitwidths ``bits`` in ONE launch
    (``ob_quant_pack_group``) and hands the codes to the layers' caches, so their
    forwards find fresh codes without a pack launch each. The reference quantizes per
    layer inside each forward (quant.py:123-126); a Conformer-S training step packs 144
    layers x 2 bitwidths, each a launch-bound ~5 us kernel.

    The descriptor table (parameter and code buffer addresses) is built once; ``run()``
    rebuilds it if a layer's weight moved (``.to()``, re-allocation)."""

    ITEM = np.dtype([("W", "<u8"), ("alpha", "<u8"), ("codes", "<u8"), ("codes_t", "<u8"),
                     ("N", "<i8"), ("K", "<i8"), ("block0", "<i8"), ("bits", "<i4"),
                     ("alpha_raw", "<i4")])  # == ob_pack_item (include/onebit_hip.h)

    def __init__(self, module: nn.Module, bits=(2, 1)):
        self.layers = [m for m in module.modules()
                       if isinstance(m, QuantizedLinear) and m.quant_off in (None, "bf16w")
                       and m._packed is None]  # packed layers keep their loaded codes
        self.bits = tuple(bits)
        self._ptrs = None
        self.table = None
        self.codes = []

    def _build(self):
        lib = _lib.load()
        items = np.zeros(sum(1 if m.quant_off == "bf16w" else len(self.bits) for m in self.layers),
                         dtype=self.ITEM)
        self.codes = []
        block0 = 0
        i = 0
        for m in self.layers:
            _require_device(m.weight, m.alpha)
            n, k = m.weight.shape
            per = {}
            if m.quant_off == "bf16w":  # quant-off ceiling: bf16 weight images (bits 16)
                c = torch.empty((n, k), dtype=torch.int16, device=m.weight.device)
                ct = torch.empty((k, n), dtype=torch.int16, device=m.weight.device)
                items[i] = (m.weight.data_ptr(), m.alpha.data_ptr(), c.data_ptr(), ct.data_ptr(),
                            n, k, block0, 16, 1)
                block0 += int(lib.ob_weight_bf16_item_blocks(n, k))
                per[16] = (c, ct)
                i += 1
                self.codes.append(per)
                continue
            for b in self.bits:
                c = torch.empty((n, (k + 15) // 16), dtype=torch.int32, device=m.weight.device)
                ct = torch.empty((k, (n + 15) // 16), dtype=torch.int32, device=m.weight.device)
                items[i] = (m.weight.data_ptr(), m.alpha.data_ptr(), c.data_ptr(), ct.data_ptr(),
                            n, k, block0, b, 1)
                block0 += int(lib.ob_quant_pack_item_blocks(n, k))
                per[b] = (c, ct)
                i += 1
            self.codes.append(per)
        self.total_blocks = block0
        self.n_items = i
        dev = self.layers[0].weight.device
        self.table = torch.from_numpy(items.view(np.uint8).copy()).to(dev)
        self._ptrs = [m.weight.data_ptr() for m in self.layers]

    def run(self) -> None:
        if not self.layers:
            return
        if self._ptrs != [m.weight.data_ptr() for m in self.layers]:
            self._build()
        lib = _lib.load()
        w0 = self.layers[0].weight
        _lib.check(lib.ob_quant_pack_group(self.table.data_ptr(), self.n_items,
                                           self.total_blocks, _lib.stream_of(w0)),
                   "ob_quant_pack_group")
        for m, per in zip(self.layers, self.codes):
            key = (m.weight.data_ptr(), m.weight._version, m.alpha.data_ptr(), m.alpha._version)
            for b, (c, ct) in per.items():
                m._codes_cache[b] = ((m.weight.data_ptr(), m.weight._version) if b == 16 else key,
                                     c, ct)


# north_star's name for the same layer.
BitLinear = QuantizedLinear
