"""The BitLinear boundary as registered torch operators (``torch.library``), so torch.compile
and op-level tooling see it: ``torch.ops.onebit.bitlinear(x, weight, alpha, bias, bits)``
is ``F.linear(x, quantize_weight(weight, |alpha| + 1e-8, bits), bias)`` of the reference
(quant.py:120-127 with quant.py:38-96 inside) on the HIP library, with the STE backward
registered through ``register_autograd``.

Building blocks (each one C-ABI call, include/onebit_hip.h):
  onebit::pack_codes(weight, alpha, bits) -> (codes, codes_t)   ob_quant_pack
  onebit::bitlinear_fwd(x2d, codes, alpha, bias, n) -> y         ob_bitlinear_fwd
  onebit::bitlinear_dx(gy, codes_t, alpha, k) -> gx              ob_bitlinear_bwd_dx
  onebit::bitlinear_dw(gy, x2d, weight, alpha, bits, has_bias) -> (gw, galpha, gb)
                                                                 ob_bitlinear_bwd_dw
Each has a fake (meta) implementation for tracing. ``QuantizedLinear`` keeps its own
autograd.Function (it caches codes per weight version and has the stacked / fused paths);
these operators are the compiler-visible form of the same kernels.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
from torch import Tensor

from . import _lib

__all__ = ["bitlinear"]


@torch.library.custom_op("onebit::pack_codes", mutates_args=())
def pack_codes_op(weight: Tensor, alpha: Tensor, bits: int) -> Tuple[Tensor, Tensor]:
    from .quant import pack_codes

    return pack_codes(weight, alpha, bits, alpha_raw=True)


@pack_codes_op.register_fake
def _(weight, alpha, bits):
    n, k = weight.shape
    return (weight.new_empty((n, (k + 15) // 16), dtype=torch.int32),
            weight.new_empty((k, (n + 15) // 16), dtype=torch.int32))


@torch.library.custom_op("onebit::bitlinear_fwd", mutates_args=())
def bitlinear_fwd(x2d: Tensor, codes: Tensor, alpha: Tensor, bias: Optional[Tensor],
                  n: int) -> Tensor:
    m, k = x2d.shape
    y = torch.empty((m, n), dtype=torch.float32, device=x2d.device)
    _lib.check(_lib.load().ob_bitlinear_fwd(x2d.data_ptr(), m, k, codes.data_ptr(),
                                            alpha.data_ptr(), 1, _lib.ptr(bias), n, y.data_ptr(),
                                            _lib.stream_of(x2d)), "ob_bitlinear_fwd")
    return y


@bitlinear_fwd.register_fake
def _(x2d, codes, alpha, bias, n):
    return x2d.new_empty((x2d.shape[0], n))


@torch.library.custom_op("onebit::bitlinear_dx", mutates_args=())
def bitlinear_dx(gy: Tensor, codes_t: Tensor, alpha: Tensor, k: int) -> Tensor:
    m, n = gy.shape
    gx = torch.empty((m, k), dtype=torch.float32, device=gy.device)
    _lib.check(_lib.load().ob_bitlinear_bwd_dx(gy.data_ptr(), m, n, codes_t.data_ptr(),
                                               alpha.data_ptr(), 1, k, gx.data_ptr(),
                                               _lib.stream_of(gy)), "ob_bitlinear_bwd_dx")
    return gx


@bitlinear_dx.register_fake
def _(gy, codes_t, alpha, k):
    return gy.new_empty((gy.shape[0], k))


@torch.library.custom_op("onebit::bitlinear_dw", mutates_args=())
def bitlinear_dw(gy: Tensor, x2d: Tensor, weight: Tensor, alpha: Tensor, bits: int,
                 has_bias: bool) -> Tuple[Tensor, Tensor, Tensor]:
    m, n = gy.shape
    k = x2d.shape[1]
    lib = _lib.load()
    gw = torch.empty_like(weight)
    galpha = torch.empty((), dtype=torch.float32, device=gy.device)
    gb = torch.empty((n if has_bias else 0,), dtype=torch.float32, device=gy.device)
    wsb = lib.ob_bitlinear_bwd_dw_workspace(m, n, k)
    ws = torch.empty((max(wsb, 1),), dtype=torch.uint8, device=gy.device)
    _lib.check(lib.ob_bitlinear_bwd_dw(gy.data_ptr(), x2d.data_ptr(), m, n, k, weight.data_ptr(),
                                       alpha.data_ptr(), 1, bits, gw.data_ptr(),
                                       galpha.data_ptr(), gb.data_ptr() if has_bias else None,
                                       ws.data_ptr(), wsb, _lib.stream_of(gy)),
               "ob_bitlinear_bwd_dw")
    return gw, galpha, gb


@bitlinear_dw.register_fake
def _(gy, x2d, weight, alpha, bits, has_bias):
    return (torch.empty_like(weight), alpha.new_empty(()),
            gy.new_empty((gy.shape[1] if has_bias else 0,)))


@torch.library.custom_op("onebit::bitlinear", mutates_args=())
def bitlinear_op(x: Tensor, weight: Tensor, alpha: Tensor, bias: Optional[Tensor],
                 bits: int) -> Tensor:
    if bits not in (1, 2):
        raise ValueError("bitwidth must be one of {1,2,32}")  # quant.py:65-66
    codes, _ = pack_codes_op(weight, alpha, bits)
    n, k = weight.shape
    y = bitlinear_fwd(x.reshape(-1, k).contiguous(), codes, alpha, bias, n)
    return y.view(*x.shape[:-1], n)


@bitlinear_op.register_fake
def _(x, weight, alpha, bias, bits):
    return x.new_empty((*x.shape[:-1], weight.shape[0]))


def _setup_context(ctx, inputs, output):
    x, weight, alpha, bias, bits = inputs
    ctx.save_for_backward(x, weight, alpha)
    ctx.bits = bits
    ctx.has_bias = bias is not None


def _backward(ctx, gy):
    x, weight, alpha = ctx.saved_tensors
    n, k = weight.shape
    g2 = gy.reshape(-1, n).contiguous()
    x2 = x.reshape(-1, k).contiguous()
    _, codes_t = pack_codes_op(weight, alpha, ctx.bits)
    gx = bitlinear_dx(g2, codes_t, alpha, k).view(x.shape)
    gw, galpha, gb = bitlinear_dw(g2, x2, weight, alpha, ctx.bits, ctx.has_bias)
    return gx, gw, galpha.reshape(alpha.shape), (gb if ctx.has_bias else None), None


bitlinear_op.register_autograd(_backward, setup_context=_setup_context)


def bitlinear(x: Tensor, weight: Tensor, alpha: Tensor, bias: Optional[Tensor],
              bits: int) -> Tensor:
    """quant.py:120-127 for bitwidth 1 / 2 as the registered operator."""
    return torch.ops.onebit.bitlinear(x, weight, alpha, bias, bits)
