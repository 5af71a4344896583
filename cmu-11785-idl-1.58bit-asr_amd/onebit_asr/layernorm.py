"""LayerNorm over the last dim on the HIP library (csrc/layernorm.hip).

Used by the Conformer's ``LayerNorm`` wrapper (reference onebit_asr/conformer.py:19-24,
``nn.LayerNorm(d)``) on a ROCm device for fp32 inputs with d <= 512; other cases run
torch's ``F.layer_norm``. Same arithmetic as torch's (biased variance, eps inside the
square root); the backward's dgamma / dbeta are summed in a fixed order.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from . import _lib

__all__ = ["layer_norm", "layer_norm_fork", "layer_norm_amax", "fused_layernorm_supported"]


def fused_layernorm_supported(x: torch.Tensor, d: int) -> bool:
    if os.environ.get("OB_LN", "") == "torch":
        return False
    return x.is_cuda and x.dtype == torch.float32 and 1 <= d <= 512


class _LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, eps):
        d = x.shape[-1]
        x2 = x.contiguous().view(-1, d)
        rows = x2.shape[0]
        y = torch.empty_like(x2)
        need = any(ctx.needs_input_grad[:3])
        mean = torch.empty((rows,), dtype=torch.float32, device=x.device) if need else None
        rstd = torch.empty((rows,), dtype=torch.float32, device=x.device) if need else None
        lib = _lib.load()
        _lib.check(lib.ob_layernorm_fwd(x2.data_ptr(), _lib.ptr(weight), _lib.ptr(bias), rows, d,
                                        float(eps), y.data_ptr(), _lib.ptr(mean), _lib.ptr(rstd),
                                        _lib.stream_of(x2)), "ob_layernorm_fwd")
        if need:
            ctx.save_for_backward(x2, weight, mean, rstd)
            ctx.has = (weight is not None, bias is not None)
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, gy):
        x2, weight, mean, rstd = ctx.saved_tensors
        rows, d = x2.shape
        g2 = gy.contiguous().view(rows, d)
        dx = torch.empty_like(x2)
        has_w, has_b = ctx.has
        dw = torch.empty((d,), dtype=torch.float32, device=x2.device) if has_w and ctx.needs_input_grad[1] else None
        db = torch.empty((d,), dtype=torch.float32, device=x2.device) if has_b and ctx.needs_input_grad[2] else None
        lib = _lib.load()
        wsb = lib.ob_layernorm_bwd_workspace(rows, d)
        ws = torch.empty((max(wsb, 1),), dtype=torch.uint8, device=x2.device)
        _lib.check(lib.ob_layernorm_bwd(g2.data_ptr(), x2.data_ptr(), _lib.ptr(weight),
                                        mean.data_ptr(), rstd.data_ptr(), rows, d, dx.data_ptr(),
                                        _lib.ptr(dw), _lib.ptr(db), ws.data_ptr(), wsb,
                                        _lib.stream_of(g2)), "ob_layernorm_bwd")
        return dx.view(gy.shape), dw, db, None


def layer_norm(x: torch.Tensor, weight, bias, eps: float = 1e-5) -> torch.Tensor:
    d = x.shape[-1]
    if not fused_layernorm_supported(x, d):
        return F.layer_norm(x, (d,), weight, bias, eps)
    return _LayerNormFn.apply(x, weight, bias, eps)


@torch.no_grad()
def layer_norm_amax(x: torch.Tensor, weight, bias, eps: float = 1e-5) -> torch.Tensor:
    """Inference: LN(x) carrying its max|y| (device fp32 [1]) as ``y._ob_amax`` -- the
    per-tensor int8 scale of the BitLinear that consumes it, produced by the LN kernel itself
    (ob_layernorm_fwd_amax) instead of a separate absmax pass over y."""
    d = x.shape[-1]
    x2 = x.contiguous().view(-1, d)
    rows = x2.shape[0]
    y = torch.empty_like(x2)
    amax = torch.empty((1,), dtype=torch.float32, device=x.device)
    lib = _lib.load()
    wsb = lib.ob_layernorm_fwd_amax_workspace(1)
    ws = torch.empty((wsb,), dtype=torch.uint8, device=x.device)
    _lib.check(lib.ob_layernorm_fwd_amax(x2.data_ptr(), _lib.ptr(weight), _lib.ptr(bias), rows,
                                         d, float(eps), y.data_ptr(), None, None, 1,
                                         amax.data_ptr(), ws.data_ptr(), wsb,
                                         _lib.stream_of(x2)), "ob_layernorm_fwd_amax")
    y = y.view(x.shape)
    y._ob_amax = amax
    return y


class _LayerNormForkFn(torch.autograd.Function):
    """(LN(x), x) for a residual junction x -> (LN -> module) + x: the backward receives both
    branches' gradients and forms dx = LN_backward(dy) + dres in the LN backward kernel,
    instead of autograd's separate add over the [rows, d] tensor."""

    @staticmethod
    def forward(ctx, x, weight, bias, eps):
        y = _LayerNormFn.forward(ctx, x, weight, bias, eps)
        return y, x.view_as(x)

    @staticmethod
    def backward(ctx, gy, gres):
        if gres is None:
            return _LayerNormFn.backward(ctx, gy)
        x2, weight, mean, rstd = ctx.saved_tensors
        rows, d = x2.shape
        if gy is None:
            return gres, None, None, None
        g2 = gy.contiguous().view(rows, d)
        r2 = gres.contiguous().view(rows, d)
        dx = torch.empty_like(x2)
        has_w, has_b = ctx.has
        dw = torch.empty((d,), dtype=torch.float32, device=x2.device) if has_w and ctx.needs_input_grad[1] else None
        db = torch.empty((d,), dtype=torch.float32, device=x2.device) if has_b and ctx.needs_input_grad[2] else None
        lib = _lib.load()
        wsb = lib.ob_layernorm_bwd_workspace(rows, d)
        ws = torch.empty((max(wsb, 1),), dtype=torch.uint8, device=x2.device)
        _lib.check(lib.ob_layernorm_bwd_res(g2.data_ptr(), x2.data_ptr(), _lib.ptr(weight),
                                            mean.data_ptr(), rstd.data_ptr(), rows, d,
                                            r2.data_ptr(), dx.data_ptr(), _lib.ptr(dw),
                                            _lib.ptr(db), ws.data_ptr(), wsb,
                                            _lib.stream_of(g2)), "ob_layernorm_bwd_res")
        return dx.view(gy.shape), dw, db, None


def layer_norm_fork(x: torch.Tensor, weight, bias, eps: float = 1e-5):
    """(LN(x), x_residual): use x_residual for the junction's skip connection so the
    backward adds the two gradient branches inside the LN backward kernel."""
    d = x.shape[-1]
    if not fused_layernorm_supported(x, d) or not torch.is_grad_enabled() or not x.requires_grad:
        return layer_norm(x, weight, bias, eps), x
    return _LayerNormForkFn.apply(x, weight, bias, eps)
