"""Depthwise Conv1d of the conv module on the HIP kernel.

Reference: onebit_asr/conformer.py:147 ``nn.Conv1d(C, C, k, padding=k//2, groups=C)``,
full precision. The module keeps its ``nn.Conv1d`` (checkpoint keys ``...conv.dw.weight``
/ ``...conv.dw.bias``); on a ROCm device its forward/backward run ``ob_dwconv1d_*`` from
libonebit_hip.so instead of MIOpen's grouped convolution. Stock conv on CPU tensors is
the reference behaviour of this full-precision op (it is not the BitLinear hot path).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import _lib

__all__ = ["depthwise_conv1d"]


class _DwConv1dFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        b, c, t = x.shape
        kt = weight.shape[-1]
        x = x.contiguous()
        w = weight.detach().reshape(c, kt).contiguous()
        y = torch.empty_like(x)
        lib = _lib.load()
        _lib.check(lib.ob_dwconv1d_fwd(x.data_ptr(), w.data_ptr(), _lib.ptr(bias), b, c, t, kt,
                                       y.data_ptr(), _lib.stream_of(x)), "ob_dwconv1d_fwd")
        ctx.save_for_backward(x, w)
        ctx.has_bias = bias is not None
        ctx.wshape = weight.shape
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        b, c, t = x.shape
        kt = w.shape[1]
        gy = gy.contiguous()
        gx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        gw = torch.empty((c, kt), dtype=torch.float32, device=x.device)
        gb = torch.empty((c,), dtype=torch.float32, device=x.device) if ctx.has_bias else None
        lib = _lib.load()
        wsb = lib.ob_dwconv1d_bwd_workspace(b, c, kt)
        ws = torch.empty((max(wsb, 1),), dtype=torch.uint8, device=x.device)
        _lib.check(lib.ob_dwconv1d_bwd(x.data_ptr(), gy.data_ptr(), w.data_ptr(), b, c, t, kt,
                                       _lib.ptr(gx), gw.data_ptr(), _lib.ptr(gb), ws.data_ptr(), wsb,
                                       _lib.stream_of(x)), "ob_dwconv1d_bwd")
        return gx, gw.reshape(ctx.wshape), gb


def depthwise_conv1d(x: torch.Tensor, conv: nn.Conv1d) -> torch.Tensor:
    """``conv(x)`` for a depthwise, odd-width, 'same'-padded Conv1d; HIP kernel on ROCm."""
    kt = conv.kernel_size[0]
    eligible = (x.is_cuda and x.dtype == torch.float32 and conv.groups == conv.in_channels ==
                conv.out_channels and kt % 2 == 1 and kt <= 64 and conv.padding[0] == kt // 2
                and conv.stride[0] == 1 and conv.dilation[0] == 1)
    if not eligible:
        return conv(x)
    return _DwConv1dFn.apply(x, conv.weight, conv.bias)
