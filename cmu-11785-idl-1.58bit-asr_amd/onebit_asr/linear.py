"""Full-precision ``F.linear`` whose backward is safe to replay from a HIP graph.

The reference's full-precision linears (subsampling ``out``, ``ctc_head``, the decoder's
projections, feed-forward and output layers; onebit_asr/conformer.py:195,275-299,313) run
stock ``F.linear`` there. Their bias gradient is torch's column reduction, which on this
ROCm build takes a two-level "global reduce" path whose semaphores are cleared by a
``hipMemsetAsync``; captured into a HIP graph that memset is not re-executed correctly on
replays after the first (tools/memset_graph_repro.py, tools/reduce_graph_repro.py), so
every replayed step after the first produced garbage bias gradients. Here the GEMMs stay
library GEMMs (hipBLASLt / rocBLAS), and the bias gradient is the fixed-order column sum
``ob_colsum`` (csrc/fused.hip) -- deterministic and graph-safe. Same arithmetic as
``F.linear`` up to summation order.

``dtype`` (optional) computes the GEMMs in that type (BASELINE configs[3]: bf16
``nn.Linear``); inputs, outputs and gradients stay fp32.

fp32 forward (and dX) GEMMs whose shape csrc/dgemm.hip takes (K, N multiples of 4, the
split weight image within LDS) run there: exact-fp32 products on the bf16 matrix cores
(six MFMAs per k-step), bias in the epilogue. At Conformer-S the CTC head's forward
([23904 x 144] x [144 x 5004]) is the large one. Weight gradients whose N and K are
multiples of 48 (the decoder's projections and feed-forward, the subsampling output layer)
run on the dW kernel family (``ob_dense_dw``: exact-fp32 products, fixed-order chunk sums,
the bias gradient from the same pass). OB_DENSE_LINEAR=0: library GEMMs only;
OB_DENSE_LINEAR_DW=0: library weight gradients.
"""
from __future__ import annotations


from typing import Optional

import torch
import torch.nn.functional as F

from . import _lib, deferred

__all__ = ["linear", "linear_rows_split", "colsum"]



# K above this at M < 16384 rows: the library GEMM (see _dense_ok). The decoder FFN's
# K = 1024 products (linear2 forward, linear1 dX, M = 3936) ran at 30.7 / 31.0 us on the
# dgemm kernel (one 16-column tile per block: the K = 1024 image leaves no room for more)
# against 17.9 / 17.0 us on hipBLASLt, the self-attention in-projection's dX (K = 432) at
# 18.7 against 14.6 us (same-box A/Bs, profiles/r6/lib_k/).
_LIB_K = 256


def _dense_ok(x: torch.Tensor, w: torch.Tensor, k: int, n: int) -> bool:
    """ob_dense_gemm's preconditions (capi.hip: aligned16 of BOTH operands), so an operand
    it would refuse takes the library path instead of raising. A long reduction (K >
    _LIB_K: the CTC head's input gradient, K = V = 5004) runs on the HIP kernels only for
    full-size batches (the K-chunked kernel: one 128-row block per CU sweeps all of K), so
    the decoder's 3936-row products with K = 1024 / 5004 stay on the library GEMM."""
    if k > _LIB_K and x.shape[0] < 16384:
        return False
    return (k % 4 == 0 and n % 4 == 0 and x.data_ptr() % 16 == 0
            and w.data_ptr() % 16 == 0 and _lib.load().ob_dense_supported(k, n) == 1)


def _dense_dw_ws(g2: torch.Tensor, x2d: torch.Tensor, w: torch.Tensor) -> int:
    """Workspace bytes of ob_dense_dw for this linear's weight gradient, 0 if not taken
    (N, K multiples of 4; 16-byte aligned operands)."""
    if not (g2.is_cuda and x2d.is_contiguous() and w.is_contiguous()
            and g2.data_ptr() % 16 == 0 and x2d.data_ptr() % 16 == 0):
        return 0
    n, k = w.shape
    return int(_lib.load().ob_dense_dw_workspace(g2.shape[0], n, k))


def _dense(x2d: torch.Tensor, w: torch.Tensor, trans: int, bias, n: int) -> torch.Tensor:
    """x2d [M, K] . (w^T if trans == 0 else w) (+ bias) on csrc/dgemm.hip."""
    m, k = x2d.shape
    y = torch.empty((m, n), dtype=torch.float32, device=x2d.device)
    _lib.check(_lib.load().ob_dense_gemm(x2d.data_ptr(), m, k, w.data_ptr(), trans,
                                         _lib.ptr(bias), n, y.data_ptr(), _lib.stream_of(x2d)),
               "ob_dense_gemm")
    return y


def colsum(x2d: torch.Tensor) -> torch.Tensor:
    """Column sums of a [rows, N] fp32 matrix (fixed order; csrc/fused.hip)."""
    x2d = x2d.contiguous()
    rows, n = x2d.shape
    out = torch.empty((n,), dtype=torch.float32, device=x2d.device)
    lib = _lib.load()
    wsb = lib.ob_colsum_workspace(n)
    ws = torch.empty((wsb,), dtype=torch.uint8, device=x2d.device)
    _lib.check(lib.ob_colsum(x2d.data_ptr(), rows, n, out.data_ptr(), ws.data_ptr(), wsb,
                             _lib.stream_of(x2d)), "ob_colsum")
    return out


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, dtype):
        k = x.shape[-1]
        x2d = x.reshape(-1, k)
        n = weight.shape[0]
        if dtype is None and x2d.is_contiguous() and weight.is_contiguous() and _dense_ok(x2d, weight, k, n):
            y = _dense(x2d, weight, 0, bias, n)
        elif dtype is None:
            y = torch.addmm(bias, x2d, weight.t()) if bias is not None else x2d @ weight.t()
        else:
            wd = weight.to(dtype)
            yd = (torch.addmm(bias.to(dtype), x2d.to(dtype), wd.t()) if bias is not None
                  else x2d.to(dtype) @ wd.t())
            y = yd.to(torch.float32)
        ctx.save_for_backward(x2d, weight)
        ctx.meta = (bias is not None, dtype, x.shape)
        ctx.bias = bias
        if dtype is None:
            deferred.note(weight, bias)
        return y.view(*x.shape[:-1], weight.shape[0])

    @staticmethod
    def backward(ctx, g):
        x2d, weight = ctx.saved_tensors
        has_b, dtype, xshape = ctx.meta
        g2 = g.reshape(-1, weight.shape[0])
        if not g2.is_contiguous():
            g2 = g2.contiguous()
        gx = gw = gb = None
        if dtype is None:
            if ctx.needs_input_grad[0]:
                k = weight.shape[1]
                if weight.is_contiguous() and _dense_ok(g2, weight, weight.shape[0], k):
                    gx = _dense(g2, weight, 1, None, k).view(xshape)
                else:
                    gx = (g2 @ weight).view(xshape)
            wsb = _dense_dw_ws(g2, x2d, weight) if ctx.needs_input_grad[1] else 0
            if wsb:  # dW (and db) on the dW kernel family: exact-fp32 products, fixed order
                m, n, k = g2.shape[0], weight.shape[0], weight.shape[1]
                gw = deferred.grad_buf(weight)
                if has_b and ctx.needs_input_grad[2]:
                    gb = deferred.grad_buf(ctx.bias, (n,), g2.device)
                ws = torch.empty((wsb,), dtype=torch.uint8, device=g2.device)
                deferred.dense_dw(g2, x2d, m, n, k, gw, gb, ws, wsb, _lib.stream_of(g2), weight,
                                  ctx.bias)
                return gx, gw, gb, None
            if ctx.needs_input_grad[1]:
                gw = g2.t() @ x2d
        else:
            gd = g2.to(dtype)
            if ctx.needs_input_grad[0]:
                gx = (gd @ weight.to(dtype)).to(torch.float32).view(xshape)
            if ctx.needs_input_grad[1]:
                gw = (gd.t() @ x2d.to(dtype)).to(torch.float32)
        if has_b and ctx.needs_input_grad[2]:
            gb = colsum(g2)
        return gx, gw, gb, None


class _RowsSplitFn(torch.autograd.Function):
    """(F.linear(x, w[:e], b[:e]), F.linear(y, w[e:], b[e:])) for ONE packed weight: the
    cross-attention in-projection of nn.MultiheadAttention (query rows from the decoder
    state, key / value rows from the encoder memory; reference conformer.py:275-299 via
    torch's multi_head_attention_forward). Sliced through autograd, each slice's weight /
    bias gradient is scattered into a zero-filled full-size tensor and the two summed
    (fills, copies and adds of [3e, e] a layer); here the two dW GEMMs write their row ranges
    of the one gradient buffer directly, on the deferred / grouped weight-gradient path."""

    @staticmethod
    def forward(ctx, x, y, weight, bias, e):
        k = x.shape[-1]
        x2, y2 = x.reshape(-1, k), y.reshape(-1, k)
        w1, w2 = weight[:e], weight[e:]  # row ranges: contiguous views
        b1 = bias[:e] if bias is not None else None
        b2 = bias[e:] if bias is not None else None
        o1 = _dense(x2, w1, 0, b1, e)
        o2 = _dense(y2, w2, 0, b2, weight.shape[0] - e)
        ctx.save_for_backward(x2, y2, weight)
        ctx.meta = (e, x.shape, y.shape)
        ctx.bias = bias
        deferred.note(weight, bias)
        return o1.view(*x.shape[:-1], e), o2.view(*y.shape[:-1], weight.shape[0] - e)

    @staticmethod
    def backward(ctx, g1, g2):
        x2, y2, weight = ctx.saved_tensors
        e, xs, ys = ctx.meta
        n, k = weight.shape
        bias = ctx.bias
        dev = x2.device
        outs = []
        for g, inp, lo, hi, shp in ((g1, x2, 0, e, xs), (g2, y2, e, n, ys)):
            g = torch.zeros((inp.shape[0], hi - lo), dtype=torch.float32, device=dev) \
                if g is None else g.reshape(-1, hi - lo).contiguous()
            outs.append(g)
        gx = _dense(outs[0], weight[:e], 1, None, k).view(xs) if ctx.needs_input_grad[0] else None
        gy = _dense(outs[1], weight[e:], 1, None, k).view(ys) if ctx.needs_input_grad[1] else None
        gw = gb = None
        if ctx.needs_input_grad[2]:
            gw = deferred.grad_buf(weight)
            if bias is not None and ctx.needs_input_grad[3]:
                gb = deferred.grad_buf(bias, (n,), dev)
            stream = _lib.stream_of(outs[0])
            for g, inp, lo, hi in ((outs[0], x2, 0, e), (outs[1], y2, e, n)):
                ws_b = int(_lib.load().ob_dense_dw_workspace(g.shape[0], hi - lo, k))
                if not ws_b:  # (not on the dW kernels: torch, bias by the column sum)
                    gw[lo:hi] = g.t() @ inp
                    if gb is not None:
                        gb[lo:hi] = colsum(g)
                    continue
                ws = torch.empty((ws_b,), dtype=torch.uint8, device=dev)
                deferred.dense_dw(g, inp, g.shape[0], hi - lo, k, gw[lo:hi],
                                  gb[lo:hi] if gb is not None else None, ws, ws_b, stream,
                                  weight, bias)
        elif bias is not None and ctx.needs_input_grad[3]:
            gb = torch.cat([colsum(outs[0]), colsum(outs[1])])
        return gx, gy, gw, gb, None


def linear_rows_split(x: torch.Tensor, y: torch.Tensor, weight: torch.Tensor,
                      bias: Optional[torch.Tensor], e: int):
    """(linear(x, weight[:e], bias[:e]), linear(y, weight[e:], bias[e:])) with the packed
    weight's gradient formed in place (_RowsSplitFn); the sliced form where the fused path does
    not apply (CPU, shapes / alignment the dense GEMM refuses)."""
    n, k = weight.shape
    ok = (x.is_cuda and x.dtype == torch.float32 and weight.dtype == torch.float32
          and x.is_contiguous() and y.is_contiguous() and weight.is_contiguous()
          and (bias is None or bias.is_contiguous()) and 0 < e < n
          and _dense_ok(x.reshape(-1, k), weight, k, e)
          and _dense_ok(y.reshape(-1, k), weight[e:], k, n - e)
          and _dense_ok(x.reshape(-1, k), weight, e, k) and _dense_ok(y.reshape(-1, k), weight, n - e, k)
          and (weight[e:].data_ptr() % 16 == 0))
    if not ok:
        return (linear(x, weight[:e], bias[:e] if bias is not None else None),
                linear(y, weight[e:], bias[e:] if bias is not None else None))
    return _RowsSplitFn.apply(x, y, weight, bias, e)


def linear(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor] = None,
           dtype: Optional[torch.dtype] = None) -> torch.Tensor:
    """``F.linear(x, weight, bias)`` (computed in ``dtype`` if given) with a graph-safe,
    deterministic bias gradient on a ROCm device; stock ``F.linear`` elsewhere."""
    if not (x.is_cuda and x.dtype == torch.float32 and weight.dtype == torch.float32):
        if dtype is not None:
            b = bias.to(dtype) if bias is not None else None
            return F.linear(x.to(dtype), weight.to(dtype), b).to(x.dtype)
        return F.linear(x, weight, bias)
    return _LinearFn.apply(x, weight, bias, dtype)
