"""The Conformer conv module on the HIP library.

* ``conv_module_fused`` -- ConvModule.forward (conformer.py:139-167) channels-last: pw1 /
  pw2 as GEMMs on [rows, C] (no [B,C,T] transposes), GLU + depthwise conv + per-pass
  BatchNorm (batch statistics) + swish in csrc/convmod.hip (4 launches forward, 5
  backward), dropout + residual in one kernel.
* ``depthwise_conv1d`` -- the depthwise conv alone on [B, C, T] (the unfused path).

Reference: onebit_asr/conformer.py:147 ``nn.Conv1d(C, C, k, padding=k//2, groups=C)``,
full precision. The module keeps its ``nn.Conv1d`` (checkpoint keys ``...conv.dw.weight``
/ ``...conv.dw.bias``); on a ROCm device its forward/backward run ``ob_dwconv1d_*`` from
libonebit_hip.so instead of MIOpen's grouped convolution. Stock conv on CPU tensors is
the reference behaviour of this full-precision op (it is not the BitLinear hot path).
"""
from __future__ import annotations

import ctypes
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib, deferred
from .layernorm import GradScale, attach_grad_scale
from .linear import colsum

__all__ = ["depthwise_conv1d", "conv_module_supported", "conv_module_fused", "colsum",
           "conv2d_bias_relu"]


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


class _ConvCoreFn(torch.autograd.Function):
    """GLU -> depthwise conv -> BatchNorm (batch statistics, per pass) -> swish on the
    channels-last pw1 output (csrc/convmod.hip; conformer.py:156-159)."""

    @staticmethod
    def forward(ctx, u, wdw, bdw, gamma, beta, P, T, eps):
        rows, c2 = u.shape
        C = c2 // 2
        K = wdw.shape[-1]
        Bt = rows // T
        lib = _lib.load()
        z = torch.empty((rows, C), dtype=torch.float32, device=u.device)
        g = torch.empty_like(z)
        v = torch.empty_like(z)
        stats = torch.empty((P, C, 2), dtype=torch.float32, device=u.device)
        wsb = lib.ob_convmod_workspace(P, Bt, T, C, K)
        ws = torch.empty((wsb,), dtype=torch.uint8, device=u.device)
        w2 = wdw.detach().reshape(C, K).contiguous()
        _lib.check(lib.ob_convmod_fwd(u.data_ptr(), w2.data_ptr(), _lib.ptr(bdw), gamma.data_ptr(),
                                      beta.data_ptr(), P, Bt, T, C, K, eps, z.data_ptr(),
                                      g.data_ptr(), stats.data_ptr(), v.data_ptr(), ws.data_ptr(), wsb,
                                      _lib.stream_of(u)), "ob_convmod_fwd")
        ctx.meta = (P, T, K, bdw is not None, wdw.shape)
        ctx.params = (wdw, bdw)
        deferred.note(wdw, bdw)
        ctx.save_for_backward(u, z, g, stats, w2, gamma, beta)
        return v

    @staticmethod
    def backward(ctx, dv):
        u, z, g, stats, w2, gamma, beta = ctx.saved_tensors
        P, T, K, has_b, wshape = ctx.meta
        dv = dv.contiguous()
        rows, c2 = u.shape
        C = c2 // 2
        Bt = rows // T
        lib = _lib.load()
        du = torch.empty_like(u)
        dw = torch.empty((C, K), dtype=torch.float32, device=u.device)
        db = torch.empty((C,), dtype=torch.float32, device=u.device) if has_b else None
        dg = torch.empty_like(gamma)
        dbt = torch.empty_like(beta)
        wsb = lib.ob_convmod_workspace(P, Bt, T, C, K)
        ws = torch.empty((wsb,), dtype=torch.uint8, device=u.device)
        stream = _lib.stream_of(dv)
        # the depthwise weight-gradient finish joins the end-of-backward table launch when the
        # weight and bias qualify (deferred.py); the kernel reports whether the shape allowed it
        slot = deferred.cm_slot(u.device, stream) if deferred.can_defer(*ctx.params) else None
        if slot is not None:
            took = ctypes.c_int64(0)
            _lib.check(lib.ob_convmod_bwd_defer(
                dv.data_ptr(), u.data_ptr(), z.data_ptr(), g.data_ptr(), stats.data_ptr(),
                w2.data_ptr(), gamma.data_ptr(), beta.data_ptr(), P, Bt, T, C, K, du.data_ptr(),
                dw.data_ptr(), _lib.ptr(db), dg.data_ptr(), dbt.data_ptr(), ws.data_ptr(), wsb,
                slot[0], slot[1], ctypes.addressof(took), stream), "ob_convmod_bwd_defer")
            if took.value:
                deferred.cm_done(C * (K + 1))
                deferred.keep(ws)
            return du, dw.reshape(wshape), db, dg, dbt, None, None, None
        _lib.check(lib.ob_convmod_bwd(dv.data_ptr(), u.data_ptr(), z.data_ptr(), g.data_ptr(),
                                      stats.data_ptr(),
                                      w2.data_ptr(), gamma.data_ptr(), beta.data_ptr(), P, Bt, T, C,
                                      K, du.data_ptr(), dw.data_ptr(), _lib.ptr(db), dg.data_ptr(),
                                      dbt.data_ptr(), ws.data_ptr(), wsb, _lib.stream_of(dv)),
                   "ob_convmod_bwd")
        return du, dw.reshape(wshape), db, dg, dbt, None, None, None


class _ResidualDropFn(torch.autograd.Function):
    """x + dropout(y) (conformer.py:160-167) with the fused kernels' hash mask."""

    @staticmethod
    def forward(ctx, x, y, p, rng, off, spec):
        x, y = x.contiguous(), y.contiguous()
        out = torch.empty_like(y)
        n = y.shape[-1]
        rows = y.numel() // n
        _lib.check(_lib.load().ob_residual_drop_fwd(x.data_ptr(), y.data_ptr(), rows, n, 1.0, p,
                                                    _lib.ptr(rng), off, None, 0, out.data_ptr(),
                                                    _lib.stream_of(y)), "ob_residual_drop_fwd")
        ctx.meta = (p, rng, off, spec)
        return out

    @staticmethod
    def backward(ctx, g):
        p, rng, off, spec = ctx.meta
        g = g.contiguous()
        n = g.shape[-1]
        rows = g.numel() // n
        gy = spec.take(g)  # formed by the next LN's backward (layernorm.GradScale)
        if gy is None:
            gy = torch.empty_like(g)
            _lib.check(_lib.load().ob_drop_scale_bwd(g.data_ptr(), rows, n, 1.0, p, _lib.ptr(rng),
                                                     off, None, 0, gy.data_ptr(),
                                                     _lib.stream_of(g)), "ob_drop_scale_bwd")
        return g, gy, None, None, None, None


class _BlasPref:
    """Route the GEMMs issued inside the block to one BLAS library. For the conv module's
    fp32 pointwise GEMMs ([B*T, C] x [C, 2C] and [B*T, C] x [C, C]) hipBLASLt's heuristic
    picks 16x16x1 fp32 tiles; rocBLAS's 16x16x4 / 32x32x2 fp32 kernels are faster here
    (tools/blas_pick.py: 118 vs 145 us backward at [23904, 144] x [144, 288])."""

    def __init__(self, lib: str):
        self.lib = lib

    def __enter__(self):
        import warnings

        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            self.prev = torch.backends.cuda.preferred_blas_library()
            torch.backends.cuda.preferred_blas_library(self.lib)

    def __exit__(self, *exc):
        import warnings

        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            torch.backends.cuda.preferred_blas_library(self.prev)
        return False


# pointwise convs the dense kernels do not take run on rocBLAS (measured faster than
# hipBLASLt for these shapes, tools/blas_pick.py)
_PW_BLAS = "cublas"  # ("cublas" selects rocBLAS on ROCm)

# parity-test hooks (tests/test_dense_gpu.py, tests/test_convmod_gpu.py flip them): "blas"
# runs the pointwise convs on the library; False runs pw2 and the residual as two launches
_PW = "hip"
_PW_RESID = True


def _aligned(t: torch.Tensor) -> bool:
    return t.data_ptr() % 16 == 0


def _dense_ok(x2d: torch.Tensor, w: torch.Tensor) -> bool:
    """csrc/dgemm.hip takes this pointwise conv (forward and both backward GEMMs)."""
    if _PW != "hip" or not (x2d.is_cuda and x2d.dtype == torch.float32 == w.dtype):
        return False
    n, k = w.shape
    lib = _lib.load()
    return (x2d.is_contiguous() and w.is_contiguous() and _aligned(x2d) and _aligned(w)
            and lib.ob_dense_supported(k, n) == 1 and lib.ob_dense_supported(n, k) == 1
            and lib.ob_dense_dw_workspace(x2d.shape[0], n, k) > 0)


class _PointwiseFn(torch.autograd.Function):
    """A 1x1 Conv1d on channels-last rows: y = x W^T + b (conformer.py:143,147). Eligible
    shapes run on csrc/dgemm.hip (exact-fp32 products on the bf16 matrix cores: forward,
    dX = dY W, and dW / db through the dW kernel family); others on rocBLAS fp32."""

    @staticmethod
    def forward(ctx, x2d, wp, b):
        # wp: the Conv1d weight parameter itself ([out, in, 1]; a leaf, so its gradient may be
        # finished at the end of the backward, deferred.py); w: its [out, in] view
        w = wp.view(wp.shape[0], -1)
        ctx.wshape = wp.shape
        ctx.hip = _dense_ok(x2d, w)
        if ctx.hip:
            m, k = x2d.shape
            n = w.shape[0]
            y = torch.empty((m, n), dtype=torch.float32, device=x2d.device)
            _lib.check(_lib.load().ob_dense_gemm(x2d.data_ptr(), m, k, w.data_ptr(), 0,
                                                 _lib.ptr(b), n, y.data_ptr(),
                                                 _lib.stream_of(x2d)), "ob_dense_gemm")
        else:
            with _BlasPref(_PW_BLAS):
                y = torch.addmm(b, x2d, w.t()) if b is not None else x2d @ w.t()
        ctx.save_for_backward(x2d, w)
        ctx.has_b = b is not None
        ctx.bias = b
        ctx.wparam = wp
        if ctx.hip:
            deferred.note(wp, b)
        return y

    @staticmethod
    def backward(ctx, g):
        return _pointwise_backward(ctx, g, *ctx.needs_input_grad[:3])


def _pointwise_backward(ctx, g, need_x, need_w, need_b):
    """gx, gw, gb of y = x W^T + b from g = dL/dy (ctx: _PointwiseFn's saved state: x2d, w,
    hip, wshape, has_b, bias, wparam)."""
    x2d, w = ctx.saved_tensors[:2]
    gx = gw = gb = None
    g = g.contiguous()
    need_b = need_b and ctx.has_b
    if ctx.hip and _aligned(g):
        lib = _lib.load()
        m, k = x2d.shape
        n = w.shape[0]
        st = _lib.stream_of(g)
        if need_x:
            gx = torch.empty_like(x2d)
            _lib.check(lib.ob_dense_gemm(g.data_ptr(), m, n, w.data_ptr(), 1, None, k,
                                         gx.data_ptr(), st), "ob_dense_gemm")
        if need_w or need_b:
            gw = deferred.grad_buf(ctx.wparam, ctx.wshape, g.device)  # [out, in, 1]
            gb = deferred.grad_buf(ctx.bias, (n,), g.device) if need_b else None
            wsb = lib.ob_dense_dw_workspace(m, n, k)
            ws = torch.empty((wsb,), dtype=torch.uint8, device=g.device)
            deferred.dense_dw(g, x2d, m, n, k, gw, gb, ws, wsb, st, ctx.wparam, ctx.bias)
            if not need_w:
                gw = None
        return gx, gw, gb
    with _BlasPref(_PW_BLAS):
        if need_x:
            gx = g @ w
        if need_w:
            gw = (g.t() @ x2d).view(ctx.wshape)
    if need_b:
        gb = colsum(g)
    return gx, gw, gb


class _PointwiseResidualFn(torch.autograd.Function):
    """R + dropout(x W^T + b): the conv module's pw2 and its residual tail (conformer.py:147,
    :160-167) in one dgemm launch (ob_dense_gemm_residual_drop; the same arithmetic as
    ob_dense_gemm + ob_residual_drop_fwd). Backward: dR = g; dy = dropout backward of g
    (formed by the next LN's backward, layernorm.GradScale); then pw2's backward."""

    @staticmethod
    def forward(ctx, res, x2d, wp, b, p, rng, off, spec):
        w = wp.view(wp.shape[0], -1)
        ctx.wshape = wp.shape
        ctx.hip = True
        m, k = x2d.shape
        n = w.shape[0]
        out = torch.empty((m, n), dtype=torch.float32, device=x2d.device)
        _lib.check(_lib.load().ob_dense_gemm_residual_drop(
            x2d.data_ptr(), m, k, w.data_ptr(), _lib.ptr(b), n, res.data_ptr(), p, _lib.ptr(rng),
            off, out.data_ptr(), _lib.stream_of(x2d)), "ob_dense_gemm_residual_drop")
        ctx.save_for_backward(x2d, w)
        ctx.has_b = b is not None
        ctx.bias = b
        ctx.wparam = wp
        ctx.meta = (p, rng, off, spec)
        deferred.note(wp, b)
        return out

    @staticmethod
    def backward(ctx, g):
        p, rng, off, spec = ctx.meta
        g = g.contiguous()
        n = g.shape[-1]
        rows = g.numel() // n
        gy = spec.take(g)
        if gy is None:
            gy = torch.empty_like(g)
            _lib.check(_lib.load().ob_drop_scale_bwd(g.data_ptr(), rows, n, 1.0, p, _lib.ptr(rng),
                                                     off, None, 0, gy.data_ptr(),
                                                     _lib.stream_of(g)), "ob_drop_scale_bwd")
        gx, gw, gb = _pointwise_backward(ctx, gy, ctx.needs_input_grad[1],
                                         ctx.needs_input_grad[2], ctx.needs_input_grad[3])
        return g, gx, gw, gb, None, None, None, None


class _BiasReluFn(torch.autograd.Function):
    """relu(y + b[c]) on an NCHW conv output, in place (conformer.py:183-186: Conv2d's bias
    and the ReLU after it); backward gives dy and db in one pass over the planes."""

    @staticmethod
    def forward(ctx, y, bias):
        b, c, h, w = y.shape
        _lib.check(_lib.load().ob_bias_relu_fwd(y.data_ptr(), bias.data_ptr(), b, c, h * w,
                                                _lib.stream_of(y)), "ob_bias_relu_fwd")
        ctx.mark_dirty(y)
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, g):
        (y,) = ctx.saved_tensors
        g = g.contiguous()
        b, c, h, w = y.shape
        gy = torch.empty_like(y)
        db = torch.empty((c,), dtype=torch.float32, device=y.device)
        lib = _lib.load()
        wsb = lib.ob_relu_bias_bwd_workspace(b, c)
        ws = torch.empty((wsb,), dtype=torch.uint8, device=y.device)
        _lib.check(lib.ob_relu_bias_bwd(g.data_ptr(), y.data_ptr(), b, c, h * w, gy.data_ptr(),
                                        db.data_ptr(), ws.data_ptr(), wsb, _lib.stream_of(g)),
                   "ob_relu_bias_bwd")
        return gy, db


def conv2d_bias_relu(x: torch.Tensor, conv: nn.Conv2d) -> torch.Tensor:
    """relu(conv(x)) with the bias add and the ReLU in one HIP pass each way."""
    y = F.conv2d(x, conv.weight, None, conv.stride, conv.padding, conv.dilation, conv.groups)
    if conv.bias is None:
        return F.relu(y)
    return _BiasReluFn.apply(y.contiguous(), conv.bias)


class _SubsampleFn(torch.autograd.Function):
    """Conv2dSubsampling's convolutions (conformer.py:183-186) in csrc/subsample.hip,
    channels-last: [B, T, F] feats -> Y2 [B, T2, F2, C] = relu(conv(relu(conv(x)))). The
    second conv's weight is re-split into its bf16 MFMA images each forward; backward gives
    the four weight / bias gradients (the feats get none)."""

    @staticmethod
    def forward(ctx, x, w0, b0, w2, b2):
        lib = _lib.load()
        bsz, t, f = x.shape
        c = w0.shape[0]
        t1, f1 = (t - 3) // 2 + 1, (f - 3) // 2 + 1
        t2, f2 = (t1 - 3) // 2 + 1, (f1 - 3) // 2 + 1
        img = torch.empty((lib.ob_subsample_image_bytes(c),), dtype=torch.uint8,
                          device=x.device)
        y1 = torch.empty((bsz, t1, f1, c), dtype=torch.float32, device=x.device)
        y2 = torch.empty((bsz, t2, f2, c), dtype=torch.float32, device=x.device)
        st = _lib.stream_of(x)
        _lib.check(lib.ob_subsample_pack(w2.data_ptr(), c, img.data_ptr(), st),
                   "ob_subsample_pack")
        _lib.check(lib.ob_subsample_fwd(x.data_ptr(), bsz, t, f, c, w0.data_ptr(),
                                        b0.data_ptr(), img.data_ptr(), b2.data_ptr(),
                                        y1.data_ptr(), y2.data_ptr(), st), "ob_subsample_fwd")
        ctx.save_for_backward(x, w0, b0, y1, y2, img)
        return y2

    @staticmethod
    def backward(ctx, g):
        if ctx.needs_input_grad[0]:
            raise NotImplementedError("Conv2dSubsampling HIP path: no gradient for the feats")
        x, w0, b0, y1, y2, img = ctx.saved_tensors
        g = g.contiguous()
        bsz, t, f = x.shape
        c = y1.shape[-1]
        lib = _lib.load()
        wsb = lib.ob_subsample_bwd_workspace(bsz, t, f, c)
        ws = torch.empty((wsb,), dtype=torch.uint8, device=x.device)
        dw0 = torch.empty((c, 1, 3, 3), dtype=torch.float32, device=x.device)
        db0 = torch.empty((c,), dtype=torch.float32, device=x.device)
        dw2 = torch.empty((c, c, 3, 3), dtype=torch.float32, device=x.device)
        db2 = torch.empty((c,), dtype=torch.float32, device=x.device)
        _lib.check(lib.ob_subsample_bwd(x.data_ptr(), w0.data_ptr(), b0.data_ptr(), y1.data_ptr(),
                                        y2.data_ptr(), g.data_ptr(),
                                        bsz, t, f, c, img.data_ptr(), dw0.data_ptr(),
                                        db0.data_ptr(), dw2.data_ptr(), db2.data_ptr(),
                                        ws.data_ptr(), wsb, _lib.stream_of(g)),
                   "ob_subsample_bwd")
        return None, dw0, db0, dw2, db2


def _std_conv(conv: nn.Conv2d) -> bool:
    return (conv.kernel_size == (3, 3) and conv.stride == (2, 2) and conv.padding == (0, 0)
            and conv.dilation == (1, 1) and conv.groups == 1 and conv.bias is not None
            and conv.weight.dtype == torch.float32)


def subsample_supported(x: torch.Tensor, conv0: nn.Conv2d, conv2: nn.Conv2d) -> bool:
    """csrc/subsample.hip applies: CUDA fp32 [B, T, F] feats that need no gradient, the
    reference's two 3x3 / stride-2 convolutions, a supported channel count."""
    if os.environ.get("OB_SUBSAMPLE", "hip") != "hip":
        return False
    if not (x.is_cuda and x.dtype == torch.float32 and x.dim() == 3 and not x.requires_grad
            and _std_conv(conv0) and _std_conv(conv2) and conv0.in_channels == 1
            and conv2.in_channels == conv2.out_channels == conv0.out_channels):
        return False
    return _lib.load().ob_subsample_bwd_workspace(x.size(0), x.size(1), x.size(2),
                                                  conv0.out_channels) > 0


def subsample_convs(x: torch.Tensor, conv0: nn.Conv2d, conv2: nn.Conv2d) -> torch.Tensor:
    """[B, T, F] -> [B, T2, F2, C] (channels last) = relu(conv2(relu(conv0(x))))."""
    return _SubsampleFn.apply(x.contiguous(), conv0.weight, conv0.bias, conv2.weight, conv2.bias)


def _pointwise(x: torch.Tensor, conv: nn.Conv1d) -> torch.Tensor:
    c_in = x.shape[-1]
    y = _PointwiseFn.apply(x.reshape(-1, c_in), conv.weight, conv.bias)
    return y.view(*x.shape[:-1], conv.out_channels)


def conv_module_supported(x: torch.Tensor, module) -> bool:
    """The channels-last fused conv module applies (HIP kernels, eligible shapes)."""
    if os.environ.get("OB_FUSED", "1") == "0":
        return False
    dw, bn = module.dw, module.bn
    kt = dw.kernel_size[0]
    ok = (x.is_cuda and x.dtype == torch.float32 and x.dim() == 3
          and dw.groups == dw.in_channels == dw.out_channels == x.size(-1)
          and kt % 2 == 1 and dw.padding[0] == kt // 2 and dw.stride[0] == 1
          and dw.dilation[0] == 1 and bn.affine and not bn.track_running_stats
          and (getattr(module, "quantize_pointwise", False)
               or (module.pw1.kernel_size[0] == 1 and module.pw2.kernel_size[0] == 1)))
    if not ok:
        return False
    return _lib.load().ob_convmod_workspace(1, x.size(0), x.size(1), x.size(-1), kt) > 0


def conv_module_fused(x: torch.Tensor, h: torch.Tensor, module, passes: int, p_drop: float,
                      bitwidth=None):
    """ConvModule.forward (conformer.py:149-167) on [Bt, T, C] without leaving channels-last:
    pw1 / pw2 as GEMMs (bias in the GEMM epilogue), the GLU / depthwise / BatchNorm / swish
    core in csrc/convmod.hip, dropout + residual in one kernel. ``h`` = LN(x)."""
    from .fused import _rng

    bt, t, c = x.shape
    quant = getattr(module, "quantize_pointwise", False)  # ternary pw1/pw2 (opt-in)
    u = module.pw1(h, bitwidth) if quant else _pointwise(h, module.pw1)
    v = _ConvCoreFn.apply(u.reshape(bt * t, 2 * c), module.dw.weight, module.dw.bias,
                          module.bn.weight, module.bn.bias, passes, t, float(module.bn.eps))
    rng, off = _rng(x.device) if p_drop > 0 else (None, 0)
    spec = GradScale(1.0, p_drop, rng, off)
    if not quant and _PW_RESID and _dense_ok(v, module.pw2.weight.view(c, -1)) and _aligned(x):
        # pw2 + dropout + residual in one dgemm launch
        xr = x.contiguous()
        out = _PointwiseResidualFn.apply(xr.view(bt * t, c), v, module.pw2.weight, module.pw2.bias,
                                         float(p_drop), rng, off, spec)
        return attach_grad_scale(out.view(bt, t, c), spec)
    o = module.pw2(v, bitwidth) if quant else _pointwise(v, module.pw2)
    return attach_grad_scale(_ResidualDropFn.apply(x, o.view(bt, t, c), float(p_drop), rng, off,
                                                   spec), spec)
