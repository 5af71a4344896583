"""LayerNorm over the last dim on the HIP library (csrc/layernorm.hip).

Used by the Conformer's ``LayerNorm`` wrapper (reference onebit_asr/conformer.py:19-24,
``nn.LayerNorm(d)``) on a ROCm device for fp32 inputs with d <= 512; other cases run
torch's ``F.layer_norm``. Same arithmetic as torch's (biased variance, eps inside the
square root); the backward's dgamma / dbeta are summed in a fixed order.
"""
from __future__ import annotations

from typing import NamedTuple

import torch
import torch.nn.functional as F

from . import _lib, deferred

__all__ = ["layer_norm", "layer_norm_fork", "layer_norm_amax", "layer_norm_i8", "Int8Act",
           "fused_layernorm_supported", "GradScale", "attach_grad_scale"]

_GSCALE = True  # parity-test hook (False: the consumers run ob_drop_scale_bwd)


class GradScale:
    """Hand-off between a residual tail "R + rscale * rowvalid * dropout(y)" (the fused FFN,
    out_proj and conv-module outputs, conformer.py:39-45, :131-138, :160-167) and the LN that
    normalises that output next. The tail's backward needs dy = rscale * rowvalid *
    drop(gout), gout being exactly the LN backward's dx (the tail's output feeds only that
    LN); the LN backward forms it as a second output (ob_layernorm_bwd_ex) while dx is in
    registers, instead of the tail running ob_drop_scale_bwd over dx afterwards. The tail
    takes the result only if its incoming gradient IS that dx (same storage); anything else
    (another consumer's gradient added in, hooks) falls back to the separate kernel."""

    __slots__ = ("rscale", "p", "rng", "off", "lens", "T", "dx_ptr", "dy2")

    def __init__(self, rscale: float, p: float, rng, off: int, lens=None, T: int = 0):
        self.rscale, self.p, self.rng, self.off = float(rscale), float(p), rng, int(off)
        self.lens, self.T = lens, int(T)
        self.dx_ptr, self.dy2 = 0, None

    def take(self, gout: torch.Tensor):
        dy2, self.dy2 = self.dy2, None
        if dy2 is not None and gout.data_ptr() == self.dx_ptr and gout.numel() == dy2.numel():
            return dy2.view(gout.shape)
        return None


def attach_grad_scale(out: torch.Tensor, spec: GradScale) -> torch.Tensor:
    if _GSCALE and torch.is_grad_enabled():
        out._ob_gscale = spec
    return out


def _bwd_call(lib, g2, x2, weight, mean, rstd, rows, d, dres, dx, dw, db, ws, wsb, spec, stream,
              params=()):
    slot = None
    if (rows > 0 and params and (dw is not None or db is not None)
            and deferred.can_defer(*params)):
        # dgamma / dbeta reduced at the end of the backward with every other LN's (deferred.py)
        slot = deferred.ln_slot(x2.device, stream, d)
    if slot is not None:
        deferred.keep(ws)
        dy2 = torch.empty_like(dx) if spec is not None else None
        st = lib.ob_layernorm_bwd_defer(
            g2.data_ptr(), x2.data_ptr(), _lib.ptr(weight), mean.data_ptr(), rstd.data_ptr(),
            rows, d, _lib.ptr(dres), dx.data_ptr(), _lib.ptr(dw), _lib.ptr(db), ws.data_ptr(), wsb,
            _lib.ptr(dy2), spec.rscale if spec is not None else 1.0,
            spec.p if spec is not None else 0.0, _lib.ptr(spec.rng) if spec is not None else None,
            spec.off if spec is not None else 0,
            _lib.ptr(spec.lens) if spec is not None else None, spec.T if spec is not None else 0,
            slot[0], slot[1], stream)
        if st == _lib.OB_OK:
            deferred.ln_done(1, d)
        if spec is not None:
            spec.dx_ptr, spec.dy2 = dx.data_ptr(), dy2
        return st
    if spec is None:
        if dres is None:
            return lib.ob_layernorm_bwd(g2.data_ptr(), x2.data_ptr(), _lib.ptr(weight),
                                        mean.data_ptr(), rstd.data_ptr(), rows, d, dx.data_ptr(),
                                        _lib.ptr(dw), _lib.ptr(db), ws.data_ptr(), wsb, stream)
        return lib.ob_layernorm_bwd_res(g2.data_ptr(), x2.data_ptr(), _lib.ptr(weight),
                                        mean.data_ptr(), rstd.data_ptr(), rows, d,
                                        dres.data_ptr(), dx.data_ptr(), _lib.ptr(dw),
                                        _lib.ptr(db), ws.data_ptr(), wsb, stream)
    dy2 = torch.empty_like(dx)
    st = lib.ob_layernorm_bwd_ex(g2.data_ptr(), x2.data_ptr(), _lib.ptr(weight), mean.data_ptr(),
                                 rstd.data_ptr(), rows, d, _lib.ptr(dres), dx.data_ptr(),
                                 _lib.ptr(dw), _lib.ptr(db), ws.data_ptr(), wsb, dy2.data_ptr(),
                                 spec.rscale, spec.p, _lib.ptr(spec.rng), spec.off,
                                 _lib.ptr(spec.lens), spec.T, stream)
    spec.dx_ptr, spec.dy2 = dx.data_ptr(), dy2
    return st


def fused_layernorm_supported(x: torch.Tensor, d: int) -> bool:
    return x.is_cuda and x.dtype == torch.float32 and 1 <= d <= 512


class _LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, eps, spec=None, pre=None, pair=None):
        """pre: this LN's (y, mean, rstd), already formed by the previous LN's pair launch;
        pair: (weight2, bias2, eps2, box) -- also form the NEXT LN of y in the same launch
        (ob_layernorm_fwd_pair) and put its (y2, mean2, rstd2) into box."""
        d = x.shape[-1]
        ctx.spec = spec
        x2 = x.contiguous().view(-1, d)
        rows = x2.shape[0]
        need = any(ctx.needs_input_grad[:3])
        lib = _lib.load()
        ctx.link = None
        if pre is not None:
            y, mean, rstd = pre[:3]
            ctx.pre_link = pre[3] if len(pre) > 3 else None
            if pair is not None and len(pair) > 4:
                # the next LN of y was formed too (by the GEMM epilogue that produced x): hand
                # it on as a pair launch would
                w2, b2, eps2, box, (y2, mean2, rstd2) = pair
                link = _PairLink(x2, weight, bias, mean, rstd, spec, ctx.needs_input_grad[:3])
                ctx.link = link
                box.append((w2, b2, float(eps2), y2, mean2, rstd2, link))
        elif pair is not None:
            w2, b2, eps2, box = pair
            y = torch.empty_like(x2)
            mean = torch.empty((rows,), dtype=torch.float32, device=x.device)
            rstd = torch.empty((rows,), dtype=torch.float32, device=x.device)
            y2 = torch.empty_like(x2)
            mean2 = torch.empty((rows,), dtype=torch.float32, device=x.device)
            rstd2 = torch.empty((rows,), dtype=torch.float32, device=x.device)
            _lib.check(lib.ob_layernorm_fwd_pair(
                x2.data_ptr(), _lib.ptr(weight), _lib.ptr(bias), _lib.ptr(w2), _lib.ptr(b2), rows,
                d, float(eps), float(eps2), y.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                y2.data_ptr(), mean2.data_ptr(), rstd2.data_ptr(), _lib.stream_of(x2)),
                "ob_layernorm_fwd_pair")
            # the consumer's backward may run both LN backwards in one launch: it finds this
            # LN's saved state here and leaves the result for this node's backward
            link = _PairLink(x2, weight, bias, mean, rstd, spec, ctx.needs_input_grad[:3])
            ctx.link = link
            box.append((w2, b2, float(eps2), y2, mean2, rstd2, link))
        else:
            y = torch.empty_like(x2)
            mean = torch.empty((rows,), dtype=torch.float32, device=x.device) if need else None
            rstd = torch.empty((rows,), dtype=torch.float32, device=x.device) if need else None
            _lib.check(lib.ob_layernorm_fwd(x2.data_ptr(), _lib.ptr(weight), _lib.ptr(bias), rows,
                                            d, float(eps), y.data_ptr(), _lib.ptr(mean),
                                            _lib.ptr(rstd), _lib.stream_of(x2)),
                       "ob_layernorm_fwd")
        if need:
            ctx.save_for_backward(x2, weight, mean, rstd)
            ctx.has = (weight is not None, bias is not None)
            ctx.params = (weight, bias)
            deferred.note(weight, bias)
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, gy):
        link = getattr(ctx, "link", None)
        if link is not None and link.result is not None:
            du, dw, db, deferred1 = link.result
            link.result = None
            if gy.data_ptr() != du.data_ptr():
                # the output had a consumer besides the next LN: autograd summed that
                # consumer's gradient into du (gy = du + g_other). The LN backward is linear
                # in its output gradient, so the pair's result is completed with the LN
                # backward of g_other (to the rounding of the subtraction).
                return _pair_correction(ctx, gy, du, dw, db, deferred1)
            return du.view(gy.shape), dw, db, None, None, None, None
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
        _lib.check(_bwd_call(lib, g2, x2, weight, mean, rstd, rows, d, None, dx, dw, db, ws, wsb,
                             ctx.spec, _lib.stream_of(g2), ctx.params), "ob_layernorm_bwd")
        return dx.view(gy.shape), dw, db, None, None, None, None


# parity-test hooks (tests/test_stacked_step_gpu.py): False = every LN its own launch /
# the pair's backwards one by one
_PAIR = True
_PAIR_BWD = True


class _PairLink:
    """The first LN of a pair (its saved input / statistics / parameters), shared with the
    second LN's fork node, whose backward can then run both LN backwards in one launch
    (ob_layernorm_bwd_pair) and leave (dx, dgamma, dbeta) here for the first LN's node."""

    __slots__ = ("x2", "weight", "bias", "mean", "rstd", "spec", "need", "result")

    def __init__(self, x2, weight, bias, mean, rstd, spec, need):
        self.x2, self.weight, self.bias, self.mean, self.rstd = x2, weight, bias, mean, rstd
        self.spec, self.need, self.result = spec, tuple(need), None


def _take_pre(x: torch.Tensor, weight, bias, eps):
    """The (y, mean, rstd) a pair launch already formed for LN(x) with these parameters."""
    pre = getattr(x, "_ob_ln_pre", None)
    if pre is None or pre[0] is not weight or pre[1] is not bias or pre[2] != float(eps):
        return None
    x._ob_ln_pre = None
    return pre[3:]


def _take_pre2(x: torch.Tensor, weight, bias, eps):
    """The (y2, mean2, rstd2) of the LN following LN(x), formed with LN(x) by the epilogue of
    the GEMM that produced x (fused.ffn_residual's ln_next)."""
    pre = getattr(x, "_ob_ln_pre2", None)
    if pre is None:
        return None
    x._ob_ln_pre2 = None
    if pre[0] is not weight or pre[1] is not bias or pre[2] != float(eps):
        return None
    return pre[3:6]


def layer_norm(x: torch.Tensor, weight, bias, eps: float = 1e-5) -> torch.Tensor:
    d = x.shape[-1]
    if not fused_layernorm_supported(x, d):
        return F.layer_norm(x, (d,), weight, bias, eps)
    return _LayerNormFn.apply(x, weight, bias, eps, getattr(x, "_ob_gscale", None),
                              _take_pre(x, weight, bias, eps))


def layer_norm_pair(x: torch.Tensor, weight, bias, eps, weight2, bias2, eps2) -> torch.Tensor:
    """LN(x) whose output's next LN (weight2, bias2, eps2) is formed in the same launch and
    picked up by that LN's layer_norm / layer_norm_fork call (bit-identical to two launches).
    Training only (grad enabled): inference consumers may take the int8 LN instead."""
    d = x.shape[-1]
    if not (_PAIR and torch.is_grad_enabled() and fused_layernorm_supported(x, d)):
        return layer_norm(x, weight, bias, eps)
    box = []
    pre = _take_pre(x, weight, bias, eps)
    pre2 = _take_pre2(x, weight2, bias2, eps2) if pre is not None else None
    pair = (weight2, bias2, eps2, box) if pre2 is None else (weight2, bias2, eps2, box, pre2)
    y = _LayerNormFn.apply(x, weight, bias, eps, getattr(x, "_ob_gscale", None), pre, pair)
    if box:
        y._ob_ln_pre = box[0]
    return y


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


class Int8Act(NamedTuple):
    """An activation held as its int8 image in HBM: q [rows, d] int8 at the scale
    127 / max(amax, 1e-5), amax device fp32 [1], shape = the fp32 tensor's shape."""
    q: torch.Tensor
    amax: torch.Tensor
    shape: torch.Size


@torch.no_grad()
def layer_norm_i8(x: torch.Tensor, weight, bias, eps: float = 1e-5) -> Int8Act:
    """Inference: LN(x) as an int8 operand (ob_layernorm_fwd_i8): the absmax pass and a
    second LN pass that writes the int8 image only -- the fp32 LN(x) never reaches HBM, and
    the int8 BitLinears that consume it read d bytes per row instead of 4d."""
    d = x.shape[-1]
    x2 = x.contiguous().view(-1, d)
    rows = x2.shape[0]
    yq = torch.empty((rows, d), dtype=torch.int8, device=x.device)
    amax = torch.empty((1,), dtype=torch.float32, device=x.device)
    lib = _lib.load()
    wsb = lib.ob_layernorm_fwd_amax_workspace(1)
    ws = torch.empty((wsb,), dtype=torch.uint8, device=x.device)
    _lib.check(lib.ob_layernorm_fwd_i8(x2.data_ptr(), _lib.ptr(weight), _lib.ptr(bias), rows, d,
                                       float(eps), 1, amax.data_ptr(), yq.data_ptr(),
                                       ws.data_ptr(), wsb, _lib.stream_of(x2)),
               "ob_layernorm_fwd_i8")
    return Int8Act(yq, amax, x.shape)


class _LayerNormForkFn(torch.autograd.Function):
    """(LN(x), x) for a residual junction x -> (LN -> module) + x: the backward receives both
    branches' gradients and forms dx = LN_backward(dy) + dres in the LN backward kernel,
    instead of autograd's separate add over the [rows, d] tensor."""

    @staticmethod
    def forward(ctx, x, weight, bias, eps, spec=None, pre=None):
        y = _LayerNormFn.forward(ctx, x, weight, bias, eps, spec, pre)
        return y, x.view_as(x)

    @staticmethod
    def backward(ctx, gy, gres):
        link = getattr(ctx, "pre_link", None)
        if (_PAIR_BWD and link is not None and gy is not None and ctx.spec is None
                and any(link.need)):
            return _pair_backward(ctx, link, gy, gres)
        if gres is None:
            return _LayerNormFn.backward(ctx, gy)[:6]
        x2, weight, mean, rstd = ctx.saved_tensors
        rows, d = x2.shape
        if gy is None:
            return gres, None, None, None, None, None
        g2 = gy.contiguous().view(rows, d)
        r2 = gres.contiguous().view(rows, d)
        dx = torch.empty_like(x2)
        has_w, has_b = ctx.has
        dw = torch.empty((d,), dtype=torch.float32, device=x2.device) if has_w and ctx.needs_input_grad[1] else None
        db = torch.empty((d,), dtype=torch.float32, device=x2.device) if has_b and ctx.needs_input_grad[2] else None
        lib = _lib.load()
        wsb = lib.ob_layernorm_bwd_workspace(rows, d)
        ws = torch.empty((max(wsb, 1),), dtype=torch.uint8, device=x2.device)
        _lib.check(_bwd_call(lib, g2, x2, weight, mean, rstd, rows, d, r2, dx, dw, db, ws, wsb,
                             ctx.spec, _lib.stream_of(g2), ctx.params), "ob_layernorm_bwd_res")
        return dx.view(gy.shape), dw, db, None, None, None


def _pair_backward(ctx, link, gy, gres):
    """Both LN backwards of a pair in one launch: this (second) LN's dx + gres feeds the first
    LN's backward in registers; the first LN's (dx, dgamma, dbeta) are left on the link."""
    y1, w2, mean2, rstd2 = ctx.saved_tensors
    rows, d = y1.shape
    g2 = gy.contiguous().view(rows, d)
    r2 = gres.contiguous().view(rows, d) if gres is not None else None
    u = link.x2
    du = torch.empty_like(u)
    has_w2, has_b2 = ctx.has
    dw2 = torch.empty((d,), dtype=torch.float32, device=u.device) if has_w2 and ctx.needs_input_grad[1] else None
    db2 = torch.empty((d,), dtype=torch.float32, device=u.device) if has_b2 and ctx.needs_input_grad[2] else None
    w1, b1 = link.weight, link.bias
    dw1 = torch.empty((d,), dtype=torch.float32, device=u.device) if w1 is not None and link.need[1] else None
    db1 = torch.empty((d,), dtype=torch.float32, device=u.device) if b1 is not None and link.need[2] else None
    lib = _lib.load()
    stream = _lib.stream_of(g2)
    wsb = lib.ob_layernorm_bwd_pair_workspace(rows, d)
    ws = torch.empty((max(wsb, 1),), dtype=torch.uint8, device=u.device)
    table, s2, s1 = None, -1, -1
    d2 = rows > 0 and (dw2 is not None or db2 is not None) and deferred.can_defer(*ctx.params)
    d1 = rows > 0 and (dw1 is not None or db1 is not None) and deferred.can_defer(w1, b1)
    n_def = int(d2) + int(d1)
    if n_def:
        t = deferred.ln_slot(u.device, stream, d, n_def)
        if t is not None:
            table = t[0]
            s2 = t[1] if d2 else -1
            s1 = t[1] + int(d2) if d1 else -1
        else:
            n_def = 0
    if n_def:
        deferred.keep(ws)
    spec = link.spec
    dy2 = torch.empty_like(du) if spec is not None else None
    _lib.check(lib.ob_layernorm_bwd_pair(
        g2.data_ptr(), y1.data_ptr(), _lib.ptr(w2), mean2.data_ptr(), rstd2.data_ptr(),
        _lib.ptr(r2), u.data_ptr(), _lib.ptr(w1), link.mean.data_ptr(), link.rstd.data_ptr(),
        rows, d, du.data_ptr(), _lib.ptr(dw2), _lib.ptr(db2), _lib.ptr(dw1), _lib.ptr(db1),
        ws.data_ptr(), wsb, _lib.ptr(dy2), spec.rscale if spec is not None else 1.0,
        spec.p if spec is not None else 0.0, _lib.ptr(spec.rng) if spec is not None else None,
        spec.off if spec is not None else 0, _lib.ptr(spec.lens) if spec is not None else None,
        spec.T if spec is not None else 0, table, s2, s1, stream), "ob_layernorm_bwd_pair")
    if n_def:
        deferred.ln_done(n_def, d)
    if spec is not None:
        spec.dx_ptr, spec.dy2 = du.data_ptr(), dy2
    link.result = (du, dw1, db1, s1 >= 0)
    # du goes to the first LN's node as this node's input gradient; that node returns it
    return du.view(gy.shape), dw2, db2, None, None, None


def _pair_correction(ctx, gy, du, dw1, db1, deferred1):
    """The first LN of a pair whose output had another consumer: du, dw1, db1 are its
    backward for the pair consumer's gradient only; add the LN backward of the rest
    (g_other = gy - du) -- dgamma / dbeta after the deferred tables have written theirs.

    A fallback, accurate to the rounding of the TOTAL gradient: g_other is recovered by a
    subtraction, so each element carries an error up to ulp(|du|); when |du| >> |g_other| the
    other consumer's share is resolved only to that absolute level (tests/
    test_defer_safety_gpu.py bounds it at 1e-5 of max |dx|). The Conformer never takes this
    path (a block's output feeds only the LN pair), so it guards correctness, not speed."""
    x2, weight, mean, rstd = ctx.saved_tensors
    rows, d = x2.shape
    g_other = (gy.reshape(rows, d) - du.view(rows, d)).contiguous()
    dx = torch.empty_like(x2)
    dw = torch.empty((d,), dtype=torch.float32, device=x2.device) if dw1 is not None else None
    db = torch.empty((d,), dtype=torch.float32, device=x2.device) if db1 is not None else None
    lib = _lib.load()
    wsb = lib.ob_layernorm_bwd_workspace(rows, d)
    ws = torch.empty((max(wsb, 1),), dtype=torch.uint8, device=x2.device)
    _lib.check(lib.ob_layernorm_bwd_res(g_other.data_ptr(), x2.data_ptr(), _lib.ptr(weight),
                                        mean.data_ptr(), rstd.data_ptr(), rows, d,
                                        du.data_ptr(), dx.data_ptr(), _lib.ptr(dw), _lib.ptr(db),
                                        ws.data_ptr(), wsb, _lib.stream_of(g_other)),
               "ob_layernorm_bwd_res")
    for pending, extra, param in ((dw1, dw, weight), (db1, db, ctx.params[1])):
        if extra is None:
            continue
        if deferred1:  # the table writes `pending` at the flush: add to the installed .grad
            deferred.add_grad_after_flush(param, extra)
        else:
            pending.add_(extra)
    return dx.view(gy.shape), dw1, db1, None, None, None, None


def layer_norm_fork(x: torch.Tensor, weight, bias, eps: float = 1e-5):
    """(LN(x), x_residual): use x_residual for the junction's skip connection so the
    backward adds the two gradient branches inside the LN backward kernel."""
    d = x.shape[-1]
    if not fused_layernorm_supported(x, d) or not torch.is_grad_enabled() or not x.requires_grad:
        return layer_norm(x, weight, bias, eps), x
    return _LayerNormForkFn.apply(x, weight, bias, eps, getattr(x, "_ob_gscale", None),
                                  _take_pre(x, weight, bias, eps))
