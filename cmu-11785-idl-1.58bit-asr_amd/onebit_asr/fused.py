"""Fused BitLinear call sites: the elementwise ops around a QuantizedLinear at its call
sites in the reference, folded into the ternary GEMM's epilogue (csrc/tgemm.hip) and one
elementwise backward kernel (csrc/fused.hip).

* ``ffn_residual`` -- FeedForwardModule.forward after its LayerNorm (conformer.py:34-45):
  ``x + 0.5 * dropout(lin2(dropout(swish(lin1(h)))))`` as two GEMM launches forward
  (lin1 -> swish -> dropout; lin2 -> dropout -> *0.5 -> +x) and, backward, one dropout/scale
  kernel, lin2's dX GEMM with the dropout and swish backward in its epilogue, and the two
  layers' dX / dW kernels. torch's unfused sequence is 5 extra elementwise kernels forward
  and 4 backward, each a full pass over a [rows, 576] or [rows, 144] fp32 tensor.
* ``linear_residual`` -- MHSA's tail (conformer.py:131-138):
  ``x + pad_zero(dropout(out_proj(ctx)))`` as one GEMM launch (+ one kernel backward).

Results equal the unfused module code: with dropout off (p = 0 or eval) bit for bit -- the
epilogue performs the same fp32 operations in the same order -- and with dropout on, the
same function of a different (hash-based) keep mask.

Dropout masks: one device {seed, counter} per device; ``advance_step`` (called once per
training step, also inside a captured step) moves the counter by 2^32 and each call site
draws with counter + its own host-side offset, so no per-call device copy is needed and a
replayed graph draws fresh masks every step. The backward regenerates the forward's mask
from the same (seed, counter + offset).
"""
from __future__ import annotations

import ctypes
import os
from typing import Dict, Optional

import torch

from . import _lib, deferred
from .layernorm import GradScale, Int8Act, attach_grad_scale
from .quant import PassBits, QuantizedLinear

__all__ = ["ffn_residual", "linear_residual", "fused_supported", "advance_step",
           "i8_fused_supported", "ffn_residual_i8", "linear_residual_i8", "qkv_projections",
           "i8_linear"]

# parity-test hooks (tests/test_fused_gpu.py): False = q / k / v dW, forward one by one
_DW_GROUP = True
# q / k / v input gradients summed in one launch (tests flip it to compare with the three
# launches: plain dX of q, then k and v accumulated through the residual epilogue)
_DX_SUM = True
_QKV_FWD_GROUP = True
_STATE: Dict[torch.device, list] = {}  # device -> [rng tensor {seed, counter}, host offset]


def _seed() -> int:
    return (int(torch.initial_seed()) * 0x9E3779B97F4A7C15 + 0x5851F42D) & ((1 << 62) - 1)


def _rng(device: torch.device):
    st = _STATE.get(device)
    if st is None:
        st = [torch.tensor([_seed(), 0], dtype=torch.int64, device=device), 0]
        _STATE[device] = st
    off = st[1]
    st[1] = (st[1] + 1) & ((1 << 32) - 1)
    return st[0], off


def rng_snapshot(device: torch.device):
    """The fused call sites' dropout state on ``device`` ({seed, counter} tensor + the host
    offset), for undoing warm-up steps (graph_step.GraphedTrainStep)."""
    st = _STATE.get(device)
    return None if st is None else (st[0].clone(), st[1])


def rng_restore(device: torch.device, snap) -> None:
    """Back to ``snap``; ``None`` (no state existed) = the state a first draw would create,
    written in place (a capture that follows must not allocate)."""
    st = _STATE.get(device)
    if snap is None:
        if st is not None:
            st[0].copy_(torch.tensor([_seed(), 0], dtype=torch.int64))
            st[1] = 0
        return
    if st is None:
        _STATE[device] = [snap[0].clone(), snap[1]]
    else:
        st[0].copy_(snap[0])  # in place: captured kernels keep reading this tensor
        st[1] = snap[1]


def advance_step(device: torch.device) -> None:
    """New dropout masks for every fused call site of the next step (one tiny kernel)."""
    st = _STATE.get(device)
    if st is not None:
        st[0][1:].add_(1 << 32)


def fused_supported(x: torch.Tensor, *layers: QuantizedLinear, bitwidth=None) -> bool:
    if os.environ.get("OB_FUSED", "1") == "0":
        return False
    if not (isinstance(bitwidth, PassBits) or bitwidth in (1, 2)):
        return False  # 32 (F.linear), DynamicBitwidth and invalid values take the module path
    for m in layers:  # packed-ternary layers are inference-only: training raises here too
        if m._packed is not None:
            m._check_packed_use(bitwidth)
    return x.is_cuda and x.dtype == torch.float32 and all(
        m.act_quant is None and m.quant_off in (None, "bf16w") for m in layers)


def _bits_args(bitwidth):
    """(P, pass_bits tensor or None, bits for single-pass entries)."""
    if isinstance(bitwidth, PassBits):
        return bitwidth.passes, bitwidth.tensor, None
    return 1, None, int(bitwidth)


class Codes(tuple):
    """(codes2, codes1, codes2_t, codes1_t) of one layer, with the C ABI's alpha_raw for its
    forward and dX GEMMs: 1 / 1 for ternary codes; 2 / 2 for the quant-off ceiling
    (quant_off="bf16w": the slots hold the bf16 weight images W [N][K] / W^T [K][N], no
    alpha), whose weight gradient is a plain dense dW (dense=True)."""
    fwd_raw = 1
    dx_raw = 1
    dense = False


def _codes(layer: QuantizedLinear, P: int, bits: Optional[int]):
    """(codes2, codes1, codes2_t, codes1_t); single-pass: both slots hold the layer's bits."""
    if layer.quant_off == "bf16w":
        img, img_t = layer._bf16_images()
        c = Codes((img, img, img_t, img_t))
        c.fwd_raw, c.dx_raw, c.dense = 2, 2, True
        return c
    if P == 1 and bits is not None and bits != 2:
        c, ct = layer._codes(bits)
        return Codes((c, c, ct, ct))
    c2, c2t = layer._codes(2)
    if P == 1:
        return Codes((c2, c2, c2t, c2t))
    c1, c1t = layer._codes(1)
    return Codes((c2, c1, c2t, c1t))


def _dx(lib, dy, P, m, n, codes, pb, alpha, k, stream):
    dx = torch.empty((P * m, k), dtype=torch.float32, device=dy.device)
    _lib.check(lib.ob_bitlinear_bwd_dx_passes(dy.data_ptr(), P, m, n, codes[2].data_ptr(),
                                              codes[3].data_ptr(), pb.data_ptr(), alpha.data_ptr(),
                                              codes.dx_raw, k, dx.data_ptr(), stream)
               if pb is not None else
               lib.ob_bitlinear_bwd_dx(dy.data_ptr(), m, n, codes[2].data_ptr(), alpha.data_ptr(),
                                       codes.dx_raw, k, dx.data_ptr(), stream), "ob_bitlinear_bwd_dx")
    return dx


def _dw(lib, dy, x, P, m, n, k, weight, alpha, has_bias, pb, bits, stream, bias=None,
        dense=False):
    """dW / dalpha / db of one BitLinear; the finish deferred to the end of the backward
    (deferred.py) when nothing can read these gradients before it. dense (quant-off): the
    plain dW = dY^T X and db on the same kernels, no STE mask, no alpha gradient."""
    gw = deferred.grad_buf(weight)
    gb = deferred.grad_buf(bias, (n,), dy.device) if has_bias else None
    if dense:
        wsb = lib.ob_dense_dw_workspace(P * m, n, k)
        if not wsb:  # shapes off the dW kernels: library fp32
            from .linear import colsum

            return dy.t() @ x, None, colsum(dy) if has_bias else None
        ws = torch.empty((wsb,), dtype=torch.uint8, device=dy.device)
        deferred.dense_dw(dy, x, P * m, n, k, gw, gb, ws, wsb, stream, weight, bias)
        return gw, None, gb
    ga = deferred.grad_buf(alpha, (), dy.device)
    if pb is not None and deferred.dwg_take(dy, x, P, m, n, k, gw, gb, stream, weight, bias,
                                            alpha=alpha, ga=ga, pass_bits=pb):
        return gw, ga, gb  # computed by the grouped launch at the end of the backward
    slot = (deferred.dw_slot(dy.device, stream)
            if pb is not None and deferred.can_defer(weight, alpha, bias) else None)
    if slot is not None:
        wsb = lib.ob_bitlinear_bwd_dw_passes_workspace(P, m, n, k)
        ws = torch.empty((max(wsb, 1),), dtype=torch.uint8, device=dy.device)
        nb = ctypes.c_int64(0)
        _lib.check(lib.ob_bitlinear_bwd_dw_passes_defer(
            dy.data_ptr(), x.data_ptr(), P, m, n, k, weight.data_ptr(), alpha.data_ptr(), 1,
            pb.data_ptr(), gw.data_ptr(), ga.data_ptr(), _lib.ptr(gb), ws.data_ptr(), wsb,
            slot[0], slot[1], slot[2], ctypes.addressof(nb), stream),
            "ob_bitlinear_bwd_dw_passes_defer")
        deferred.dw_done(1, nb.value)
        deferred.keep(ws)
        return gw, ga, gb
    if pb is not None:
        wsb = lib.ob_bitlinear_bwd_dw_passes_workspace(P, m, n, k)
        ws = torch.empty((max(wsb, 1),), dtype=torch.uint8, device=dy.device)
        st = lib.ob_bitlinear_bwd_dw_passes(dy.data_ptr(), x.data_ptr(), P, m, n, k,
                                            weight.data_ptr(), alpha.data_ptr(), 1, pb.data_ptr(),
                                            gw.data_ptr(), ga.data_ptr(), _lib.ptr(gb),
                                            ws.data_ptr(), wsb, stream)
    else:
        wsb = lib.ob_bitlinear_bwd_dw_workspace(m, n, k)
        ws = torch.empty((max(wsb, 1),), dtype=torch.uint8, device=dy.device)
        st = lib.ob_bitlinear_bwd_dw(dy.data_ptr(), x.data_ptr(), m, n, k, weight.data_ptr(),
                                     alpha.data_ptr(), 1, bits, gw.data_ptr(), ga.data_ptr(),
                                     _lib.ptr(gb), ws.data_ptr(), wsb, stream)
    _lib.check(st, "ob_bitlinear_bwd_dw")
    return gw, ga, gb


class _FFNFn(torch.autograd.Function):
    """conformer.py:36-45 from the LN output h: x + 0.5 * drop(lin2(drop(swish(lin1(h)))))."""

    @staticmethod
    def forward(ctx, h, x, w1, a1, b1, w2, a2, b2, meta, lnreq=None):
        """lnreq: ([(weight, bias, eps)] x 1 or 2, box) -- the LayerNorm(s) that read the output
        next, formed in lin2's epilogue (ob_bitlinear_fwd_residual_ln); their (y, mean, rstd)
        go into box (left empty when the launch shape does not take them)."""
        P, pb, bits, codes1, codes2, p, rng, off1, off2, _ = meta
        rows, k = h.shape
        m = rows // P
        n1, n2 = w1.shape[0], w2.shape[0]
        lib = _lib.load()
        stream = _lib.stream_of(h)
        pre = torch.empty((rows, n1), dtype=torch.float32, device=h.device)
        act = torch.empty((rows, n1), dtype=torch.float32, device=h.device)
        _lib.check(lib.ob_bitlinear_fwd_swish_drop(
            h.data_ptr(), P, m, k, codes1[0].data_ptr(), codes1[1].data_ptr(), _lib.ptr(pb),
            a1.data_ptr(), codes1.fwd_raw, _lib.ptr(b1), n1, p, _lib.ptr(rng), off1, pre.data_ptr(),
            act.data_ptr(), stream), "ob_bitlinear_fwd_swish_drop")
        out = torch.empty((rows, n2), dtype=torch.float32, device=h.device)
        st = _lib.OB_ERR_SHAPE
        if lnreq is not None:
            reqs, box = lnreq
            lno = [(torch.empty_like(out), torch.empty((rows,), dtype=torch.float32, device=h.device),
                    torch.empty((rows,), dtype=torch.float32, device=h.device)) for _ in reqs]
            r1, o1 = (reqs[1], lno[1]) if len(reqs) > 1 else ((None, None, 0.0), (None,) * 3)
            st = lib.ob_bitlinear_fwd_residual_ln(
                act.data_ptr(), P, m, n1, codes2[0].data_ptr(), codes2[1].data_ptr(),
                _lib.ptr(pb), a2.data_ptr(), codes2.fwd_raw, _lib.ptr(b2), n2, x.data_ptr(), 0.5,
                p, _lib.ptr(rng), off2, None, 0, out.data_ptr(), len(reqs), _lib.ptr(reqs[0][0]),
                _lib.ptr(reqs[0][1]), float(reqs[0][2]), *(_lib.ptr(t) for t in lno[0]),
                _lib.ptr(r1[0]), _lib.ptr(r1[1]), float(r1[2]), *(_lib.ptr(t) for t in o1), stream)
            if st == _lib.OB_OK:
                box.extend((*r, *o) for r, o in zip(reqs, lno))
            elif st != _lib.OB_ERR_SHAPE:
                _lib.check(st, "ob_bitlinear_fwd_residual_ln")
        if st != _lib.OB_OK:
            _lib.check(lib.ob_bitlinear_fwd_residual(
                act.data_ptr(), P, m, n1, codes2[0].data_ptr(), codes2[1].data_ptr(),
                _lib.ptr(pb), a2.data_ptr(), codes2.fwd_raw, _lib.ptr(b2), n2, x.data_ptr(), 0.5,
                p, _lib.ptr(rng), off2, None, 0, out.data_ptr(), stream),
                "ob_bitlinear_fwd_residual")
        ctx.meta = meta
        ctx.has_bias = (b1 is not None, b2 is not None)
        ctx.biases = (b1, b2)
        deferred.note(w1, a1, b1, w2, a2, b2)
        ctx.save_for_backward(h, pre, act, w1, a1, w2, a2)
        return out

    @staticmethod
    def backward(ctx, gout):
        h, pre, act, w1, a1, w2, a2 = ctx.saved_tensors
        P, pb, bits, codes1, codes2, p, rng, off1, off2, spec = ctx.meta
        gout = gout.contiguous()
        rows, k = h.shape
        m = rows // P
        n1, n2 = w1.shape[0], w2.shape[0]
        lib = _lib.load()
        stream = _lib.stream_of(gout)
        dy2 = spec.take(gout)  # formed by the next LN's backward (layernorm.GradScale)
        if dy2 is None:
            dy2 = torch.empty_like(gout)
            _lib.check(lib.ob_drop_scale_bwd(gout.data_ptr(), rows, n2, 0.5, p, _lib.ptr(rng),
                                             off2, None, 0, dy2.data_ptr(), stream),
                       "ob_drop_scale_bwd")
        dpre = torch.empty((rows, n1), dtype=torch.float32, device=gout.device)
        _lib.check(lib.ob_bitlinear_bwd_dx_swish_drop(
            dy2.data_ptr(), P, m, n2, codes2[2].data_ptr(), codes2[3].data_ptr(), _lib.ptr(pb),
            a2.data_ptr(), codes2.dx_raw, n1, pre.data_ptr(), p, _lib.ptr(rng), off1,
            dpre.data_ptr(), stream),
            "ob_bitlinear_bwd_dx_swish_drop")
        gw2, ga2, gb2 = _dw(lib, dy2, act, P, m, n2, n1, w2, a2, ctx.has_bias[1], pb, bits, stream,
                            ctx.biases[1], codes2.dense)
        gh = _dx(lib, dpre, P, m, n1, codes1, pb, a1, k, stream) if ctx.needs_input_grad[0] else None
        gw1, ga1, gb1 = _dw(lib, dpre, h, P, m, n1, k, w1, a1, ctx.has_bias[0], pb, bits, stream,
                            ctx.biases[0], codes1.dense)
        return gh, gout, gw1, ga1, gb1, gw2, ga2, gb2, None, None


# parity-test hook (tests/test_fused_gpu.py): False = the LNs after the FFN their own launches
_LN_EPI = True


class _LinearResidualFn(torch.autograd.Function):
    """conformer.py:131-138: R + rscale * rowvalid * drop(lin(x))."""

    @staticmethod
    def forward(ctx, x, resid, w, a, b, meta):
        P, pb, bits, codes, rscale, p, rng, off, lens, T, _ = meta
        rows, k = x.shape
        m = rows // P
        n = w.shape[0]
        lib = _lib.load()
        out = torch.empty((rows, n), dtype=torch.float32, device=x.device)
        _lib.check(lib.ob_bitlinear_fwd_residual(
            x.data_ptr(), P, m, k, codes[0].data_ptr(), codes[1].data_ptr(), _lib.ptr(pb),
            a.data_ptr(), codes.fwd_raw, _lib.ptr(b), n, resid.data_ptr(), rscale, p, _lib.ptr(rng), off,
            _lib.ptr(lens), T, out.data_ptr(), _lib.stream_of(x)), "ob_bitlinear_fwd_residual")
        ctx.meta = meta
        ctx.has_bias = b is not None
        ctx.bias = b
        deferred.note(w, a, b)
        ctx.save_for_backward(x, w, a)
        return out

    @staticmethod
    def backward(ctx, gout):
        x, w, a = ctx.saved_tensors
        P, pb, bits, codes, rscale, p, rng, off, lens, T, spec = ctx.meta
        gout = gout.contiguous()
        rows, k = x.shape
        m = rows // P
        n = w.shape[0]
        lib = _lib.load()
        stream = _lib.stream_of(gout)
        dy = spec.take(gout)  # formed by the next LN's backward (layernorm.GradScale)
        if dy is None:
            dy = torch.empty_like(gout)
            _lib.check(lib.ob_drop_scale_bwd(gout.data_ptr(), rows, n, rscale, p, _lib.ptr(rng),
                                             off, _lib.ptr(lens), T, dy.data_ptr(), stream),
                       "ob_drop_scale_bwd")
        gx = _dx(lib, dy, P, m, n, codes, pb, a, k, stream) if ctx.needs_input_grad[0] else None
        gw, ga, gb = _dw(lib, dy, x, P, m, n, k, w, a, ctx.has_bias, pb, bits, stream, ctx.bias,
                         codes.dense)
        return gx, gout, gw, ga, gb, None


class _QKVFn(torch.autograd.Function):
    """The three projections of one input (conformer.py:111-113: q/k/v_proj(x) on the same
    LN output) as one autograd node: three GEMMs forward; backward, dX of q plain and the dX
    GEMMs of k and v accumulated into it through the GEMM's residual epilogue (C = R + y,
    in place), instead of autograd's two separate adds over [rows, d]; three dW GEMMs."""

    @staticmethod
    def forward(ctx, h, wq, aq, bq, wk, ak, bk, wv, av, bv, meta):
        P, pb, bits, codes = meta
        rows, k = h.shape
        m = rows // P
        lib = _lib.load()
        stream = _lib.stream_of(h)
        outs = []
        if pb is not None and _QKV_FWD_GROUP and wq.shape == wk.shape == wv.shape and \
                codes[0].fwd_raw == codes[1].fwd_raw == codes[2].fwd_raw:
            # the three projections in one launch (their column tiles side by side)
            n = wq.shape[0]
            outs = [torch.empty((rows, n), dtype=torch.float32, device=h.device) for _ in range(3)]
            arrs = [_lib.ptr_array(v) for v in (
                [c[0].data_ptr() for c in codes], [c[1].data_ptr() for c in codes],
                [aq.data_ptr(), ak.data_ptr(), av.data_ptr()],
                [_lib.ptr(bq), _lib.ptr(bk), _lib.ptr(bv)], [y.data_ptr() for y in outs])]
            ad = [ctypes.addressof(x) for x in arrs]
            _lib.check(lib.ob_bitlinear_fwd_passes_group(
                3, h.data_ptr(), P, m, k, ad[0], ad[1], pb.data_ptr(), ad[2], codes[0].fwd_raw,
                ad[3], n, ad[4], stream), "ob_bitlinear_fwd_passes_group")
        for w, a, b, c in (((wq, aq, bq, codes[0]), (wk, ak, bk, codes[1]), (wv, av, bv, codes[2]))
                           if not outs else ()):
            n = w.shape[0]
            y = torch.empty((rows, n), dtype=torch.float32, device=h.device)
            st = (lib.ob_bitlinear_fwd_passes(h.data_ptr(), P, m, k, c[0].data_ptr(),
                                              c[1].data_ptr(), pb.data_ptr(), a.data_ptr(),
                                              c.fwd_raw, _lib.ptr(b), n, y.data_ptr(), stream)
                  if pb is not None else
                  lib.ob_bitlinear_fwd(h.data_ptr(), m, k, c[0].data_ptr(), a.data_ptr(),
                                       c.fwd_raw, _lib.ptr(b), n, y.data_ptr(), stream))
            _lib.check(st, "ob_bitlinear_fwd")
            outs.append(y)
        ctx.meta = meta
        ctx.has_bias = (bq is not None, bk is not None, bv is not None)
        ctx.biases = (bq, bk, bv)
        deferred.note(wq, aq, bq, wk, ak, bk, wv, av, bv)
        ctx.save_for_backward(h, wq, aq, wk, ak, wv, av)
        return tuple(outs)

    @staticmethod
    def backward(ctx, gq, gk, gv):
        h, wq, aq, wk, ak, wv, av = ctx.saved_tensors
        P, pb, bits, codes = ctx.meta
        rows, k = h.shape
        m = rows // P
        lib = _lib.load()
        stream = _lib.stream_of(h)
        layers = [(g.contiguous(), w, a, c, hb) for g, w, a, c, hb in
                  zip((gq, gk, gv), (wq, wk, wv), (aq, ak, av), codes, ctx.has_bias)
                  if g is not None]
        gh = None
        if (ctx.needs_input_grad[0] and _DX_SUM and pb is not None and len(layers) == 3
                and len({c.dx_raw for c in codes}) == 1 and not codes[0].dense):
            # the three input gradients summed in ONE launch (ob_bitlinear_bwd_dx_passes_sum)
            n = wq.shape[0]
            out = torch.empty((rows, k), dtype=torch.float32, device=h.device)
            arrs = [_lib.ptr_array(v) for v in (
                [g.data_ptr() for g, _, _, _, _ in layers], [c[2].data_ptr() for c in codes],
                [c[3].data_ptr() for c in codes], [a.data_ptr() for _, _, a, _, _ in layers])]
            ad = [ctypes.addressof(x) for x in arrs]
            st = lib.ob_bitlinear_bwd_dx_passes_sum(3, ad[0], P, m, n, ad[1], ad[2], pb.data_ptr(),
                                                    ad[3], codes[0].dx_raw, k, out.data_ptr(),
                                                    stream)
            if st != _lib.OB_ERR_SHAPE:  # (shape not taken: the per-layer launches below)
                _lib.check(st, "ob_bitlinear_bwd_dx_passes_sum")
                gh = out
        if ctx.needs_input_grad[0] and gh is None:
            for g, w, a, c, _ in layers:
                n = w.shape[0]
                if gh is None:
                    gh = _dx(lib, g, P, m, n, c, pb, a, k, stream)
                    continue
                # gh += a * g . Q  (the dX GEMM with C = R = gh: each element read, then written,
                # by one lane)
                _lib.check(lib.ob_bitlinear_fwd_residual(
                    g.data_ptr(), P, m, n, c[2].data_ptr(), c[3].data_ptr(), _lib.ptr(pb),
                    a.data_ptr(), c.dx_raw, None, k, gh.data_ptr(), 1.0, 0.0, None, 0, None, 0,
                    gh.data_ptr(), stream), "ob_bitlinear_fwd_residual (dX accumulate)")
        grads = {}
        if pb is not None and not codes[0].dense:  # the grouped launch at the end of the backward
            for g, w, a, c, hb in layers:
                b = ctx.biases[[id(t) for t in (wq, wk, wv)].index(id(w))]
                o = (deferred.grad_buf(w), deferred.grad_buf(a, (), h.device),
                     deferred.grad_buf(b, (w.shape[0],), h.device) if hb else None)
                if deferred.dwg_take(g, h, P, m, w.shape[0], k, o[0], o[2], stream, w, b, alpha=a,
                                     ga=o[1], pass_bits=pb):
                    grads[id(w)] = o
        if _DW_GROUP and not grads and pb is not None and len(layers) == 3 and not codes[0].dense and \
                len({w.shape for _, w, _, _, _ in layers}) == 1:
            # the three dW GEMMs share X = h: their finishes in one launch
            n = layers[0][1].shape[0]
            wsb = lib.ob_bitlinear_bwd_dw_passes_group_workspace(3, P, m, n, k)
            if wsb:
                outs = [(torch.empty_like(w), torch.empty((), dtype=torch.float32, device=h.device),
                         torch.empty((n,), dtype=torch.float32, device=h.device) if hb else None)
                        for _, w, _, _, hb in layers]
                ws = torch.empty((wsb,), dtype=torch.uint8, device=h.device)
                arrs = [_lib.ptr_array(v) for v in (
                    [g.data_ptr() for g, _, _, _, _ in layers],
                    [w.data_ptr() for _, w, _, _, _ in layers],
                    [a.data_ptr() for _, _, a, _, _ in layers],
                    [o[0].data_ptr() for o in outs], [o[1].data_ptr() for o in outs],
                    [_lib.ptr(o[2]) for o in outs])]
                ad = [ctypes.addressof(x) for x in arrs]
                slot = (deferred.dw_slot(h.device, stream, 3)
                        if deferred.can_defer(wq, aq, wk, ak, wv, av, *ctx.biases) else None)
                if slot is not None:
                    nb = ctypes.c_int64(0)
                    _lib.check(lib.ob_bitlinear_bwd_dw_passes_group_defer(
                        3, ad[0], h.data_ptr(), P, m, n, k, ad[1], ad[2], 1, pb.data_ptr(), ad[3],
                        ad[4], ad[5], ws.data_ptr(), wsb, slot[0], slot[1], slot[2],
                        ctypes.addressof(nb), stream), "ob_bitlinear_bwd_dw_passes_group_defer")
                    deferred.dw_done(3, nb.value)
                    deferred.keep(ws)
                else:
                    _lib.check(lib.ob_bitlinear_bwd_dw_passes_group(
                        3, ad[0], h.data_ptr(), P, m, n, k, ad[1], ad[2], 1, pb.data_ptr(), ad[3],
                        ad[4], ad[5], ws.data_ptr(), wsb, stream), "ob_bitlinear_bwd_dw_passes_group")
                for (_, w, _, _, _), o in zip(layers, outs):
                    grads[id(w)] = o
        for i, (g, w, a, c, hb) in zip(range(3), layers):
            if id(w) not in grads:
                b = ctx.biases[[id(t) for t in (wq, wk, wv)].index(id(w))]
                grads[id(w)] = _dw(lib, g, h, P, m, w.shape[0], k, w, a, hb, pb, bits, stream, b,
                                   c.dense)
        out = [gh]
        for w in (wq, wk, wv):
            out.extend(grads.get(id(w), (None, None, None)))
        return (*out, None)


def qkv_projections(h: torch.Tensor, q_proj: QuantizedLinear, k_proj: QuantizedLinear,
                    v_proj: QuantizedLinear, bitwidth):
    """(q_proj(h), k_proj(h), v_proj(h)) as one autograd node (_QKVFn)."""
    P, pb, bits = _bits_args(bitwidth)
    h2 = _flat(h, q_proj.in_features)
    if h2.shape[0] % P:
        raise ValueError(f"{h2.shape[0]} rows do not split into {P} passes")
    meta = (P, pb, bits, tuple(_codes(l, P, bits) for l in (q_proj, k_proj, v_proj)))
    q, k, v = _QKVFn.apply(h2, q_proj.weight, q_proj.alpha, q_proj.bias, k_proj.weight,
                           k_proj.alpha, k_proj.bias, v_proj.weight, v_proj.alpha, v_proj.bias,
                           meta)
    lead = h.shape[:-1]
    return (q.view(*lead, -1), k.view(*lead, -1), v.view(*lead, -1))


def _flat(t: torch.Tensor, width: int) -> torch.Tensor:
    t2 = t.reshape(-1, width)
    return t2 if t2.is_contiguous() else t2.contiguous()


def ffn_residual(h: torch.Tensor, x: torch.Tensor, lin1: QuantizedLinear, lin2: QuantizedLinear,
                 bitwidth, p_drop: float, ln_next=None) -> torch.Tensor:
    """x + 0.5 * dropout(lin2(dropout(swish(lin1(h))))) (conformer.py:36-45); h = LN(x).

    ln_next: [(weight, bias, eps)] of the LayerNorm that normalises the output next (and,
    second entry, the LayerNorm of that one's output -- a block's final LN and the next
    block's first): formed in lin2's epilogue and picked up by those LNs' layer_norm /
    layer_norm_fork / layer_norm_pair calls (bit-identical to their own launches). Training
    only (grad enabled): inference consumers may take the int8 LN instead."""
    P, pb, bits = _bits_args(bitwidth)
    h2, x2 = _flat(h, lin1.in_features), _flat(x, lin2.out_features)
    if h2.shape[0] % P:
        raise ValueError(f"{h2.shape[0]} rows do not split into {P} passes")
    rng, off1 = _rng(h.device) if p_drop > 0 else (None, 0)
    off2 = _rng(h.device)[1] if p_drop > 0 else 0
    spec = GradScale(0.5, p_drop, rng, off2)
    meta = (P, pb, bits, _codes(lin1, P, bits), _codes(lin2, P, bits), float(p_drop), rng,
            off1, off2, spec)
    box = []
    lnreq = (([(w, b, float(e)) for w, b, e in ln_next], box)
             if ln_next and _LN_EPI and torch.is_grad_enabled() and 1 <= len(ln_next) <= 2
             else None)
    out = _FFNFn.apply(h2, x2, lin1.weight, lin1.alpha, lin1.bias, lin2.weight, lin2.alpha,
                       lin2.bias, meta, lnreq)
    out = attach_grad_scale(out.view(x.shape), spec)
    if box:
        out._ob_ln_pre = box[0]
        if len(box) > 1:
            out._ob_ln_pre2 = box[1]
    return out


def linear_residual(inp: torch.Tensor, x: torch.Tensor, lin: QuantizedLinear, bitwidth,
                    p_drop: float, rscale: float = 1.0, lens: Optional[torch.Tensor] = None,
                    frames: int = 0) -> torch.Tensor:
    """x + rscale * pad_zero(dropout(lin(inp))) (conformer.py:131-138); ``lens`` int32 [B]
    valid frames per utterance of ``frames`` rows each (None: no padding)."""
    P, pb, bits = _bits_args(bitwidth)
    i2, x2 = _flat(inp, lin.in_features), _flat(x, lin.out_features)
    if i2.shape[0] % P:
        raise ValueError(f"{i2.shape[0]} rows do not split into {P} passes")
    rng, off = _rng(inp.device) if p_drop > 0 else (None, 0)
    if lens is not None:
        lens = lens.to(torch.int32).contiguous()
    spec = GradScale(rscale, p_drop, rng, off, lens, frames)
    meta = (P, pb, bits, _codes(lin, P, bits), float(rscale), float(p_drop), rng, off, lens,
            int(frames), spec)
    out = _LinearResidualFn.apply(i2, x2, lin.weight, lin.alpha, lin.bias, meta)
    return attach_grad_scale(out.view(x.shape), spec)


# ----------------------------------------------------------------------------------------
# int8-activation inference (act_quant="absmax_int8", no autograd, dropout off): the same
# call sites on the int8 matrix cores (csrc/tgemm_i8.hip) with the elementwise tails in the
# GEMM epilogue, and each activation's per-tensor absmax taken from the kernel that
# produced it (the LN kernel, lin1's swish epilogue) instead of a separate pass.

def i8_fused_supported(x: torch.Tensor, *layers: QuantizedLinear, bitwidth=None,
                       p_drop: float = 0.0) -> bool:
    if os.environ.get("OB_FUSED", "1") == "0" or p_drop > 0.0 or torch.is_grad_enabled():
        return False
    if isinstance(bitwidth, PassBits) or bitwidth not in (1, 2):
        return False
    for m in layers:
        if m._packed is not None:
            m._check_packed_use(bitwidth)
    lib = _lib.load()
    return (x.is_cuda and x.dtype == torch.float32
            and all(m.act_quant == "absmax_int8" and m.quant_off is None
                    and m.out_features % 4 == 0 and m.in_features % 16 == 0
                    and m.in_features <= 576 for m in layers)
            and lib is not None)


def _i8_epi(a2: torch.Tensor, amax: torch.Tensor, lin: QuantizedLinear, bits: int, mode: int,
            R: Optional[torch.Tensor] = None, rscale: float = 1.0,
            lens: Optional[torch.Tensor] = None, frames: int = 0):
    rows, k = a2.shape
    n = lin.out_features
    codes, _ = lin._codes(bits)
    y = torch.empty((rows, n), dtype=torch.float32, device=a2.device)
    amax_out = torch.empty((1,), dtype=torch.float32, device=a2.device) if mode == 1 else None
    lib = _lib.load()
    _lib.check(lib.ob_bitlinear_fwd_i8_epi(
        a2.data_ptr(), 1, rows, k, codes.data_ptr(), None, None, lin.alpha.data_ptr(), 1,
        amax.data_ptr(), _lib.ptr(lin.bias), n, mode, _lib.ptr(R), float(rscale), _lib.ptr(lens),
        int(frames), _lib.ptr(amax_out), y.data_ptr(), _lib.stream_of(a2)),
        "ob_bitlinear_fwd_i8_epi")
    return y, amax_out


def _amax_of(t: torch.Tensor) -> torch.Tensor:
    from .quant import act_absmax

    amax = getattr(t, "_ob_amax", None)
    return amax if amax is not None and amax.numel() == 1 else act_absmax(t.contiguous(), 1)


def _i8q(aq: torch.Tensor, amax: torch.Tensor, lin: QuantizedLinear, bits: int, mode: int,
         R: Optional[torch.Tensor] = None, rscale: float = 1.0):
    """ob_bitlinear_fwd_i8q: lin on an int8 operand aq [rows, K] (quantised at amax).
    mode 0 / 2: fp32 output (plain / + rscale * y onto R); mode 3: (int8 silu(y), its amax)."""
    rows, k = aq.shape
    n = lin.out_features
    codes, _ = lin._codes(bits)
    dt = torch.int8 if mode == 3 else torch.float32
    y = torch.empty((rows, n), dtype=dt, device=aq.device)
    amax_out = torch.empty((1,), dtype=torch.float32, device=aq.device) if mode == 3 else None
    lib = _lib.load()
    _lib.check(lib.ob_bitlinear_fwd_i8q(
        aq.data_ptr(), 1, rows, k, codes.data_ptr(), None, None, lin.alpha.data_ptr(), 1,
        amax.data_ptr(), _lib.ptr(lin.bias), n, mode, _lib.ptr(R), float(rscale), None, 0,
        _lib.ptr(amax_out), y.data_ptr(), _lib.stream_of(aq)), "ob_bitlinear_fwd_i8q")
    return y, amax_out


def i8_linear(h: Int8Act, lin: QuantizedLinear, bitwidth) -> torch.Tensor:
    """lin(h) (fp32 out) for an activation held as its int8 image (q/k/v on LN(x))."""
    y, _ = _i8q(h.q, h.amax, lin, int(bitwidth), 0)
    return y.view(*h.shape[:-1], lin.out_features)


@torch.no_grad()
def ffn_residual_i8(h, x: torch.Tensor, lin1: QuantizedLinear,
                    lin2: QuantizedLinear, bitwidth) -> torch.Tensor:
    """x + 0.5 * lin2(swish(lin1(h))) (conformer.py:36-45, eval) with int8 activations; h =
    LN(x) as an Int8Act (layer_norm_i8: every activation is int8 in HBM -- lin1 writes the
    int8 image of swish(lin1(h)) at its own absmax, lin2 reads it), or as fp32, ideally
    carrying its absmax (LayerNorm.emit_amax; the operands are quantised in registers)."""
    bits = int(bitwidth)
    x2 = _flat(x, lin2.out_features).contiguous()
    if isinstance(h, Int8Act):
        a, amax_a = _i8q(h.q, h.amax, lin1, bits, 3)
        out, _ = _i8q(a, amax_a, lin2, bits, 2, R=x2, rscale=0.5)
        return out.view(x.shape)
    amax_h = _amax_of(h)
    h2 = _flat(h, lin1.in_features).contiguous()
    a, amax_a = _i8_epi(h2, amax_h, lin1, bits, 1)
    out, _ = _i8_epi(a, amax_a, lin2, bits, 2, R=x2, rscale=0.5)
    return out.view(x.shape)


@torch.no_grad()
def linear_residual_i8(inp: torch.Tensor, x: torch.Tensor, lin: QuantizedLinear, bitwidth,
                       rscale: float = 1.0, lens: Optional[torch.Tensor] = None,
                       frames: int = 0) -> torch.Tensor:
    """x + rscale * pad_zero(lin(inp)) (conformer.py:131-138, eval) with int8 activations."""
    bits = int(bitwidth)
    i2 = _flat(inp, lin.in_features).contiguous()
    x2 = _flat(x, lin.out_features).contiguous()
    if lens is not None:
        lens = lens.to(torch.int32).contiguous()
    out, _ = _i8_epi(i2, _amax_of(i2), lin, bits, 2, R=x2, rscale=rscale, lens=lens,
                     frames=frames)
    return out.view(x.shape)
