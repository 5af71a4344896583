"""CTC loss on the HIP kernel (reference losses.py:41-47 semantics), with device-side lengths.

torch's CUDA CTC copies its length tensors to the host (a device->host sync per call), which
also makes the step uncapturable in a HIP graph. ``ctc_loss_mean`` computes the same loss
(blank, zero_infinity=True, reduction 'mean': per-sample nll / max(target_len, 1), then the
batch mean) and torch's gradient, reading lengths on device. Inputs: log-probs [B, T, V]
(batch-major), targets [B, S] int64 (padded), lengths int64 [B] on the same device.
"""
from __future__ import annotations

import torch

from . import _lib

__all__ = ["ctc_loss_mean", "ctc_loss_mean_groups", "ctc_loss_logits_groups"]


class _CTCFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, log_probs, targets, input_lengths, target_lengths, blank):
        b, t, v = log_probs.shape
        s = targets.shape[1]
        lp = log_probs.contiguous()
        tg = targets.contiguous().to(torch.int64)
        il = input_lengths.contiguous().to(torch.int64)
        tl = target_lengths.contiguous().to(torch.int64)
        lib = _lib.load()
        wsb = lib.ob_ctc_loss_workspace(b, t, s)
        ws = torch.empty((wsb,), dtype=torch.uint8, device=lp.device)
        loss = torch.empty((), dtype=torch.float32, device=lp.device)
        _lib.check(lib.ob_ctc_loss_fwd(lp.data_ptr(), tg.data_ptr(), il.data_ptr(), tl.data_ptr(),
                                       b, t, v, s, blank, loss.data_ptr(), ws.data_ptr(), wsb,
                                       _lib.stream_of(lp)), "ob_ctc_loss_fwd")
        ctx.save_for_backward(lp, tg, il, tl, ws)
        ctx.blank = blank
        return loss

    @staticmethod
    def backward(ctx, gout):
        lp, tg, il, tl, ws = ctx.saved_tensors
        b, t, v = lp.shape
        s = tg.shape[1]
        grad = torch.empty_like(lp)
        gout = gout.contiguous().to(torch.float32)
        lib = _lib.load()
        _lib.check(lib.ob_ctc_loss_bwd(lp.data_ptr(), tg.data_ptr(), il.data_ptr(), tl.data_ptr(),
                                       b, t, v, s, ctx.blank, gout.data_ptr(), grad.data_ptr(),
                                       ws.data_ptr(), ws.numel(), _lib.stream_of(lp)),
                   "ob_ctc_loss_bwd")
        return grad, None, None, None, None


def ctc_loss_mean(log_probs_btv, targets, input_lengths, target_lengths, blank: int):
    return _CTCFn.apply(log_probs_btv, targets, input_lengths, target_lengths, blank)


class _CTCGroupsFn(torch.autograd.Function):
    """G groups of B/G utterances in one launch per direction: losses [G]."""

    @staticmethod
    def forward(ctx, log_probs, targets, input_lengths, target_lengths, blank, groups):
        b, t, v = log_probs.shape
        s = targets.shape[1]
        lp = log_probs.contiguous()
        tg = targets.contiguous().to(torch.int64)
        il = input_lengths.contiguous().to(torch.int64)
        tl = target_lengths.contiguous().to(torch.int64)
        lib = _lib.load()
        wsb = lib.ob_ctc_loss_workspace(b, t, s)
        ws = torch.empty((wsb,), dtype=torch.uint8, device=lp.device)
        loss = torch.empty((groups,), dtype=torch.float32, device=lp.device)
        _lib.check(lib.ob_ctc_loss_fwd_groups(lp.data_ptr(), tg.data_ptr(), il.data_ptr(),
                                              tl.data_ptr(), groups, b, t, v, s, blank,
                                              loss.data_ptr(), ws.data_ptr(), wsb,
                                              _lib.stream_of(lp)), "ob_ctc_loss_fwd_groups")
        ctx.save_for_backward(lp, tg, il, tl, ws)
        ctx.meta = (blank, groups)
        return loss

    @staticmethod
    def backward(ctx, gout):
        lp, tg, il, tl, ws = ctx.saved_tensors
        blank, groups = ctx.meta
        b, t, v = lp.shape
        s = tg.shape[1]
        grad = torch.empty_like(lp)
        gout = gout.contiguous().to(torch.float32)
        lib = _lib.load()
        _lib.check(lib.ob_ctc_loss_bwd_groups(lp.data_ptr(), tg.data_ptr(), il.data_ptr(),
                                              tl.data_ptr(), groups, b, t, v, s, blank,
                                              gout.data_ptr(), grad.data_ptr(), ws.data_ptr(),
                                              ws.numel(), _lib.stream_of(lp)),
                   "ob_ctc_loss_bwd_groups")
        return grad, None, None, None, None, None


def ctc_loss_mean_groups(log_probs_btv, targets, input_lengths, target_lengths, blank: int,
                         groups: int):
    """ctc_loss_mean of each of ``groups`` consecutive equal slices of the batch, one launch:
    returns the [groups] losses (the stacked passes' CTC terms)."""
    return _CTCGroupsFn.apply(log_probs_btv, targets, input_lengths, target_lengths, blank, groups)


class _CTCLogitsGroupsFn(torch.autograd.Function):
    """log_softmax + CTC of each of G groups from the CTC head's logits [B, T, V]: the
    log-probabilities are gathered at blank and the labels only, the gradient is w.r.t. the
    logits (csrc/ctc.hip, ob_ctc_loss_logits_*): no [B*T, V] log_softmax / log-prob gradient
    tensors (478 MB each at Conformer-S)."""

    @staticmethod
    def forward(ctx, logits, targets, input_lengths, target_lengths, blank, groups):
        b, t, v = logits.shape
        s = targets.shape[1]
        x = logits.contiguous()
        tg = targets.contiguous().to(torch.int64)
        il = input_lengths.contiguous().to(torch.int64)
        tl = target_lengths.contiguous().to(torch.int64)
        lib = _lib.load()
        wsb = lib.ob_ctc_logits_workspace(b, t, s)
        ws = torch.empty((wsb,), dtype=torch.uint8, device=x.device)
        loss = torch.empty((groups,), dtype=torch.float32, device=x.device)
        _lib.check(lib.ob_ctc_loss_logits_fwd_groups(x.data_ptr(), tg.data_ptr(), il.data_ptr(),
                                                     tl.data_ptr(), groups, b, t, v, s, blank,
                                                     loss.data_ptr(), ws.data_ptr(), wsb,
                                                     _lib.stream_of(x)),
                   "ob_ctc_loss_logits_fwd_groups")
        ctx.save_for_backward(x, tg, il, tl, ws)
        ctx.meta = (blank, groups)
        return loss

    @staticmethod
    def backward(ctx, gout):
        x, tg, il, tl, ws = ctx.saved_tensors
        blank, groups = ctx.meta
        b, t, v = x.shape
        s = tg.shape[1]
        grad = torch.empty_like(x)
        gout = gout.contiguous().to(torch.float32)
        lib = _lib.load()
        _lib.check(lib.ob_ctc_loss_logits_bwd_groups(x.data_ptr(), tg.data_ptr(), il.data_ptr(),
                                                     tl.data_ptr(), groups, b, t, v, s, blank,
                                                     gout.data_ptr(), grad.data_ptr(),
                                                     ws.data_ptr(), ws.numel(),
                                                     _lib.stream_of(x)),
                   "ob_ctc_loss_logits_bwd_groups")
        return grad, None, None, None, None, None


def ctc_loss_logits_groups(logits_btv, targets, input_lengths, target_lengths, blank: int,
                           groups: int):
    """ctc_loss_mean_groups(log_softmax(logits_btv)) without the log_softmax tensor:
    the [groups] losses of ``groups`` consecutive equal batch slices."""
    return _CTCLogitsGroupsFn.apply(logits_btv, targets, input_lengths, target_lengths, blank,
                                    groups)
