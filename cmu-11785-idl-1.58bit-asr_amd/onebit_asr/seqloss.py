"""The stacked step's decoder losses in one HIP pass per direction (csrc/seqloss.hip).

Same losses as the torch expressions they replace: ``att_ce_loss`` with label smoothing
(reference onebit_asr/losses.py:22-35, including its scalar-mean quirk: the mean over ALL
positions times msum / max(msum, 1)) for every pass, and ``kl_logits`` (losses.py:50-59,
KL(stopgrad softmax(teacher) || softmax(student)) averaged over non-pad decoder inputs) for
passes 1..P-1 against pass 0, as train.py:82-111 combines them. torch runs ~20 kernels per
direction and materialises log_softmax / softmax tensors of the [P, B, U, V] logits; the
kernels read each row once (twice with its teacher row) and write only the gradient.
"""
from __future__ import annotations

import torch

from . import _lib

__all__ = ["att_kl_losses", "att_kl_supported"]


def att_kl_supported(logits: torch.Tensor, label_smoothing: float) -> bool:
    v = logits.size(-1)
    return (logits.is_cuda and logits.dtype == torch.float32 and 0.0 < label_smoothing < 1.0
            and v % 4 == 0 and 4 <= v <= 8192)


class _AttKLFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, tgt_out, tgt_pad, passes, pad_id, ls):
        pbu, v = logits.numel() // logits.size(-1), logits.size(-1)
        bu = tgt_out.numel()
        if pbu != passes * bu:
            raise ValueError(f"logits rows {pbu} != passes {passes} x positions {bu}")
        x = logits.contiguous()
        tg = tgt_out.contiguous().view(-1).to(torch.int64)
        pad = tgt_pad.contiguous().view(-1).to(torch.uint8)
        lib = _lib.load()
        wsb = lib.ob_att_kl_workspace(passes, bu)
        ws = torch.empty((wsb,), dtype=torch.uint8, device=x.device)
        out = torch.empty((2 * passes - 1,), dtype=torch.float32, device=x.device)
        l_att, l_kl = out[:passes], out[passes:]
        _lib.check(lib.ob_att_kl_loss_fwd(x.data_ptr(), tg.data_ptr(), pad.data_ptr(), passes, bu,
                                          v, pad_id, ls, l_att.data_ptr(),
                                          l_kl.data_ptr() if passes > 1 else 0, ws.data_ptr(),
                                          wsb, _lib.stream_of(x)),
                   "ob_att_kl_loss_fwd")
        ctx.save_for_backward(x, tg, pad, ws)
        ctx.meta = (passes, ls)
        return l_att, l_kl

    @staticmethod
    def backward(ctx, g_att, g_kl):
        x, tg, pad, ws = ctx.saved_tensors
        passes, ls = ctx.meta
        v = x.size(-1)
        g_att = (torch.zeros(passes, device=x.device) if g_att is None
                 else g_att.contiguous().to(torch.float32))
        g_kl = (torch.zeros(max(passes - 1, 1), device=x.device) if g_kl is None
                else g_kl.contiguous().to(torch.float32))
        grad = torch.empty_like(x)
        lib = _lib.load()
        _lib.check(lib.ob_att_kl_loss_bwd(x.data_ptr(), tg.data_ptr(), pad.data_ptr(), passes,
                                          tg.numel(), v, ls, g_att.data_ptr(), g_kl.data_ptr(),
                                          grad.data_ptr(), ws.data_ptr(), ws.numel(),
                                          _lib.stream_of(x)),
                   "ob_att_kl_loss_bwd")
        return grad, None, None, None, None, None


def att_kl_losses(logits: torch.Tensor, tgt_out: torch.Tensor, tgt_pad: torch.Tensor,
                  passes: int, pad_id: int, label_smoothing: float):
    """logits [P*B, U, V] (pass-major), tgt_out / tgt_pad [B, U] -> (l_att [P], l_kl [P-1])."""
    return _AttKLFn.apply(logits, tgt_out, tgt_pad, passes, pad_id, float(label_smoothing))
