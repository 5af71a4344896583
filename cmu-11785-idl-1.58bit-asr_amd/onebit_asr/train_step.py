"""The measured unit of work: one training step of the reference (onebit_asr/train.py:76-120).

Per batch the reference runs three encoder+decoder passes -- a 2-bit teacher, a 1-bit
student and a stochastic-precision (SP) mix -- and combines their attention-CE, CTC and
KL terms into one loss (train.py:82-111), then backward, grad-norm clip 5.0, AdamW and the
warmup-cosine schedule (train.py:114-120, 259-264).

``OneBitStep`` wraps the three passes in ONE module forward, so that a
``DistributedDataParallel`` wrapper sees one forward per backward (the reference calls
``model`` three times plus ``decode_logits`` outside ``forward``, which DDP's reducer would
not pair with a single backward). With DDP every rank draws the same SP mask from a
generator seeded identically on all ranks (train.py:56-59 draws from the global RNG).
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import deferred
from .losses import att_ce_loss, ctc_loss_from_logits, kl_logits, make_att_targets
from .seqloss import att_kl_losses, att_kl_supported


__all__ = ["OneBitStep", "WarmupCosine", "sample_sp_mask", "train_step", "SPECIAL_IDS",
           "make_optimizer"]

# dataloader_stub.py:199-207: pad 0, bos 1, eos 2, blank 3; SPM ids offset by +4.
SPECIAL_IDS = {"pad_id": 0, "bos_id": 1, "eos_id": 2, "blank_id": 3}


def sample_sp_mask(n_layers: int, low_p: float = 0.2, high_p: float = 0.9,
                   generator: Optional[torch.Generator] = None) -> List[int]:
    """train.py:56-59: block i runs 1-bit with probability logspace(0.2..0.9)[i]."""
    probs = torch.logspace(math.log10(low_p), math.log10(high_p), steps=n_layers)
    draws = torch.rand((n_layers,), generator=generator)
    return [int(d < p) for d, p in zip(draws.tolist(), probs.tolist())]


class WarmupCosine:
    """train.py:32-53. lr is rewritten after each optimizer step (so the first step runs at
    the optimizer's initial lr -- a reference quirk kept as is)."""

    def __init__(self, optimizer, warmup_steps: int, total_steps: int, min_lr_ratio: float = 0.1):
        self.optimizer = optimizer
        self.warmup_steps = warmup_steps
        self.total_steps = total_steps
        self.min_lr_ratio = min_lr_ratio
        self.step_num = 0
        for group in optimizer.param_groups:
            if "initial_lr" not in group:
                group["initial_lr"] = float(group.get("lr", 1e-3))

    def scale(self, step: int) -> float:
        if step < self.warmup_steps:
            return step / max(1, self.warmup_steps)
        span = max(1, self.total_steps - self.warmup_steps)
        progress = min(max((step - self.warmup_steps) / span, 0.0), 1.0)
        return self.min_lr_ratio + 0.5 * (1 - self.min_lr_ratio) * (1 + math.cos(math.pi * progress))

    def reset(self):
        """Back to step 0 at the initial learning rate (before any optimizer step)."""
        self.step_num = 0
        for group in self.optimizer.param_groups:
            if isinstance(group["lr"], torch.Tensor):
                group["lr"].fill_(group["initial_lr"])
            else:
                group["lr"] = group["initial_lr"]

    def step(self):
        self.step_num += 1
        s = self.scale(self.step_num)
        for group in self.optimizer.param_groups:
            if isinstance(group["lr"], torch.Tensor):  # capturable AdamW: lr read on device
                group["lr"].fill_(group["initial_lr"] * s)
            else:
                group["lr"] = group["initial_lr"] * s


def make_optimizer(params, lr: float = 5e-4) -> torch.optim.Optimizer:
    """train.py:259: AdamW(lr, betas=(0.9, 0.98), weight_decay=1e-2) over all parameters
    (weight decay therefore also applies to every alpha)."""
    return torch.optim.AdamW(params, lr=lr, betas=(0.9, 0.98), weight_decay=1e-2)


class OneBitStep(nn.Module):
    """train.py:82-111 as one forward returning the combined loss.

    ``stacked=True`` (the default on a ROCm device) runs the three passes as ONE forward
    over the batch repeated three times: every full-precision op runs once on 3B
    utterances instead of three times on B, each BitLinear runs its three passes in one
    launch per kernel (``PassBits``: pass p at its own bitwidth, read on device), BatchNorm
    keeps per-pass statistics, and the losses are formed per pass exactly as in the
    reference. Each pass computes what the reference computes; only the order in which
    the passes' gradient contributions are summed differs. ``stacked=False`` is the
    reference's literal three forwards. ``branch_streams`` (stacked, CUDA; off by default):
    the decoder branch runs on a side stream beside the CTC branch (``_forward_stacked``);
    measured same-box in the graphed step it is 0.2 ms SLOWER (24.53 vs 24.33 ms/step,
    profiles/r5/branch_ab/), so the step keeps one stream."""

    def __init__(self, model: nn.Module, n_layers: int, special: Optional[Dict[str, int]] = None,
                 gamma_ctc: float = 0.2, lambda1: float = 0.5, lambda2: float = 1.0,
                 label_smoothing: float = 0.1, stacked: Optional[bool] = None,
                 branch_streams: bool = False):
        super().__init__()
        self.model = model
        self.n_layers = n_layers
        self.special = dict(SPECIAL_IDS if special is None else special)
        self.gamma_ctc = gamma_ctc
        self.lambda1 = lambda1
        self.lambda2 = lambda2
        self.label_smoothing = label_smoothing
        self.stacked = stacked
        self.branch_streams = branch_streams
        self._side = None
        self._bits = None
        self._packer = None

    def _use_stacked(self) -> bool:
        if self.stacked is not None:
            return self.stacked
        return next(self.model.parameters()).is_cuda

    def make_bits(self, device):
        """Device bit table for graph capture: StackedBits (stacked) or DeviceBits."""
        from .quant import DeviceBits, StackedBits

        if self._use_stacked():
            return StackedBits(self.n_layers, device)
        return DeviceBits(self.n_layers, device)

    def _pass(self, batch, t_inp, t_out, t_pad, precision, sp_mask=None):
        enc, mask, ctc = self.model(batch, precision=precision, sp_mask=sp_mask)
        logits = self.model.decode_logits(enc, mask, t_inp, t_pad)
        l_att = att_ce_loss(logits, t_out, self.special["pad_id"], label_smoothing=self.label_smoothing)
        l_ctc = ctc_loss_from_logits(ctc, mask.sum(dim=1).long(), batch["tokens"],
                                     batch["token_lens"], self.special["blank_id"])
        l_int = (1 - self.gamma_ctc) * l_att + self.gamma_ctc * l_ctc
        return logits, l_int, l_ctc

    def forward(self, batch: Dict[str, torch.Tensor], sp_mask):
        """``sp_mask``: the reference's per-block list, or a ``DeviceBits`` / ``StackedBits``
        (graph mode)."""
        from .quant import StackedBits

        if isinstance(sp_mask, StackedBits):
            return self._forward_stacked(batch, sp_mask)
        if self._use_stacked() and not hasattr(sp_mask, "tensor"):
            dev = batch["feats"].device
            if self._bits is None or self._bits.tensor.device != dev:
                self._bits = StackedBits(self.n_layers, dev)
            self._bits.set(sp_mask)
            return self._forward_stacked(batch, self._bits)
        sp = self.special
        t_inp, t_out, t_pad = make_att_targets(batch["tokens"], sp["bos_id"], sp["eos_id"], sp["pad_id"])
        logits2, lint2, lctc2 = self._pass(batch, t_inp, t_out, t_pad, 2)          # teacher
        logits1, lint1, lctc1 = self._pass(batch, t_inp, t_out, t_pad, 1)          # student
        teacher = logits2.detach()
        lkl1 = kl_logits(logits1, teacher, t_pad)
        logits_s, lint_s, lctc_s = self._pass(batch, t_inp, t_out, t_pad, 2, sp_mask)  # SP
        lkl_s = kl_logits(logits_s, teacher, t_pad)
        loss = lint2 + self.lambda1 * (lint1 + lint_s) + self.lambda2 * (lkl1 + lkl_s)
        parts = torch.stack([lint2, lint1, lint_s, lkl1, lkl_s, lctc2, lctc1, lctc_s]).detach()
        return loss, parts


    def _att_kl_torch(self, logits, t_out, t_pad, P):
        """The decoder losses as torch expressions (the path when csrc/seqloss.hip does not
        apply: CPU, label smoothing 0, V % 4 != 0)."""
        pad_id = self.special["pad_id"]
        vocab, u1 = logits.size(-1), logits.size(1)
        bsz = logits.size(0) // P
        logp = F.log_softmax(logits, dim=-1).view(P, bsz, u1, vocab)
        if self.label_smoothing > 0:
            off = self.label_smoothing / (vocab - 1)
            tgt = t_out.unsqueeze(0).expand(P, bsz, u1).unsqueeze(-1)
            tgt_logp = logp.gather(-1, tgt).squeeze(-1)
            per_pos = -(off * logp.sum(dim=-1) + (1.0 - self.label_smoothing - off) * tgt_logp)
            l_mean = per_pos.reshape(P, -1).mean(dim=1)
            m = (t_out != pad_id).float()
            l_att = (l_mean[:, None] * m.reshape(1, -1)).sum(dim=1) / m.sum().clamp_min(1.0)
        else:
            l_att = torch.stack([F.nll_loss(logp[p].transpose(1, 2), t_out, ignore_index=pad_id)
                                 for p in range(P)])
        with torch.no_grad():  # softmax of the detached teacher logits (train.py:101)
            p_t = F.softmax(logits[:bsz].detach(), dim=-1)
        kl = F.kl_div(logp[1:], p_t.unsqueeze(0).expand(P - 1, -1, -1, -1),
                      reduction="none").sum(dim=-1)
        keep = (~t_pad).float()
        l_kl = (kl * keep.unsqueeze(0)).sum(dim=(1, 2)) / keep.sum().clamp_min(1.0)
        return l_att, l_kl

    def _decoder_losses(self, enc, mask, tgt_inp, tgt_pad, t_out, t_pad, P):
        logits = self.model.decode_logits(enc, mask, tgt_inp, tgt_pad)
        # attention CE per pass (losses.py:22-35, label smoothing, scalar-mean quirk) and
        # KL(teacher || student) for the student and SP passes (losses.py:50-59)
        if att_kl_supported(logits, self.label_smoothing):
            # csrc/seqloss.hip: both losses, one row pass per direction
            return att_kl_losses(logits, t_out, t_pad, P, self.special["pad_id"],
                                 self.label_smoothing)
        return self._att_kl_torch(logits, t_out, t_pad, P)

    def _side_stream(self, enc):
        """The decoder branch's stream (one per device), or None (branches off -- tests compare
        both -- or a CPU tensor)."""
        if not (self.branch_streams and enc.is_cuda):
            return None
        if self._side is None or self._side.device != enc.device:
            self._side = torch.cuda.Stream(enc.device)
        return self._side

    def _forward_stacked(self, batch, bits):
        from .ctc import ctc_loss_logits_groups

        from .fused import advance_step
        from .quant import PackGroup

        if self._packer is None:
            self._packer = PackGroup(self.model, bits=(2, 1))
        self._packer.run()  # codes of every BitLinear, both bitwidths, in one launch
        advance_step(batch["feats"].device)  # fresh dropout masks for the fused call sites
        sp = self.special
        P = bits.passes  # 0: teacher (2-bit), 1: student (1-bit), 2: SP
        bsz = batch["feats"].size(0)
        t_inp, t_out, t_pad = make_att_targets(batch["tokens"], sp["bos_id"], sp["eos_id"], sp["pad_id"])
        # the encoder repeats the (pass-independent) subsampling output P times itself
        enc, mask = self.model.encoder(batch["feats"], batch["feat_lens"], 2, bits)
        tgt_inp, tgt_pad = t_inp.repeat(P, 1), t_pad.repeat(P, 1)
        side = self._side_stream(enc)
        if side is not None:
            # Two independent branches from here to the loss: the decoder + attention-CE / KL
            # (decoder.py call sites, losses.py:22-35,50-59) on a side stream, the CTC head +
            # CTC (losses.py:41-47) on this one. Both are chains of small, latency-bound
            # launches; side by side they overlap (also in the captured graph, where the fork
            # and join are graph edges). Autograd runs each node's backward on its forward's
            # stream, so the two backward branches overlap too; deferred.py joins the streams
            # before its end-of-backward finishes.
            main = torch.cuda.current_stream(enc.device)
            side.wait_stream(main)
            # this stream's tensors read on the side stream (also by the decoder's backward):
            # their blocks must not return to this stream's pool before the side stream has
            # read them (the engine records the gradients that cross back itself)
            for t in (enc, mask, tgt_inp, tgt_pad, t_out, t_pad):
                t.record_stream(side)
            with torch.cuda.stream(side):
                l_att, l_kl = self._decoder_losses(enc, mask, tgt_inp, tgt_pad, t_out, t_pad, P)
        else:
            l_att, l_kl = self._decoder_losses(enc, mask, tgt_inp, tgt_pad, t_out, t_pad, P)
        ctc = self.model.ctc_logits(enc)
        # CTC per pass (losses.py:41-47: log_softmax + CTC), straight from the head's logits
        in_lens = mask.sum(dim=1).long()
        # the P passes' CTC losses in one launch per direction (each pass its own mean)
        l_ctc = ctc_loss_logits_groups(ctc, batch["tokens"].repeat(P, 1), in_lens,
                                       batch["token_lens"].repeat(P), sp["blank_id"], P)
        if side is not None:  # join: the loss below reads the decoder branch's results
            main.wait_stream(side)
            l_att.record_stream(main)
            l_kl.record_stream(main)
        if l_att.is_cuda and P == 3:  # one HIP launch each way (csrc/seqloss.hip)
            return _LossCombine.apply(l_att, l_ctc, l_kl, self.gamma_ctc, self.lambda1,
                                      self.lambda2)
        l_int = (1 - self.gamma_ctc) * l_att + self.gamma_ctc * l_ctc
        loss = l_int[0] + self.lambda1 * (l_int[1] + l_int[2]) + self.lambda2 * (l_kl[0] + l_kl[1])
        parts = torch.stack([l_int[0], l_int[1], l_int[2], l_kl[0], l_kl[1],
                             l_ctc[0], l_ctc[1], l_ctc[2]]).detach()
        return loss, parts


class _LossCombine(torch.autograd.Function):
    """train.py:95-111's combination of the three passes' losses (the stacked step's form of
    the expression in ``_forward_stacked``'s fallback, same rounding sequence) and the eight
    logged parts in ONE launch, its backward in one more (ob_loss_combine_*): the torch
    expression is ~20 scalar kernels forward and ~25 backward (index backwards: fills,
    copies, adds)."""

    @staticmethod
    def forward(ctx, l_att, l_ctc, l_kl, gamma, lam1, lam2):
        from . import _lib

        l_att, l_ctc, l_kl = (t.contiguous() for t in (l_att, l_ctc, l_kl))
        loss = torch.empty((), dtype=torch.float32, device=l_att.device)
        parts = torch.empty((8,), dtype=torch.float32, device=l_att.device)
        _lib.check(_lib.load().ob_loss_combine_fwd(
            l_att.data_ptr(), l_ctc.data_ptr(), l_kl.data_ptr(), gamma, lam1, lam2,
            loss.data_ptr(), parts.data_ptr(), _lib.stream_of(l_att)), "ob_loss_combine_fwd")
        ctx.meta = (gamma, lam1, lam2)
        ctx.mark_non_differentiable(parts)
        return loss, parts

    @staticmethod
    def backward(ctx, g_loss, _g_parts):
        from . import _lib

        gamma, lam1, lam2 = ctx.meta
        g_loss = g_loss.contiguous()
        d_att = torch.empty((3,), dtype=torch.float32, device=g_loss.device)
        d_ctc = torch.empty((3,), dtype=torch.float32, device=g_loss.device)
        d_kl = torch.empty((2,), dtype=torch.float32, device=g_loss.device)
        _lib.check(_lib.load().ob_loss_combine_bwd(
            g_loss.data_ptr(), gamma, lam1, lam2, d_att.data_ptr(), d_ctc.data_ptr(),
            d_kl.data_ptr(), _lib.stream_of(g_loss)), "ob_loss_combine_bwd")
        return d_att, d_ctc, d_kl, None, None, None


PART_NAMES = ["Lint2", "Lint1", "Lint_s", "Lkl1", "Lkl_s", "Lctc2", "Lctc1", "Lctc_s"]


def train_step(step_module: nn.Module, optimizer: torch.optim.Optimizer,
               sched: Optional[WarmupCosine], batch: Dict[str, torch.Tensor],
               sp_mask: List[int], max_norm: float = 5.0):
    """train.py:114-120: zero_grad, backward, clip_grad_norm_(5.0), step, sched.step().
    Returns the (device) loss and loss parts; nothing here synchronises with the host."""
    optimizer.zero_grad(set_to_none=True)
    # gradient finishes batched at the end of the backward -- except under DDP, whose reducer
    # hooks copy each gradient into its bucket (and start the all-reduce) as it lands
    ddp = isinstance(step_module, torch.nn.parallel.DistributedDataParallel)
    with deferred.scope(enabled=not ddp):
        loss, parts = step_module(batch, sp_mask)
        loss.backward()
    params = [p for p in step_module.parameters() if p.grad is not None]
    torch.nn.utils.clip_grad_norm_(params, max_norm=max_norm)
    optimizer.step()
    if sched is not None:
        sched.step()
    return loss.detach(), parts
