"""Training objectives around the hot path (stock PyTorch-ROCm, reference onebit_asr/losses.py).

The reference's numerical quirks are kept because the step's loss value is a parity
observable:

* ``make_att_targets`` appends EOS after the padding, not after the last token
  (losses.py:11-19);
* ``att_ce_loss`` with label smoothing reduces to a scalar mean over ALL positions
  before its pad mask is applied, so the mask is a no-op (losses.py:22-35);
* ``kl_logits`` masks by ``tgt_inp == pad`` (losses.py:50-59);
* CTC: log_softmax over the CTC head, ``nn.CTCLoss(blank, zero_infinity=True)``, mean
  reduction (losses.py:41-47).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

__all__ = ["make_att_targets", "att_ce_loss", "ctc_loss_from_logits", "kl_logits"]


def make_att_targets(tokens: torch.Tensor, bos_id: int, eos_id: int, pad_id: int):
    """tokens [B,U] -> (tgt_inp = [BOS|tokens], tgt_out = [tokens|EOS], tgt_inp == pad)."""
    bsz = tokens.size(0)
    bos = tokens.new_full((bsz, 1), bos_id)
    eos = tokens.new_full((bsz, 1), eos_id)
    tgt_inp = torch.cat((bos, tokens), dim=1)
    tgt_out = torch.cat((tokens, eos), dim=1)
    return tgt_inp, tgt_out, tgt_inp == pad_id


def att_ce_loss(logits: torch.Tensor, targets: torch.Tensor, pad_id: int,
                label_smoothing: float = 0.0):
    if label_smoothing > 0:
        logp = F.log_softmax(logits, dim=-1)
        n_class = logits.size(-1)
        # sum_c -q_c log p_c with q = eps/(V-1) off-target, 1-eps on target (losses.py:26-31),
        # without materialising q: off-target mass over all classes, then the target fix-up.
        off = label_smoothing / (n_class - 1)
        tgt_logp = logp.gather(-1, targets.unsqueeze(-1)).squeeze(-1)
        per_pos = -(off * logp.sum(dim=-1) + (1.0 - label_smoothing - off) * tgt_logp)
        loss = per_pos.mean()
        mask = (targets != pad_id).float()
        return (loss * mask).sum() / mask.sum().clamp_min(1.0)
    return F.cross_entropy(logits.transpose(1, 2), targets, ignore_index=pad_id)


def ctc_loss_from_logits(ctc_logits: torch.Tensor, feat_lens: torch.Tensor,
                         tokens: torch.Tensor, token_lens: torch.Tensor, blank_id: int):
    """On a ROCm device: the HIP CTC straight from the logits (same loss and gradient as
    log_softmax + CTC, lengths read on device, no host sync, no log_softmax tensor);
    elsewhere torch's nn.CTCLoss on the [T,B,V] transpose as in the reference."""
    if ctc_logits.is_cuda and ctc_logits.dtype == torch.float32 and tokens.dim() == 2:
        from .ctc import ctc_loss_logits_groups

        return ctc_loss_logits_groups(ctc_logits, tokens, feat_lens, token_lens, blank_id, 1)[0]
    log_probs = F.log_softmax(ctc_logits, dim=-1)  # [B,T,V]
    return nn.CTCLoss(blank=blank_id, zero_infinity=True)(log_probs.transpose(0, 1), tokens,
                                                         feat_lens, token_lens)


def kl_logits(student_logits: torch.Tensor, teacher_logits: torch.Tensor, pad_mask: torch.Tensor):
    """KL(stopgrad p_teacher || p_student) per position, averaged over non-pad positions."""
    with torch.no_grad():
        p_t = F.softmax(teacher_logits, dim=-1)
    kl = F.kl_div(F.log_softmax(student_logits, dim=-1), p_t, reduction="none").sum(dim=-1)
    keep = (~pad_mask).float()
    return (kl * keep).sum() / keep.sum().clamp_min(1.0)
