"""Functional CPU restatement of the reference model and step — TEST INFRASTRUCTURE ONLY.

Imported only by ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg.

Restates, as plain functions over a state dict of fp32 CPU tensors, the forward semantics
of y00njaekim/CMU-11785-IDL-1.58bit-ASR:

* ``onebit_asr/conformer.py`` — Conv2dSubsampling (:170-208), RelPositionalEncoding
  (:48-76), FFN (:27-45), rel-pos MHSA incl. rel_shift / mask / nan_to_num (:79-138),
  ConvModule with batch-statistics BatchNorm (:141-167), block/encoder wiring and the
  per-block bitwidth rule (:212-272), decoder (:275-299), CTC head (:313-319);
* ``onebit_asr/quant.py`` — via ``quant_oracle.ref_quantized_linear`` (:38-127);
* ``onebit_asr/losses.py`` (:11-59) and the step's loss combination (train.py:82-111),
  with the reference's materialised label-smoothing distribution.

It shares no code with the product package: rel_shift is re-derived as an index gather,
the sinusoid table is recomputed per call, and parameters are addressed by their
checkpoint keys. The stock third-party parts (TransformerDecoder layers, CTCLoss,
conv/LN/BN arithmetic) are torch's own, as in the reference (torch is not vendored; see
SURVEY.md §8c "Third-party arithmetic").
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from .quant_oracle import ref_quantized_linear

__all__ = ["OracleConformer", "oracle_step_loss", "oracle_losses"]


def _sinusoids(length: int, d: int) -> torch.Tensor:
    pos = torch.arange(length, dtype=torch.float32)[:, None]
    inv = torch.exp(torch.arange(0, d, 2, dtype=torch.float32) * -(math.log(10000.0) / d))
    ang = pos * inv
    table = torch.empty(length, d)
    table[:, 0::2] = torch.sin(ang)
    table[:, 1::2] = torch.cos(ang)
    return table


def _rel_shift_gather(s: torch.Tensor) -> torch.Tensor:
    """conformer.py:97-103 as an explicit gather: with P = [0 | s] (row length T2+1),
    out.flat[i] = P.flat[T1 + i]."""
    b, h, t1, t2 = s.shape
    padded = torch.cat([s.new_zeros(b, h, t1, 1), s], dim=-1).reshape(b, h, t1 * (t2 + 1))
    idx = torch.arange(t1, t1 + t1 * t2)
    return padded[:, :, idx].reshape(b, h, t1, t2)


class OracleConformer(nn.Module):
    """Holds the reference's parameters under sanitised names; forward is functional."""

    def __init__(self, state_dict: Dict[str, torch.Tensor], *, input_dim: int, vocab_size: int,
                 d_model: int, n_layers: int, n_heads: int, d_ff: int, conv_kernel: int,
                 dec_layers: int, dec_heads: int, dec_d_ff: int, dropout: float = 0.0,
                 pad_id: int = 0):
        super().__init__()
        self.d = d_model
        self.n_layers = n_layers
        self.n_heads = n_heads
        self.kernel = conv_kernel
        self.p_drop = dropout
        self.pad_id = pad_id
        self._keys = []
        for key, val in state_dict.items():
            if key.startswith("decoder.dec.") or key.endswith(".pe"):
                continue
            self.register_parameter(key.replace(".", "__"),
                                    nn.Parameter(val.detach().to("cpu", torch.float32).clone()))
            self._keys.append(key)
        layer = nn.TransformerDecoderLayer(d_model=d_model, nhead=dec_heads,
                                           dim_feedforward=dec_d_ff, dropout=dropout,
                                           batch_first=True)
        self.dec_stack = nn.TransformerDecoder(layer, num_layers=dec_layers)
        dec_sd = {k[len("decoder.dec."):]: v.detach().cpu().float()
                  for k, v in state_dict.items() if k.startswith("decoder.dec.")}
        self.dec_stack.load_state_dict(dec_sd)

    # -- parameter access by checkpoint key ----------------------------------------
    def p(self, key: str) -> torch.Tensor:
        return getattr(self, key.replace(".", "__"))

    def named_reference_parameters(self):
        for k in self._keys:
            yield k, self.p(k)
        for k, v in self.dec_stack.named_parameters():
            yield "decoder.dec." + k, v

    def _drop(self, x):
        return F.dropout(x, self.p_drop, self.training) if self.p_drop > 0 else x

    def _ln(self, x, pre):
        return F.layer_norm(x, (x.shape[-1],), self.p(pre + ".ln.weight"), self.p(pre + ".ln.bias"))

    def _ql(self, x, pre, bits):
        bias_key = pre + ".bias"
        bias = self.p(bias_key) if bias_key in self._keys else None
        return ref_quantized_linear(x, self.p(pre + ".weight"), self.p(pre + ".alpha"), bias, bits)

    # -- blocks --------------------------------------------------------------------
    def _ffn(self, x, pre, bits):
        y = self._ql(self._ln(x, pre + ".ln"), pre + ".lin1", bits)
        y = self._drop(y * torch.sigmoid(y))
        y = self._drop(self._ql(y, pre + ".lin2", bits))
        return x + 0.5 * y

    def _mhsa(self, x, mask, bits, pos, pre):
        b, t, d = x.shape
        h, dh = self.n_heads, d // self.n_heads
        y = self._ln(x, pre + ".ln")

        def split(z, bb):
            return z.reshape(bb, t, h, dh).permute(0, 2, 1, 3)

        q = split(self._ql(y, pre + ".q_proj", bits), b)
        k = split(self._ql(y, pre + ".k_proj", bits), b)
        v = split(self._ql(y, pre + ".v_proj", bits), b)
        pp = split(self._ql(pos, pre + ".pos_proj", bits), 1)
        u = self.p(pre + ".pos_bias_u")[None, :, None, :]
        vb = self.p(pre + ".pos_bias_v")[None, :, None, :]
        ac = (q + u) @ k.transpose(-1, -2)
        bd = _rel_shift_gather((q + vb) @ pp.transpose(-1, -2))
        sc = (ac + bd) / math.sqrt(dh)
        sc = sc.masked_fill(~mask[:, None], float("-inf"))
        a = torch.softmax(sc, dim=-1)
        a = self._drop(torch.nan_to_num(a, nan=0.0))
        o = (a @ v).permute(0, 2, 1, 3).reshape(b, t, d)
        o = self._drop(self._ql(o, pre + ".out_proj", bits))
        o = o * mask[:, :, 0, None].to(o.dtype)
        return x + o

    def _conv(self, x, pre):
        y = self._ln(x, pre + ".ln").transpose(1, 2)
        y = F.conv1d(y, self.p(pre + ".pw1.weight"), self.p(pre + ".pw1.bias"))
        y = F.glu(y, dim=1)
        y = F.conv1d(y, self.p(pre + ".dw.weight"), self.p(pre + ".dw.bias"),
                     padding=self.kernel // 2, groups=self.d)
        y = F.batch_norm(y, None, None, self.p(pre + ".bn.weight"), self.p(pre + ".bn.bias"),
                         training=True)
        y = y * torch.sigmoid(y)
        y = F.conv1d(y, self.p(pre + ".pw2.weight"), self.p(pre + ".pw2.bias"))
        return x + self._drop(y).transpose(1, 2)

    # -- model ---------------------------------------------------------------------
    def encode(self, feats, feat_lens, precision: int, sp_mask: Optional[List[int]] = None):
        pre = "encoder.subsample"
        z = F.relu(F.conv2d(feats[:, None], self.p(pre + ".conv.0.weight"),
                            self.p(pre + ".conv.0.bias"), stride=2))
        z = F.relu(F.conv2d(z, self.p(pre + ".conv.2.weight"), self.p(pre + ".conv.2.bias"),
                            stride=2))
        b, c, t, f = z.shape
        x = F.linear(z.permute(0, 2, 1, 3).reshape(b, t, c * f), self.p(pre + ".out.weight"),
                     self.p(pre + ".out.bias"))
        x = self._drop(x)
        pos = _sinusoids(t, self.d)[None]
        valid = torch.arange(t)[None, :] < torch.div(feat_lens, 4, rounding_mode="floor")[:, None]
        mask = valid[:, :, None] & valid[:, None, :]
        for i in range(self.n_layers):
            if sp_mask is not None:
                bits = 1 if sp_mask[i] == 1 else 2
            else:
                bits = precision
            if bits not in (1, 2):
                bits = 32
            pre = f"encoder.blocks.{i}"
            x = self._ffn(x, pre + ".ff1", bits)
            x = self._mhsa(x, mask, bits, pos, pre + ".mhsa")
            x = self._conv(x, pre + ".conv")
            x = self._ffn(x, pre + ".ff2", bits)
            x = self._ln(x, pre + ".ln")
        return self._ln(x, "encoder.ln_out"), valid

    def forward(self, batch, precision: int, sp_mask=None):
        enc, valid = self.encode(batch["feats"], batch["feat_lens"], precision, sp_mask)
        logits = F.linear(enc, self.p("ctc_head.weight"), self.p("ctc_head.bias"))
        return enc, valid, logits

    def decode_logits(self, enc, enc_mask, tgt_inp, tgt_pad_mask):
        tt = tgt_inp.shape[1]
        causal = torch.full((tt, tt), float("-inf")).triu(1)
        y = F.embedding(tgt_inp, self.p("decoder.emb.weight"), padding_idx=self.pad_id)
        y = self.dec_stack(y, enc, tgt_mask=causal, memory_key_padding_mask=~enc_mask,
                           tgt_key_padding_mask=tgt_pad_mask)
        y = self._ln(y, "decoder.ln")
        return F.linear(y, self.p("decoder.out.weight"), self.p("decoder.out.bias"))


def oracle_losses():
    """losses.py:11-59 restated (label smoothing via the materialised distribution)."""

    def targets(tokens, bos, eos, pad):
        b = tokens.shape[0]
        tin = torch.cat([torch.full((b, 1), bos, dtype=tokens.dtype), tokens], 1)
        tout = torch.cat([tokens, torch.full((b, 1), eos, dtype=tokens.dtype)], 1)
        return tin, tout, tin == pad

    def ce(logits, tgt, pad, eps):
        logp = F.log_softmax(logits, -1)
        v = logits.shape[-1]
        dist = torch.full_like(logp, eps / (v - 1)).scatter(2, tgt[..., None], 1.0 - eps)
        per = (-(dist * logp)).sum(-1)
        m = (tgt != pad).float()
        return (per.mean() * m).sum() / m.sum().clamp_min(1.0)

    def ctc(logits, lens, tokens, tlens, blank):
        lp = F.log_softmax(logits, -1).transpose(0, 1)
        return F.ctc_loss(lp, tokens, lens, tlens, blank=blank, reduction="mean",
                          zero_infinity=True)

    def kl(student, teacher, pad_mask):
        pt = F.softmax(teacher.detach(), -1)
        ls = F.log_softmax(student, -1)
        per = torch.where(pt > 0, pt * (torch.log(pt) - ls), torch.zeros_like(pt)).sum(-1)
        m = (~pad_mask).float()
        return (per * m).sum() / m.sum().clamp_min(1.0)

    return targets, ce, ctc, kl


def oracle_step_loss(model: OracleConformer, batch, sp_mask, special=None, gamma=0.2,
                     lambda1=0.5, lambda2=1.0, eps=0.1):
    """train.py:82-111: teacher (2-bit), student (1-bit), SP pass; returns (loss, parts)."""
    sp = special or {"pad_id": 0, "bos_id": 1, "eos_id": 2, "blank_id": 3}
    targets, ce, ctc, kl = oracle_losses()
    tin, tout, tpad = targets(batch["tokens"], sp["bos_id"], sp["eos_id"], sp["pad_id"])

    def run(prec, mask=None):
        enc, valid, lc = model(batch, prec, mask)
        logits = model.decode_logits(enc, valid, tin, tpad)
        latt = ce(logits, tout, sp["pad_id"], eps)
        lctc = ctc(lc, valid.sum(1).long(), batch["tokens"], batch["token_lens"], sp["blank_id"])
        return logits, (1 - gamma) * latt + gamma * lctc, lctc

    lg2, li2, lc2 = run(2)
    lg1, li1, lc1 = run(1)
    k1 = kl(lg1, lg2, tpad)
    lgs, lis, lcs = run(2, sp_mask)
    ks = kl(lgs, lg2, tpad)
    loss = li2 + lambda1 * (li1 + lis) + lambda2 * (k1 + ks)
    parts = torch.stack([li2, li1, lis, k1, ks, lc2, lc1, lcs]).detach()
    return loss, parts
