"""Conformer encoder/decoder around the BitLinear hot path (call sites of QuantizedLinear).

Module tree, constructor signatures, forward signatures and parameter names follow the
reference's onebit_asr/conformer.py so that checkpoints (state-dict keys, eval.py:282)
and ``train.py`` call sites carry over unchanged:

* ``ConformerASR(input_dim, vocab_size, enc_d_model=256, enc_layers=12, enc_heads=4,
  enc_d_ff=1024, enc_conv_kernel=31, enc_dropout=0.1, dec_layers=2, dec_heads=4,
  dec_d_ff=1024, dec_dropout=0.1, pad_id=0)``                      (conformer.py:302-313)
* ``ConformerASR.forward(batch, precision, sp_mask=None) -> (enc_out, enc_mask, logits)``
  and ``decode_logits(enc_out, enc_mask, tgt_inp, tgt_pad_mask)``  (conformer.py:315-322)
* ``ConformerEncoder.forward(feats, feat_lens, precision, sp_mask=None)`` (:243-272)
* ``ConformerBlock.forward(x, src_mask, bitwidth_linear, pos_emb)``     (:222-228)
* ``MHSA.forward(x, mask, bitwidth, pos_emb)`` / ``FeedForwardModule.forward(x, bitwidth,
  mask=None)``                                                           (:105, :34)

Per block 9 QuantizedLinear call sites take the block's bitwidth: ff1.lin1/lin2,
mhsa.q/k/v/pos/out_proj, ff2.lin1/lin2. Everything else is full precision in the
reference (conv module "kept full-precision per paper recommendation", :225; subsampling
``out``, ``ctc_head``, decoder) and stays stock PyTorch-ROCm here.
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence

import torch
import torch.nn as nn
import torch.nn.functional as F

from .attention import fused_attention_supported, rel_pos_attention
from .conv import (conv2d_bias_relu, conv_module_fused, conv_module_supported, depthwise_conv1d,
                   subsample_convs, subsample_supported)
from .decattn import dec_attention, dec_attention_supported
from .embedding import embedding
from .fused import (ffn_residual, ffn_residual_i8, fused_supported, i8_fused_supported,
                    i8_linear, linear_residual, linear_residual_i8, qkv_projections)
from .layernorm import (Int8Act, fused_layernorm_supported, layer_norm, layer_norm_amax,
                        layer_norm_pair,
                        layer_norm_fork, layer_norm_i8)
from .linear import linear, linear_rows_split
from .quant import DeviceBits, PassBits, QuantizedLinear, StackedBits

__all__ = [
    "LayerNorm", "FeedForwardModule", "RelPositionalEncoding", "MHSA", "ConvModule",
    "Conv2dSubsampling", "ConformerBlock", "ConformerEncoder", "TransformerDecoder",
    "ConformerASR", "block_bitwidths", "subsampled_length",
]


def swish(x: torch.Tensor) -> torch.Tensor:
    # conformer.py:15-16 (x * sigmoid(x)); silu is the same function in one kernel.
    return F.silu(x)


class LayerNorm(nn.Module):
    """Wrapper kept for the ``<...>.ln.ln.weight`` checkpoint keys (conformer.py:19-24).
    On a ROCm device the normalisation runs on the HIP LayerNorm kernels (layernorm.py)."""

    def __init__(self, d_model: int):
        super().__init__()
        self.ln = nn.LayerNorm(d_model)
        # set by quant.set_act_quant on the LNs that feed int8 BitLinears: at inference the
        # LN kernel also produces the consumer's per-tensor absmax (y._ob_amax)
        self.emit_amax = False

    def forward(self, x):
        if (self.emit_amax and not torch.is_grad_enabled()
                and fused_layernorm_supported(x, x.shape[-1])):
            return layer_norm_amax(x, self.ln.weight, self.ln.bias, self.ln.eps)
        return layer_norm(x, self.ln.weight, self.ln.bias, self.ln.eps)

    def forward_i8(self, x):
        """Inference, int8 consumers: LN(x) as its int8 image + absmax (layernorm.Int8Act)."""
        return layer_norm_i8(x, self.ln.weight, self.ln.bias, self.ln.eps)

    def fork(self, x):
        """(LN(x), x) with the residual branch's gradient added in the LN backward."""
        return layer_norm_fork(x, self.ln.weight, self.ln.bias, self.ln.eps)

    def pair(self, x, nxt: "LayerNorm"):
        """LN(x), with nxt's LN of the result formed in the same launch (training)."""
        if self.emit_amax or nxt.emit_amax:
            return self(x)
        return layer_norm_pair(x, self.ln.weight, self.ln.bias, self.ln.eps, nxt.ln.weight,
                               nxt.ln.bias, nxt.ln.eps)


def _pad_rows(y: torch.Tensor, mask: Optional[torch.Tensor]) -> torch.Tensor:
    # Zero padded frames: mask is the [B,T,T] attention mask, mask[:, :, 0] the frame mask.
    if mask is None:
        return y
    return y * mask[:, :, 0].unsqueeze(-1)


class FeedForwardModule(nn.Module):
    """Macaron half-step FFN (conformer.py:27-45): x + 0.5*lin2(drop(swish(lin1(LN x))))."""

    def __init__(self, d_model: int, d_ff: int, dropout: float):
        super().__init__()
        self.ln = LayerNorm(d_model)
        self.lin1 = QuantizedLinear(d_model, d_ff)
        self.lin2 = QuantizedLinear(d_ff, d_model)
        self.dropout = nn.Dropout(dropout)

    # act_quant="absmax_int8" LN gets emit_amax (quant.set_act_quant)
    int8_ln = True

    def forward(self, x, bitwidth: int, mask=None, ln_next=None):
        """ln_next: the LayerNorm module(s) that normalise the output next, in order (training:
        formed in the last GEMM's epilogue, fused.ffn_residual)."""
        if mask is None and i8_fused_supported(x, self.lin1, self.lin2, bitwidth=bitwidth,
                                               p_drop=self.dropout.p if self.training else 0.0):
            # inference, int8 activations: LN (+absmax) -> lin1 i8 + swish (+absmax of its
            # output) -> lin2 i8 + 0.5 * residual, no separate absmax / elementwise passes
            h = (self.ln.forward_i8(x) if self.ln.emit_amax and fused_layernorm_supported(x, x.shape[-1])
                 else self.ln(x))
            return ffn_residual_i8(h, x, self.lin1, self.lin2, bitwidth)
        if mask is None and fused_supported(x, self.lin1, self.lin2, bitwidth=bitwidth):
            # same computation, elementwise ops in the GEMM epilogues (onebit_asr/fused.py)
            p = self.dropout.p if self.training else 0.0
            h, xr = self.ln.fork(x)
            lnn = ([(l.ln.weight, l.ln.bias, l.ln.eps) for l in ln_next]
                   if ln_next and not any(l.emit_amax for l in ln_next) else None)
            return ffn_residual(h, xr, self.lin1, self.lin2, bitwidth, p, lnn)
        h = self.lin1(self.ln(x), bitwidth)
        h = self.dropout(swish(h))
        h = self.dropout(self.lin2(h, bitwidth))
        return x + 0.5 * _pad_rows(h, mask)


class RelPositionalEncoding(nn.Module):
    """Absolute sinusoid table for positions 0..T-1 (conformer.py:48-76); x is not
    scaled by sqrt(d). The table is a persistent buffer ``pe`` [1, L, d] (L >= 5000),
    grown on demand."""

    def __init__(self, d_model: int, dropout_rate: float = 0.1, max_len: int = 5000):
        super().__init__()
        self.d_model = d_model
        self.dropout = nn.Dropout(p=dropout_rate)
        self.register_buffer("pe", self._table(max_len, torch.device("cpu")))

    def _table(self, length: int, device) -> torch.Tensor:
        pos = torch.arange(length, dtype=torch.float32).unsqueeze(1)
        freq = torch.exp(torch.arange(0, self.d_model, 2, dtype=torch.float32)
                         * -(math.log(10000.0) / self.d_model))
        table = torch.zeros(length, self.d_model)
        table[:, 0::2] = torch.sin(pos * freq)
        table[:, 1::2] = torch.cos(pos * freq)
        return table.unsqueeze(0).to(device)

    def extend_pe(self, length: int) -> None:
        if self.pe.size(1) < length:
            self.pe = self._table(length, self.pe.device)

    def forward(self, x):
        t = x.size(1)
        self.extend_pe(t)
        return self.dropout(x), self.pe[:, :t]


def rel_shift(scores: torch.Tensor) -> torch.Tensor:
    """Transformer-XL shift of a [B,H,T,T] score tensor exactly as conformer.py:97-103:
    prepend a zero column, reinterpret the (T, T+1) rows as a flat sequence and drop its
    first T entries."""
    b, h, t1, t2 = scores.shape
    padded = F.pad(scores, (1, 0))  # [B,H,T1,T2+1], zero column first
    return padded.reshape(b, h, -1)[:, :, t1:].reshape(b, h, t1, t2)


class MHSA(nn.Module):
    """Relative-position multi-head self-attention (conformer.py:79-138). Five BitLinear
    projections: q/k/v on LN(x), pos_proj on the batch-1 sinusoid table, out_proj."""

    int8_ln = True  # act_quant="absmax_int8": the LN also emits the q/k/v absmax

    def __init__(self, d_model: int, n_heads: int, dropout: float):
        super().__init__()
        assert d_model % n_heads == 0
        self.d_model = d_model
        self.n_heads = n_heads
        self.d_head = d_model // n_heads
        self.ln = LayerNorm(d_model)
        self.q_proj = QuantizedLinear(d_model, d_model)
        self.k_proj = QuantizedLinear(d_model, d_model)
        self.v_proj = QuantizedLinear(d_model, d_model)
        self.pos_proj = QuantizedLinear(d_model, d_model)
        self.out_proj = QuantizedLinear(d_model, d_model)
        self.dropout = nn.Dropout(dropout)
        self.pos_bias_u = nn.Parameter(torch.randn(self.n_heads, self.d_head) * 0.01)
        self.pos_bias_v = nn.Parameter(torch.randn(self.n_heads, self.d_head) * 0.01)

    def rel_shift(self, x):
        return rel_shift(x)

    def _heads(self, t: torch.Tensor, batch: int) -> torch.Tensor:
        return t.view(batch, -1, self.n_heads, self.d_head).transpose(1, 2)

    def _fused(self, x, h, mask, bitwidth, pos_emb):
        """The same computation with the attention core in one HIP kernel per direction
        (onebit_asr/attention.py); used on a ROCm device for supported shapes."""
        bsz, tlen, width = x.shape
        if isinstance(h, Int8Act):  # inference, int8 activations: LN(x) read as int8
            qp, kp, vp = (i8_linear(h, m, bitwidth) for m in (self.q_proj, self.k_proj, self.v_proj))
        elif fused_supported(h, self.q_proj, self.k_proj, self.v_proj, bitwidth=bitwidth):
            # one autograd node: dX of k / v accumulated in the GEMM epilogue (no adds)
            qp, kp, vp = qkv_projections(h, self.q_proj, self.k_proj, self.v_proj, bitwidth)
        else:
            qp = self.q_proj(h, bitwidth)
            kp = self.k_proj(h, bitwidth)
            vp = self.v_proj(h, bitwidth)
        if isinstance(bitwidth, PassBits):
            P = bitwidth.passes
            # the P stacked copies of the table: formed once per forward (the same pos_emb
            # tensor reaches every block), not once per block
            pe = getattr(pos_emb, "_ob_rows", None)
            if pe is None or pe.shape[0] != P * tlen:
                pe = pos_emb.expand(P, tlen, width).reshape(P * tlen, width)
                pos_emb._ob_rows = pe
            pp = self.pos_proj(pe, bitwidth).view(P, tlen, width)
        else:
            pp = self.pos_proj(pos_emb, bitwidth).view(1, tlen, width)
        if mask is None:
            lens = torch.full((bsz,), tlen, dtype=torch.int32, device=x.device)
        else:
            lens = getattr(mask, "_ob_lens", None)
            if lens is None:  # prefix masks (valid_i & valid_j): row 0 column = valid frames
                lens = mask[:, :, 0].sum(dim=1, dtype=torch.int32)
        p = self.dropout.p if self.training else 0.0
        ctx = rel_pos_attention(qp, kp, vp, pp, self.pos_bias_u, self.pos_bias_v, lens,
                                self.n_heads, p)
        if fused_supported(ctx, self.out_proj, bitwidth=bitwidth):
            # out_proj -> dropout -> zero padded rows -> + x in the GEMM epilogue
            return linear_residual(ctx, x, self.out_proj, bitwidth, p, 1.0,
                                   None if mask is None else lens, tlen)
        if i8_fused_supported(ctx, self.out_proj, bitwidth=bitwidth, p_drop=p):
            return linear_residual_i8(ctx, x, self.out_proj, bitwidth, 1.0,
                                      None if mask is None else lens, tlen)
        out = self.dropout(self.out_proj(ctx, bitwidth))
        return x + _pad_rows(out, mask)

    def forward(self, x, mask, bitwidth: int, pos_emb: torch.Tensor):
        bsz, tlen, width = x.shape
        assert width == self.d_model, f"Expected {self.d_model}, got {width}"
        if fused_attention_supported(x, self.d_head) and fused_supported(x, self.out_proj,
                                                                         bitwidth=bitwidth):
            h, xr = self.ln.fork(x)
            return self._fused(xr, h, mask, bitwidth, pos_emb)
        if (fused_attention_supported(x, self.d_head) and self.ln.emit_amax
                and fused_layernorm_supported(x, width)
                and i8_fused_supported(x, self.q_proj, self.k_proj, self.v_proj,
                                       bitwidth=bitwidth, p_drop=self.dropout.p if self.training else 0.0)):
            return self._fused(x, self.ln.forward_i8(x), mask, bitwidth, pos_emb)
        h = self.ln(x)
        if fused_attention_supported(h, self.d_head):
            return self._fused(x, h, mask, bitwidth, pos_emb)
        q = self._heads(self.q_proj(h, bitwidth), bsz)
        k = self._heads(self.k_proj(h, bitwidth), bsz)
        v = self._heads(self.v_proj(h, bitwidth), bsz)
        u_bias = self.pos_bias_u.view(1, self.n_heads, 1, self.d_head)
        v_bias = self.pos_bias_v.view(1, self.n_heads, 1, self.d_head)
        content = torch.matmul(q + u_bias, k.transpose(-2, -1))
        if isinstance(bitwidth, PassBits):
            # stacked passes: each pass projects the (shared) sinusoid table at its own
            # bitwidth; pass p's positions multiply pass p's queries only.
            P = bitwidth.passes
            pe = pos_emb.expand(P, tlen, width).reshape(P * tlen, width)
            p = self.pos_proj(pe, bitwidth).view(P, 1, tlen, self.n_heads, self.d_head)
            qv = (q + v_bias).view(P, bsz // P, self.n_heads, tlen, self.d_head)
            bd = torch.matmul(qv, p.permute(0, 1, 3, 4, 2))
            position = rel_shift(bd.view(bsz, self.n_heads, tlen, tlen))
        else:
            p = self._heads(self.pos_proj(pos_emb, bitwidth), 1)
            position = rel_shift(torch.matmul(q + v_bias, p.transpose(-2, -1)))
        scores = (content + position) / math.sqrt(self.d_head)
        if mask is not None:
            scores = scores.masked_fill(mask[:, None, :, :] == 0, float("-inf"))
        # Fully masked rows are all -inf -> NaN; the reference zeroes them (:124-127).
        attn = self.dropout(torch.nan_to_num(torch.softmax(scores, dim=-1), nan=0.0))
        ctx = torch.matmul(attn, v).transpose(1, 2).contiguous().view(bsz, tlen, width)
        out = self.dropout(self.out_proj(ctx, bitwidth))
        return x + _pad_rows(out, mask)


class ConvModule(nn.Module):
    """LN -> pw1 -> GLU -> depthwise k -> BatchNorm(batch stats, track_running_stats=False)
    -> swish -> pw2 (conformer.py:141-167). Full precision."""

    def __init__(self, d_model: int, kernel_size: int = 31, dropout: float = 0.1,
                 quantize_pointwise: bool = False):
        super().__init__()
        self.ln = LayerNorm(d_model)
        # north_star lists the pointwise 1x1s as BitLinear call sites; the reference keeps
        # them full precision (conformer.py:225), so ternary pw1/pw2 is opt-in: they become
        # channels-last QuantizedLinear layers (keys pw1.weight [2C, C], pw1.alpha, pw1.bias)
        # at the block's bitwidth. Off (default) = the reference's Conv1d(k=1) keys/math.
        self.quantize_pointwise = quantize_pointwise
        if quantize_pointwise:
            self.pw1 = QuantizedLinear(d_model, 2 * d_model)
        else:
            self.pw1 = nn.Conv1d(d_model, 2 * d_model, kernel_size=1)
        self.glu = nn.GLU(dim=1)
        self.dw = nn.Conv1d(d_model, d_model, kernel_size=kernel_size,
                            padding=kernel_size // 2, groups=d_model)
        self.bn = nn.BatchNorm1d(d_model, track_running_stats=False)
        if quantize_pointwise:
            self.pw2 = QuantizedLinear(d_model, d_model)
        else:
            self.pw2 = nn.Conv1d(d_model, d_model, kernel_size=1)
        self.dropout = nn.Dropout(dropout)

    def _bn(self, h: torch.Tensor, passes: int) -> torch.Tensor:
        if passes == 1:
            return self.bn(h)
        # Stacked passes keep per-pass batch statistics (each reference pass normalises its
        # own batch): pass p's channels become channels p*C .. p*C+C of one BatchNorm.
        pb, c, t = h.shape
        b = pb // passes
        hp = h.view(passes, b, c, t).transpose(0, 1).reshape(b, passes * c, t)
        y = F.batch_norm(hp, None, None, self.bn.weight.repeat(passes),
                         self.bn.bias.repeat(passes), True, self.bn.momentum or 0.0, self.bn.eps)
        return y.view(b, passes, c, t).transpose(0, 1).reshape(pb, c, t)

    def forward(self, x, mask=None, passes: int = 1, bitwidth=None):
        """``bitwidth``: the block's BitLinear bitwidth, used only by ternary pointwise
        layers (``quantize_pointwise``); the reference passes none (conformer.py:225)."""
        if self.quantize_pointwise and bitwidth is None:
            raise ValueError("quantize_pointwise ConvModule needs the block bitwidth")
        if mask is None and conv_module_supported(x, self):
            # channels-last on the HIP kernels (conv.py / csrc/convmod.hip), same computation
            p = self.dropout.p if self.training else 0.0
            h, xr = self.ln.fork(x)
            return conv_module_fused(xr, h, self, passes, p, bitwidth)
        if self.quantize_pointwise:
            h = self.glu(self.pw1(self.ln(x), bitwidth).transpose(1, 2))
            h = swish(self._bn(depthwise_conv1d(h, self.dw), passes))
            h = self.pw2(h.transpose(1, 2), bitwidth)
            h = self.dropout(h)
            return x + _pad_rows(h, mask)
        h = self.glu(self.pw1(self.ln(x).transpose(1, 2)))
        h = self.pw2(swish(self._bn(depthwise_conv1d(h, self.dw), passes)))
        h = self.dropout(h).transpose(1, 2)
        return x + _pad_rows(h, mask)


def subsampled_length(t: int) -> int:
    """Frames after two k=3, s=2 valid convolutions (conformer.py:183-185)."""
    return ((t - 3) // 2 + 1 - 3) // 2 + 1


class Conv2dSubsampling(nn.Module):
    """[B,T,F] -> [B,T',d] with two 3x3 stride-2 Conv2d + ReLU and a Linear over
    (d x F') (conformer.py:170-208)."""

    def __init__(self, idim: int, d_model: int):
        super().__init__()
        self.d_model = d_model
        self.conv = nn.Sequential(
            nn.Conv2d(1, d_model, kernel_size=3, stride=2),
            nn.ReLU(),
            nn.Conv2d(d_model, d_model, kernel_size=3, stride=2),
            nn.ReLU(),
        )
        f_out = ((idim - 1) // 2 - 1) // 2
        if f_out <= 0:
            raise ValueError(f"Input dim too small for Conv2dSubsampling: idim={idim}")
        self.out = nn.Linear(d_model * f_out, d_model)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if subsample_supported(x, self.conv[0], self.conv[2]):
            # channels-last implicit GEMMs (csrc/subsample.hip): y [B, T', F', C]; the
            # Linear's columns are permuted to that order instead of transposing y
            y = subsample_convs(x, self.conv[0], self.conv[2])
            bsz, tsub, fsub, ch = y.shape
            w = self.out.weight.view(-1, ch, fsub).transpose(1, 2).reshape(-1, fsub * ch)
            return linear(y.view(bsz, tsub, fsub * ch), w, self.out.bias)
        if x.is_cuda and x.dtype == torch.float32:  # bias + ReLU fused (conv.py)
            y = conv2d_bias_relu(conv2d_bias_relu(x.unsqueeze(1), self.conv[0]), self.conv[2])
        else:
            y = self.conv(x.unsqueeze(1))                  # [B, C, T', F']
        bsz, ch, tsub, fsub = y.shape
        y = y.transpose(1, 2).reshape(bsz, tsub, ch * fsub)  # channel-major per frame
        return linear(y, self.out.weight, self.out.bias)


class ConformerBlock(nn.Module):
    """ff1 -> mhsa -> conv (FP) -> ff2 -> LN (conformer.py:212-228)."""

    def __init__(self, d_model: int, d_ff: int, n_heads: int, conv_kernel: int, dropout: float,
                 block_index: int, quantize_conv_pointwise: bool = False):
        super().__init__()
        self.block_index = block_index
        self.ff1 = FeedForwardModule(d_model, d_ff, dropout)
        self.mhsa = MHSA(d_model, n_heads, dropout)
        self.conv = ConvModule(d_model, kernel_size=conv_kernel, dropout=dropout,
                               quantize_pointwise=quantize_conv_pointwise)
        self.ff2 = FeedForwardModule(d_model, d_ff, dropout)
        self.ln = LayerNorm(d_model)

    def forward(self, x, src_mask, bitwidth_linear: int, pos_emb: torch.Tensor,
                next_ln: Optional["LayerNorm"] = None):
        """next_ln: the LayerNorm that will normalise this block's output next (the following
        block's ff1.ln or the encoder's ln_out); its forward is formed together with this
        block's final LN (layernorm.layer_norm_pair)."""
        x = self.ff1(x, bitwidth_linear, ln_next=[self.mhsa.ln])
        x = self.mhsa(x, src_mask, bitwidth_linear, pos_emb)
        passes = bitwidth_linear.passes if isinstance(bitwidth_linear, PassBits) else 1
        # the reference does not pass the mask here (:225); the bitwidth reaches only
        # opt-in ternary pointwise layers
        x = self.conv(x, passes=passes,
                      bitwidth=bitwidth_linear if self.conv.quantize_pointwise else None)
        x = self.ff2(x, bitwidth_linear,
                     ln_next=[self.ln] if next_ln is None or next_ln.emit_amax else [self.ln, next_ln])
        return self.ln(x) if next_ln is None else self.ln.pair(x, next_ln)


def block_bitwidths(n_layers: int, precision: int, sp_mask: Optional[Sequence[int]]) -> List[int]:
    """Per-block BitLinear bitwidth (conformer.py:265-269): ``precision`` everywhere, or with
    an SP mask 1 where sp_mask[i] == 1 else 2; anything outside {1, 2} runs at 32."""
    if isinstance(sp_mask, (DeviceBits, StackedBits)):  # bitwidths read on device
        return [sp_mask[i] for i in range(n_layers)]
    out = []
    for i in range(n_layers):
        bw = precision if sp_mask is None else (1 if sp_mask[i] == 1 else 2)
        out.append(bw if bw in (1, 2) else 32)
    return out


class ConformerEncoder(nn.Module):
    def __init__(self, input_dim: int, d_model: int, n_layers: int, n_heads: int,
                 d_ff: int, conv_kernel: int, dropout: float,
                 quantize_conv_pointwise: bool = False):
        super().__init__()
        self.subsample = Conv2dSubsampling(input_dim, d_model)
        self.pos_enc = RelPositionalEncoding(d_model, dropout)
        self.blocks = nn.ModuleList([
            ConformerBlock(d_model, d_ff, n_heads, conv_kernel, dropout, i,
                           quantize_conv_pointwise)
            for i in range(n_layers)
        ])
        self.ln_out = LayerNorm(d_model)

    def forward(self, feats: torch.Tensor, feat_lens: torch.Tensor,
                precision: int, sp_mask: Optional[List[int]] = None):
        """conformer.py:243-272. Frame validity uses feat_lens // 4 against the T' actually
        produced by the convolutions (so it can disagree by one frame, as in the reference).

        With a ``StackedBits`` table (the three passes of a training step stacked on the
        batch dim) ``feats`` holds ONE copy of the batch: the subsampling convolutions have
        no dropout and full-precision weights, so all passes compute the same [B, T', d]
        output; it is computed once and repeated per pass (autograd sums the passes'
        gradients into the one backward)."""
        x = self.subsample(feats)
        if isinstance(sp_mask, StackedBits):
            x = x.repeat(sp_mask.passes, 1, 1)
            feat_lens = feat_lens.repeat(sp_mask.passes)
        tsub = x.size(1)
        x, pos_emb = self.pos_enc(x)
        frames = torch.arange(tsub, device=feats.device).unsqueeze(0)
        key_mask = frames < (feat_lens // 4).unsqueeze(1)            # [B, T'] bool
        attn_mask = key_mask.unsqueeze(2) & key_mask.unsqueeze(1)     # [B, T', T']
        # valid frames per utterance, for the fused attention kernels (prefix masks)
        attn_mask._ob_lens = key_mask.sum(dim=1, dtype=torch.int32)
        bws = block_bitwidths(len(self.blocks), precision, sp_mask)
        n = len(self.blocks)
        for i, (blk, bw) in enumerate(zip(self.blocks, bws)):
            nxt = self.blocks[i + 1].ff1.ln if i + 1 < n else self.ln_out
            x = blk(x, attn_mask, bw, pos_emb, next_ln=nxt)
        return self.ln_out(x), key_mask




def _residual_dropout(x: torch.Tensor, y: torch.Tensor, p: float, training: bool):
    """x + dropout(y) of a post-norm decoder sublayer (nn.TransformerDecoderLayer's
    ``norm_k(x + dropout_k(sublayer(x)))``) in one kernel with the fused call sites' hash
    mask (conv.py _ResidualDropFn); the dropout backward is formed by the following
    LayerNorm's backward (layernorm.GradScale) instead of a pass of its own."""
    if not (training and p > 0):
        return x + y
    if not (x.is_cuda and x.shape == y.shape):
        return x + F.dropout(y, p, training)
    from .conv import _ResidualDropFn
    from .fused import _rng
    from .layernorm import GradScale, attach_grad_scale

    rng, off = _rng(x.device)
    spec = GradScale(1.0, p, rng, off)
    return attach_grad_scale(_ResidualDropFn.apply(x, y, float(p), rng, off, spec), spec)


class TransformerDecoder(nn.Module):
    """Stock 2-layer nn.TransformerDecoder head (conformer.py:275-299), full precision.

    The modules (and so the initialisation and the checkpoint keys
    ``decoder.dec.layers.i.{self_attn,multihead_attn}.{in_proj_weight,in_proj_bias,
    out_proj.*}``, ``linear1/2``, ``norm1/2/3``) are torch's ``nn.TransformerDecoderLayer``
    (batch_first, post-norm, relu). On a ROCm device the forward is restated functionally
    (``_layer``) with the same math on graph-safe pieces -- ``linear`` (fixed-order bias
    gradients), the HIP LayerNorm, explicit scaled-dot-product attention -- because torch's
    own bias-gradient reductions are not replayable from a HIP graph on this ROCm build
    (onebit_asr/linear.py). CPU tensors run torch's modules as they are."""

    def __init__(self, vocab_size: int, d_model: int, n_layers: int, n_heads: int,
                 d_ff: int, dropout: float, pad_id: int):
        super().__init__()
        self.emb = nn.Embedding(vocab_size, d_model, padding_idx=pad_id)
        layer = nn.TransformerDecoderLayer(d_model=d_model, nhead=n_heads, dim_feedforward=d_ff,
                                           dropout=dropout, batch_first=True)
        self.dec = nn.TransformerDecoder(layer, num_layers=n_layers)
        self.ln = LayerNorm(d_model)
        self.out = nn.Linear(d_model, vocab_size)

    @staticmethod
    def _attention(mha: nn.MultiheadAttention, x, mem, bias, training: bool):
        """torch.nn.functional.multi_head_attention_forward (need_weights=False) for
        batch-first inputs: packed in-projection, softmax(q k^T / sqrt(dh) + bias) with
        attention dropout, out-projection. ``bias`` is the additive mask, or a
        (key-padding mask, causal) pair for the HIP core (decattn.py)."""
        e, h = mha.embed_dim, mha.num_heads
        dh = e // h
        w, b = mha.in_proj_weight, mha.in_proj_bias
        bsz, lq, _ = x.shape
        if isinstance(bias, tuple):  # HIP attention core on the packed projections
            kmask, causal = bias
            if mem is None:
                ctx = dec_attention(linear(x, w, b), None, h, kmask, causal, mha.dropout,
                                    training)
            else:
                qp, kvp = linear_rows_split(x, mem, w, b, e)
                ctx = dec_attention(qp, kvp, h, kmask, causal, mha.dropout, training)
            return linear(ctx, mha.out_proj.weight, mha.out_proj.bias)
        if mem is None:  # self-attention: one packed projection, chunks q | k | v
            q, k, v = linear(x, w, b).chunk(3, dim=-1)
            lk = lq
        else:
            q = linear(x, w[:e], b[:e])
            k, v = linear(mem, w[e:], b[e:]).chunk(2, dim=-1)
            lk = mem.size(1)
        q = q.reshape(bsz, lq, h, dh).transpose(1, 2)
        k = k.reshape(bsz, lk, h, dh).transpose(1, 2)
        v = v.reshape(bsz, lk, h, dh).transpose(1, 2)
        att = torch.matmul(q, k.transpose(-2, -1)) * (1.0 / math.sqrt(dh)) + bias
        att = F.dropout(torch.softmax(att, dim=-1), mha.dropout, training)
        ctx = torch.matmul(att, v).transpose(1, 2).reshape(bsz, lq, e)
        return linear(ctx, mha.out_proj.weight, mha.out_proj.bias)

    def _layer(self, lyr: nn.TransformerDecoderLayer, x, mem, self_bias, cross_bias):
        """nn.TransformerDecoderLayer.forward, norm_first=False:
        x = norm1(x + sa(x)); x = norm2(x + mha(x, mem)); x = norm3(x + ff(x))."""
        tr = self.training
        n1, n2, n3 = lyr.norm1, lyr.norm2, lyr.norm3
        sa = self._attention(lyr.self_attn, x, None, self_bias, tr)
        x = layer_norm(_residual_dropout(x, sa, lyr.dropout1.p, tr), n1.weight, n1.bias, n1.eps)
        ca = self._attention(lyr.multihead_attn, x, mem, cross_bias, tr)
        x = layer_norm(_residual_dropout(x, ca, lyr.dropout2.p, tr), n2.weight, n2.bias, n2.eps)
        ff = linear(F.dropout(F.relu(linear(x, lyr.linear1.weight, lyr.linear1.bias)),
                              lyr.dropout.p, tr), lyr.linear2.weight, lyr.linear2.bias)
        return layer_norm(_residual_dropout(x, ff, lyr.dropout3.p, tr), n3.weight, n3.bias,
                          n3.eps)

    def forward(self, tgt_inp, memory, memory_mask, tgt_key_padding_mask):
        tt = tgt_inp.size(1)
        tok = embedding(tgt_inp, self.emb.weight, self.emb.padding_idx)
        dh = memory.size(-1) // self.dec.layers[0].self_attn.num_heads
        if (dec_attention_supported(memory, tt, tt, dh)
                and dec_attention_supported(memory, tt, memory.size(1), dh)):
            # the HIP core takes the masks as they are: key padding (+ causal) per batch row
            self_bias = (tgt_key_padding_mask, True)
            cross_bias = (memory_mask == 0, False)
            y = tok
            for lyr in self.dec.layers:
                y = self._layer(lyr, y, memory, self_bias, cross_bias)
            if self.dec.norm is not None:
                y = layer_norm(y, self.dec.norm.weight, self.dec.norm.bias, self.dec.norm.eps)
            return linear(self.ln(y), self.out.weight, self.out.bias)
        future = torch.ones(tt, tt, device=tgt_inp.device).triu(diagonal=1).bool()
        causal = torch.zeros(tt, tt, device=tgt_inp.device).masked_fill(future, float("-inf"))
        if not (memory.is_cuda and memory.dtype == torch.float32):
            # tgt_is_causal=True is what torch's _detect_is_causal_mask concludes for this mask
            # in the reference call (the explicit mask is still used).
            y = self.dec(tok, memory, tgt_mask=causal,
                         memory_key_padding_mask=(memory_mask == 0),
                         tgt_key_padding_mask=tgt_key_padding_mask, tgt_is_causal=True)
            return self.out(self.ln(y))
        # additive masks as multi_head_attention_forward merges them: causal + key padding
        # for self-attention, memory padding for cross-attention ([B, 1, Lq, Lk])
        neg = float("-inf")
        self_bias = causal.view(1, 1, tt, tt) + torch.zeros(
            tgt_key_padding_mask.shape, device=tok.device).masked_fill(
            tgt_key_padding_mask, neg).view(-1, 1, 1, tt)
        cross_bias = torch.zeros(memory_mask.shape, device=tok.device).masked_fill(
            memory_mask == 0, neg).view(memory_mask.size(0), 1, 1, -1)
        y = tok
        for lyr in self.dec.layers:
            y = self._layer(lyr, y, memory, self_bias, cross_bias)
        if self.dec.norm is not None:
            y = layer_norm(y, self.dec.norm.weight, self.dec.norm.bias, self.dec.norm.eps)
        return linear(self.ln(y), self.out.weight, self.out.bias)


class ConformerASR(nn.Module):
    def __init__(self, input_dim: int, vocab_size: int,
                 enc_d_model=256, enc_layers=12, enc_heads=4, enc_d_ff=1024,
                 enc_conv_kernel=31, enc_dropout=0.1,
                 dec_layers=2, dec_heads=4, dec_d_ff=1024, dec_dropout=0.1,
                 pad_id=0, quantize_conv_pointwise: bool = False):
        """``quantize_conv_pointwise`` (not in the reference, default off): ternary conv-module
        pw1/pw2 (north_star's "conv-module pointwise 1x1s"); diverges from the reference's
        full-precision pointwise convs (conformer.py:225) when on."""
        super().__init__()
        self.encoder = ConformerEncoder(input_dim, enc_d_model, enc_layers, enc_heads,
                                        enc_d_ff, enc_conv_kernel, enc_dropout,
                                        quantize_conv_pointwise)
        self.decoder = TransformerDecoder(vocab_size, enc_d_model, dec_layers, dec_heads,
                                          dec_d_ff, dec_dropout, pad_id)
        self.ctc_head = nn.Linear(enc_d_model, vocab_size)

    def forward(self, batch, precision: int, sp_mask=None):
        enc_out, enc_mask = self.encoder(batch["feats"], batch["feat_lens"], precision, sp_mask)
        return enc_out, enc_mask, self.ctc_logits(enc_out)

    def ctc_logits(self, enc_out):
        return linear(enc_out, self.ctc_head.weight, self.ctc_head.bias)

    def decode_logits(self, enc_out, enc_mask, tgt_inp, tgt_pad_mask):
        return self.decoder(tgt_inp, enc_out, enc_mask, tgt_pad_mask)
