"""The decoder's attention core on one HIP launch per direction (csrc/decattn.hip).

Reference: the stock ``nn.TransformerDecoderLayer`` of conformer.py:275-299, i.e. torch's
``multi_head_attention_forward`` between the in- and out-projections:
``ctx = dropout(softmax((q k^T) * (1/sqrt(dh)) + mask)) v`` per head, ``mask`` = -inf at
padded keys (``tgt_key_padding_mask`` for self-attention, ``memory_mask == 0`` for
cross-attention) and, for self-attention, at future keys (the causal mask). The packed
projection outputs are read in place (self-attention: one ``[B, L, 3e]`` tensor holding
q | k | v; cross-attention: ``q [B, Lq, e]`` and ``kv [B, Lk, 2e]``) and their gradients are
written into the packed gradients, so no head-split copies or ``chunk`` views exist.
Dropout uses the library's counter hash (fused.py's shared rng), not torch's Philox stream.
"""
from __future__ import annotations


import torch

from . import _lib

__all__ = ["dec_attention", "dec_attention_supported"]

_ON = True  # parity-test hook (tests/test_decattn_gpu.py: False = the torch attention ops)


def dec_attention_supported(x: torch.Tensor, lq: int, lk: int, dh: int) -> bool:
    return (_ON and x.is_cuda and x.dtype == torch.float32
            and bool(_lib.load().ob_decattn_supported(lq, lk, dh)))


class _DecAttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, xq, xkv, heads, kmask, causal, p, rng, off):
        lib = _lib.load()
        xq = xq.contiguous()
        B, Lq, wq = xq.shape
        if xkv is None:  # self-attention: q | k | v column blocks of one tensor
            e = wq // 3
            src, Lk, sq, skv, koff, voff = xq, Lq, wq, wq, e, 2 * e
        else:
            xkv = xkv.contiguous()
            e = wq
            src, Lk, sq, skv, koff, voff = xkv, xkv.shape[1], e, xkv.shape[2], 0, e
        dh = e // heads
        probs = torch.empty((B, heads, Lq, Lk), dtype=torch.float32, device=xq.device)
        out = torch.empty((B, Lq, e), dtype=torch.float32, device=xq.device)
        km = kmask.contiguous() if kmask is not None else None
        base = src.data_ptr()
        _lib.check(lib.ob_decattn_fwd(xq.data_ptr(), sq, base + 4 * koff, skv, base + 4 * voff, skv,
                                      _lib.ptr(km), int(causal), B, heads, Lq, Lk, dh, float(p),
                                      _lib.ptr(rng), int(off), probs.data_ptr(), out.data_ptr(),
                                      _lib.stream_of(xq)), "ob_decattn_fwd")
        ctx.meta = (heads, float(p), xkv is None, e, Lk, sq, skv, koff, voff)
        ctx.save_for_backward(xq, xkv if xkv is not None else xq, probs, out)
        return out

    @staticmethod
    def backward(ctx, dout):
        # the library's backward overwrites probs with dS' (ob_decattn_bwd consumes it)
        if getattr(ctx, "consumed", False):
            raise RuntimeError("decoder attention: backward ran twice on one forward "
                               "(retain_graph); its saved probabilities were consumed")
        ctx.consumed = True
        heads, p, self_mode, e, Lk, sq, skv, koff, voff = ctx.meta
        xq, xkv, probs, out = ctx.saved_tensors
        dout = dout.contiguous()
        B, Lq, _ = xq.shape
        dh = e // heads
        lib = _lib.load()
        dxq = torch.empty_like(xq)
        if self_mode:
            src, dsrc, dxkv = xq, dxq, None
        else:
            src = xkv
            dxkv = torch.empty_like(xkv)
            dsrc = dxkv
        base, dbase = src.data_ptr(), dsrc.data_ptr()
        _lib.check(lib.ob_decattn_bwd(dout.data_ptr(), out.data_ptr(), xq.data_ptr(), sq, base + 4 * koff, skv,
                                      base + 4 * voff, skv, B, heads, Lq, Lk, dh, p,
                                      probs.data_ptr(), dxq.data_ptr(), sq, dbase + 4 * koff, skv,
                                      dbase + 4 * voff, skv, _lib.stream_of(dout)),
                   "ob_decattn_bwd")
        return dxq, dxkv, None, None, None, None, None, None


def dec_attention(xq: torch.Tensor, xkv, heads: int, kmask, causal: bool, p: float,
                  training: bool) -> torch.Tensor:
    """ctx [B, Lq, e] of the decoder attention (module docstring); ``xkv`` None = self-
    attention on the packed ``xq = [q | k | v]``. ``kmask`` bool [B, Lk] (True = masked)."""
    p = p if training else 0.0
    rng, off = (None, 0)
    if p > 0:
        from .fused import _rng

        rng, off = _rng(xq.device)
    return _DecAttnFn.apply(xq, xkv, heads, kmask, causal, p, rng, off)
