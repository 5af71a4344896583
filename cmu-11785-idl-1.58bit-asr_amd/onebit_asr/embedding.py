"""Decoder token embedding with a deterministic, graph-safe HIP backward.

Reference: onebit_asr/conformer.py:279-299 (``nn.Embedding(vocab, d, padding_idx=pad)`` on
the BOS-prefixed targets). The forward is torch's gather; the backward is
``ob_embedding_bwd`` (fixed-order segmented sum, zero row at ``padding_idx``) instead of
torch's sort-based kernel sequence.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _lib

__all__ = ["embedding"]


class _EmbeddingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, idx, weight, padding_idx):
        ctx.save_for_backward(idx)
        ctx.meta = (weight.shape[0], weight.shape[1], padding_idx)
        return F.embedding(idx, weight, padding_idx)

    @staticmethod
    def backward(ctx, g):
        (idx,) = ctx.saved_tensors
        v, c, pad = ctx.meta
        g = g.contiguous()
        flat = idx.reshape(-1).contiguous()
        dw = torch.empty((v, c), dtype=torch.float32, device=g.device)
        lib = _lib.load()
        _lib.check(lib.ob_embedding_bwd(flat.data_ptr(), flat.numel(), g.data_ptr(), c, v,
                                        -1 if pad is None else pad, dw.data_ptr(),
                                        _lib.stream_of(g)), "ob_embedding_bwd")
        return None, dw, None


def embedding(idx: torch.Tensor, weight: torch.Tensor, padding_idx=None) -> torch.Tensor:
    if weight.is_cuda and weight.dtype == torch.float32 and idx.dtype == torch.int64 \
            and weight.shape[1] <= 1024 and torch.is_grad_enabled() and weight.requires_grad:
        return _EmbeddingFn.apply(idx, weight, padding_idx)
    return F.embedding(idx, weight, padding_idx)
