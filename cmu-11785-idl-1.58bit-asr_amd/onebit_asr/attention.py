"""Fused relative-position attention core of MHSA on the HIP library.

Reference: onebit_asr/conformer.py:115-127 (between MHSA's projections and out_proj):
``((q+u) k^T + rel_shift((q+v) p^T)) / sqrt(d)``, padding masked to -inf, softmax,
``nan_to_num``, dropout, ``A v``. ``rel_pos_attention`` computes exactly that from the
projection outputs in their natural [B, T, H*d] layout and returns the context in the
layout out_proj consumes, with one forward kernel and one backward kernel (+ a small
reduction); see csrc/relattn.hip. Gradients flow to q, k, v, pos, pos_bias_u, pos_bias_v.
By default the forward saves the softmax probabilities as MFMA-fragment tiles and the
backward reads them. The flash-style backward (``set_backward_mode("flash")`` or
``OB_ATTN_BWD=flash``; T <= 256 and d_head <= 36) saves only per-row softmax statistics, the
dropout keep bits and a few rel_shift rows, and recomputes the probabilities on chip; it is
slower at Conformer-S, hence opt-in.

Dropout uses the kernels' counter-based hash of (seed, counter + offset): the device state
and per-call host offsets are the fused BitLinear call sites' (fused._rng), whose counter
``fused.advance_step`` moves once per step, so a captured step draws fresh masks on every
replay without a per-call device update (two launches per call before). The mask is not
torch's RNG stream (no reference-visible quantity depends on it).
"""
from __future__ import annotations

import os
from typing import Dict, Tuple

import torch

from . import _lib

__all__ = ["rel_pos_attention", "fused_attention_supported", "dropout_mask", "probs_dense",
           "set_backward_mode"]

# device -> (rng tensor, offset) of the latest call with dropout (tests read the mask back)
LAST_RNG: Dict[torch.device, Tuple[torch.Tensor, int]] = {}


def fused_attention_supported(q: torch.Tensor, d_head: int) -> bool:
    if os.environ.get("OB_ATTN", "") == "torch":
        return False
    return (q.is_cuda and q.dtype == torch.float32 and 1 <= q.size(1) <= 512
            and d_head in (16, 32, 36, 64))


class _RelAttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, pos, u, vb, lens, n_heads, p_drop, rng, rng_off):
        bt, t, c = q.shape
        P = pos.size(0)
        d = c // n_heads
        out = torch.empty_like(q)
        need = any(ctx.needs_input_grad[:6])
        lib = _lib.load()
        saved = (torch.empty((lib.ob_relattn_saved_elems(bt, t, n_heads, d),),
                             dtype=torch.float32, device=q.device) if need else None)
        _lib.check(
            lib.ob_relattn_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), pos.data_ptr(),
                               u.data_ptr(), vb.data_ptr(), lens.data_ptr(), bt, P, t, n_heads, d,
                               p_drop, _lib.ptr(rng), rng_off, _lib.ptr(saved), None,
                               out.data_ptr(), _lib.stream_of(q)),
            "ob_relattn_fwd",
        )
        ctx.meta = (n_heads, p_drop, rng_off)
        if need:
            ctx.save_for_backward(q, k, v, pos, u, vb, lens, saved, rng, out)
        return out

    @staticmethod
    def backward(ctx, g):
        q, k, v, pos, u, vb, lens, saved, rng, out = ctx.saved_tensors
        n_heads, p_drop, rng_off = ctx.meta
        g = g.contiguous()
        bt, t, c = q.shape
        P = pos.size(0)
        d = c // n_heads
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        dpos = torch.empty_like(pos)
        du, dvb = torch.empty_like(u), torch.empty_like(vb)
        lib = _lib.load()
        wsb = lib.ob_relattn_bwd_workspace(bt, t, n_heads, d)
        ws = torch.empty((wsb,), dtype=torch.uint8, device=q.device)
        _lib.check(
            lib.ob_relattn_bwd(g.data_ptr(), out.data_ptr(), q.data_ptr(), k.data_ptr(), v.data_ptr(),
                               pos.data_ptr(), u.data_ptr(), vb.data_ptr(), lens.data_ptr(), bt,
                               P, t, n_heads, d, p_drop, _lib.ptr(rng), rng_off, saved.data_ptr(),
                               saved.numel(), dq.data_ptr(), dk.data_ptr(), dv.data_ptr(), dpos.data_ptr(),
                               du.data_ptr(), dvb.data_ptr(), ws.data_ptr(), wsb,
                               _lib.stream_of(g)),
            "ob_relattn_bwd",
        )
        return dq, dk, dv, dpos, du, dvb, None, None, None, None, None


def set_backward_mode(mode: str) -> str:
    """'probs' (default) or 'flash': the process-wide attention backward (csrc/relattn.hip).
    Returns the previous mode. A backward whose forward ran under the other mode raises."""
    if mode not in ("probs", "flash"):
        raise ValueError(f"mode must be 'probs' or 'flash', got {mode!r}")
    prev = _lib.load().ob_relattn_set_bwd_mode(1 if mode == "flash" else 0)
    return "flash" if prev == 1 else "probs"


def rel_pos_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, pos: torch.Tensor,
                      pos_bias_u: torch.Tensor, pos_bias_v: torch.Tensor, lens: torch.Tensor,
                      n_heads: int, dropout_p: float = 0.0) -> torch.Tensor:
    """q, k, v [Bt, T, H*d]; pos [P, T, H*d] (Bt = P * B, batch row b uses pass b // B);
    pos_bias_u/v [H, d]; lens int [Bt] valid frames. Returns the context [Bt, T, H*d]."""
    q, k, v, pos = (x.contiguous() for x in (q, k, v, pos))
    lens = lens.to(torch.int32).contiguous()
    rng, off = None, 0
    if dropout_p > 0:
        from .fused import _rng

        rng, off = _rng(q.device)  # a distinct offset per call; the backward reuses it
        LAST_RNG[q.device] = (rng, off)
    return _RelAttnFn.apply(q, k, v, pos, pos_bias_u.contiguous(), pos_bias_v.contiguous(), lens,
                            n_heads, float(dropout_p), rng, off)


def probs_dense(probs: torch.Tensor, bt: int, n_heads: int, t: int) -> torch.Tensor:
    """The forward's fragment-tiled probabilities (csrc/relattn.hip) as [Bt, H, T, T]."""
    nt = (t + 15) // 16
    x = probs.view(bt * n_heads, nt, nt, 4, 16, 4)  # [bh][a][t][g][r][e]
    x = x.permute(0, 1, 4, 2, 3, 5).reshape(bt, n_heads, 16 * nt, 16 * nt)
    return x[:, :, :t, :t]


def dropout_mask(shape, p: float, rng: torch.Tensor, rng_off: int = 0) -> torch.Tensor:
    """The keep-mask (uint8, 1 = kept) the kernels draw for a tensor of ``shape`` whose last
    dim is the row the mask index runs along (attention: [.., T, T]; a flat BitLinear /
    LayerNorm tensor: (n,)) (tests)."""
    n = 1
    for s in shape:
        n *= s
    out = torch.empty(n, dtype=torch.uint8, device=rng.device)
    lib = _lib.load()
    _lib.check(lib.ob_relattn_dropout_mask(n, int(shape[-1]), float(p), rng.data_ptr(),
                                           int(rng_off), out.data_ptr(), _lib.stream_of(rng)),
               "ob_relattn_dropout_mask")
    return out.view(*shape)
