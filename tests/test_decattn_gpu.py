"""The decoder's HIP attention core (ob_decattn_*, onebit_asr/decattn.py) against the
reference op sequence of torch's multi_head_attention_forward as the decoder uses it
(conformer.py:275-299: (q k^T) * (1/sqrt(dh)) + mask, softmax, dropout, @ v), evaluated in
float64 on the CPU with autograd.

Bars: ctx max|err| <= 1e-5 * max|ref| + 1e-6; probs (|stored|) max|err| <= 1e-6; dq, dk, dv
(written into the packed projection gradients) max|err| <= 1e-4 * max|ref| + 1e-6. Dropout is
checked with the kernel's own keep bits (the sign of the stored probabilities) applied in the
reference. Cases: self-attention (packed q|k|v, causal + key padding), cross-attention
(q, packed k|v, memory padding), Lq = 1, Lk = 256, dh = 16 / 36 / 64. Whole decoder: the HIP
path equals the additive-mask path it replaces (dropout 0).
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

CASES = [  # (B, H, Lq, Lk, dh, self_mode)
    (3, 4, 41, 41, 36, True),
    (3, 4, 41, 250, 36, False),
    (2, 2, 1, 1, 16, True),
    (2, 4, 7, 256, 16, False),
    (2, 2, 64, 64, 64, True),
    (5, 4, 13, 97, 36, False),
    (2, 4, 100, 130, 36, False),  # dq in 48-query tiles, the last one ragged
    (2, 2, 100, 100, 32, True),
]


def _inputs(B, H, Lq, Lk, dh, self_mode, dev, seed=0):
    g = torch.Generator().manual_seed(seed)
    e = H * dh
    if self_mode:
        xq = torch.randn(B, Lq, 3 * e, generator=g)
        xkv = None
        lens = torch.randint(1, Lq + 1, (B,), generator=g)
        kmask = torch.arange(Lq)[None, :] >= lens[:, None]
    else:
        xq = torch.randn(B, Lq, e, generator=g)
        xkv = torch.randn(B, Lk, 2 * e, generator=g)
        lens = torch.randint(1, Lk + 1, (B,), generator=g)
        lens[0] = Lk
        kmask = torch.arange(Lk)[None, :] >= lens[:, None]
    dout = torch.randn(B, Lq, e, generator=g)
    return xq.to(dev), (xkv.to(dev) if xkv is not None else None), kmask.to(dev), dout.to(dev)


def _ref(xq, xkv, kmask, H, causal, keep=None, p=0.0):
    """float64 reference (the decoder's additive-mask formulation)."""
    B, Lq, wq = xq.shape
    if xkv is None:
        e = wq // 3
        q, k, v = xq.split(e, dim=-1)
    else:
        e = wq
        q = xq
        k, v = xkv.split(e, dim=-1)
    Lk = k.shape[1]
    dh = e // H
    heads = lambda t, L: t.reshape(B, L, H, dh).transpose(1, 2)  # noqa: E731
    qh, kh, vh = heads(q, Lq), heads(k, Lk), heads(v, Lk)
    bias = torch.zeros(B, 1, Lq, Lk, dtype=xq.dtype)
    bias = bias.masked_fill(kmask.view(B, 1, 1, Lk), float("-inf"))
    if causal:
        fut = torch.ones(Lq, Lk).triu(1).bool()
        bias = bias.masked_fill(fut.view(1, 1, Lq, Lk), float("-inf"))
    att = torch.matmul(qh, kh.transpose(-2, -1)) * (1.0 / math.sqrt(dh)) + bias
    A = torch.softmax(att, dim=-1)
    Ad = A if keep is None else A * keep * (1.0 / (1.0 - p))
    ctx = torch.matmul(Ad, vh).transpose(1, 2).reshape(B, Lq, e)
    return ctx, A


def _close(got, ref, rel):
    err = (got.double().cpu() - ref).abs().max().item()
    bar = rel * ref.abs().max().item() + 1e-6
    assert err <= bar, (err, bar)


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_decattn_vs_reference(gpu, case, p):
    from onebit_asr import _lib
    from onebit_asr.decattn import _DecAttnFn

    B, H, Lq, Lk, dh, self_mode = case
    xq, xkv, kmask, dout = _inputs(B, H, Lq, Lk, dh, self_mode, gpu)
    assert _lib.load().ob_decattn_supported(Lq, Lk, dh) == 1
    rng = torch.tensor([1234, 7], dtype=torch.int64, device=gpu)
    xq_ = xq.clone().requires_grad_(True)
    xkv_ = xkv.clone().requires_grad_(True) if xkv is not None else None
    ctx = _DecAttnFn.apply(xq_, xkv_, H, kmask, self_mode, p, rng if p > 0 else None, 3)
    ctx.backward(dout)
    # the kernel's probabilities and keep bits: rerun the forward entry point directly
    lib = _lib.load()
    e = H * dh
    probs = torch.empty(B, H, Lq, Lk, device=gpu)
    ctx2 = torch.empty(B, Lq, e, device=gpu)
    if self_mode:
        src, sq, skv, ko, vo = xq, 3 * e, 3 * e, e, 2 * e
    else:
        src, sq, skv, ko, vo = xkv, e, 2 * e, 0, e
    _lib.check(lib.ob_decattn_fwd(xq.data_ptr(), sq, src.data_ptr() + 4 * ko, skv,
                                  src.data_ptr() + 4 * vo, skv, kmask.data_ptr(), int(self_mode),
                                  B, H, Lq, Lk, dh, p, rng.data_ptr() if p > 0 else None, 3,
                                  probs.data_ptr(), ctx2.data_ptr(), None), "fwd")
    torch.cuda.synchronize()
    assert torch.equal(ctx2, ctx.detach())  # deterministic
    keep = None if p == 0 else (~torch.signbit(probs)).double().cpu()
    if p > 0 and keep.numel() >= 1000:  # the mask really drops about p of the elements
        frac = 1.0 - keep.mean().item()
        assert abs(frac - p) < 0.05, frac
    rq = xq.double().cpu().requires_grad_(True)
    rkv = xkv.double().cpu().requires_grad_(True) if xkv is not None else None
    rctx, A = _ref(rq, rkv, kmask.cpu(), H, self_mode, keep, p)
    rctx.backward(dout.double().cpu())
    _close(ctx, rctx.detach(), 1e-5)
    _close(probs.abs(), A.detach(), 1e-6)
    _close(xq_.grad, rq.grad, 1e-4)
    if xkv is not None:
        _close(xkv_.grad, rkv.grad, 1e-4)


def test_decoder_hip_path_equals_additive_path(gpu):
    """TransformerDecoder.forward on the HIP core == the additive-mask torch path (dropout 0):
    outputs and every parameter gradient."""
    import onebit_asr.decattn as da
    from onebit_asr.conformer import TransformerDecoder

    torch.manual_seed(0)
    dec = TransformerDecoder(vocab_size=50, d_model=144, n_layers=2, n_heads=4, d_ff=256,
                             dropout=0.0, pad_id=0).to(gpu)
    B, tt, T = 4, 11, 37
    tgt = torch.randint(1, 50, (B, tt), device=gpu)
    pad = torch.zeros(B, tt, dtype=torch.bool, device=gpu)
    pad[1, 7:] = True
    pad[3, 2:] = True
    mem = torch.randn(B, T, 144, device=gpu)
    mmask = torch.ones(B, T, device=gpu)
    mmask[2, 20:] = 0
    outs, grads = [], []
    for on in (True, False):
        da._ON = on
        try:
            dec.zero_grad(set_to_none=True)
            m = mem.clone().requires_grad_(True)
            y = dec(tgt, m, mmask, pad)
            y.backward(torch.randn_like(y, generator=None) * 0 + torch.linspace(
                -1, 1, y.numel(), device=gpu).view_as(y))
            outs.append(y.detach())
            grads.append({n: p.grad.clone() for n, p in dec.named_parameters()
                          if p.grad is not None} | {"memory": m.grad.clone()})
        finally:
            da._ON = True
    scale = outs[1].abs().max().item()
    assert (outs[0] - outs[1]).abs().max().item() <= 1e-5 * scale
    assert grads[0].keys() == grads[1].keys()
    for n in grads[1]:
        ref = grads[1][n]
        err = (grads[0][n] - ref).abs().max().item()
        assert err <= 1e-4 * ref.abs().max().item() + 1e-6, (n, err)


def test_decattn_second_backward_refused(gpu):
    """The backward writes dS' over the saved probabilities (ob_decattn_bwd consumes them), so
    a second backward through the same forward (retain_graph) raises instead of reading dS'
    as P."""
    from onebit_asr.decattn import _DecAttnFn

    xq = torch.randn(2, 5, 3 * 64, device=gpu, requires_grad=True)
    ctx = _DecAttnFn.apply(xq, None, 4, None, True, 0.0, None, 0)
    ctx.sum().backward(retain_graph=True)
    with pytest.raises(RuntimeError, match="consumed"):
        ctx.sum().backward()
