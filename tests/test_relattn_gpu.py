"""Fused relative-position attention (ob_relattn_*) against the reference op sequence
(conformer.py:115-127: (q+u)k^T + rel_shift((q+v)p^T), /sqrt(d), padding -> -inf,
softmax, nan_to_num, dropout, A v) evaluated in float64 on the CPU with autograd.

Bars: ctx max|err| <= 1e-5 * max|ref| + 1e-6; probs max|err| <= 1e-6; every gradient
(q, k, v, pos, pos_bias_u, pos_bias_v) max|err| <= 1e-4 * max|ref| + 1e-6. Dropout is
checked with the kernels' own keep-mask (ob_relattn_dropout_mask) applied in the
reference. Edge cases: T = 1, an utterance of length 0 (fully masked rows -> 0), lengths
off by one around the 64-row forward tiles and the 32-query backward chunks, stacked passes
(P > 1), T <= 256 with d <= 36 (the flash-style backward that recomputes the probabilities)
and T > 256 or d = 64 (the backward that reads stored probabilities).
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

CASES = [  # (Bt, P, T, H, d, lens)
    (2, 1, 1, 4, 16, [1, 0]),
    (4, 2, 17, 2, 16, [17, 5, 0, 17]),
    (6, 3, 65, 4, 36, [65, 64, 63, 1, 65, 33]),
    (3, 3, 182, 4, 16, [182, 100, 182]),
    (4, 2, 249, 4, 36, [249, 249, 200, 1]),
    (2, 1, 300, 4, 36, [300, 150]),
    (2, 1, 512, 2, 64, [512, 511]),
    (3, 3, 33, 4, 16, [33, 32, 1]),        # two 32-query chunks, the second one row long
    (2, 1, 256, 2, 32, [256, 200]),        # the largest flash-style shape, d 32
    (4, 2, 240, 4, 36, [240, 0, 97, 239]),  # Tp = 240: the last chunk half outside Tp
]


def _ref(q, k, v, pos, u, vb, lens, H, keep=None, p=0.0):
    """Reference ops in float64 (conformer.py:115-127 with rel_shift :97-103, the oracle's
    gather restatement -- not the product's own rel_shift)."""
    from oracle.conformer_oracle import _rel_shift_gather as rel_shift

    bt, t, c = q.shape
    d = c // H
    P = pos.size(0)
    heads = lambda x: x.view(x.size(0), t, H, d).transpose(1, 2)  # noqa: E731
    qh, kh, vh = heads(q), heads(k), heads(v)
    ph = heads(pos)                                        # [P, H, T, d]
    ph = ph.repeat_interleave(bt // P, dim=0)              # pass of each batch row
    ac = torch.matmul(qh + u.view(1, H, 1, d), kh.transpose(-2, -1))
    bd = rel_shift(torch.matmul(qh + vb.view(1, H, 1, d), ph.transpose(-2, -1)))
    s = (ac + bd) / math.sqrt(d)
    frames = torch.arange(t)
    km = frames[None, :] < lens[:, None]
    mask = km[:, :, None] & km[:, None, :]
    s = s.masked_fill(~mask[:, None], float("-inf"))
    a = torch.nan_to_num(torch.softmax(s, dim=-1), nan=0.0)
    probs = a
    if keep is not None:
        a = a * keep.to(a.dtype) / (1.0 - p)
    ctx = torch.matmul(a, vh).transpose(1, 2).reshape(bt, t, c)
    return ctx, probs


def _inputs(bt, P, t, H, d, seed):
    g = torch.Generator().manual_seed(seed)
    c = H * d
    mk = lambda *s: torch.randn(*s, generator=g)  # noqa: E731
    return mk(bt, t, c), mk(bt, t, c), mk(bt, t, c), mk(P, t, c), mk(H, d) * 0.1, mk(H, d) * 0.1


def _close(got, ref, rel, atol, what):
    err = (got.double().cpu() - ref).abs().max().item() if ref.numel() else 0.0
    bound = rel * (ref.abs().max().item() if ref.numel() else 0.0) + atol
    assert err <= bound, f"{what}: max err {err:.3e} > {bound:.3e}"


@pytest.mark.parametrize("bwd", ["probs", "flash"])
@pytest.mark.parametrize("bt,P,t,H,d,lens", CASES)
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_relattn_matches_reference(gpu, bt, P, t, H, d, lens, p, bwd):
    """bwd: the backward that reads the stored probabilities (default) or the flash-style one
    (set_backward_mode("flash"); T <= 256, d <= 36 -- other shapes take the probability path)."""
    from onebit_asr import attention as at

    prev = at.set_backward_mode(bwd)
    try:
        _check_case(gpu, bt, P, t, H, d, lens, p)
    finally:
        at.set_backward_mode(prev)


def _check_case(gpu, bt, P, t, H, d, lens, p):
    from onebit_asr import attention as at


    q, k, v, pos, u, vb = _inputs(bt, P, t, H, d, seed=bt * 1000 + t)
    lens_t = torch.tensor(lens)
    dev = [x.to(gpu).requires_grad_() for x in (q, k, v, pos, u, vb)]
    ctx = at.rel_pos_attention(*dev, lens_t.to(gpu), H, dropout_p=p)
    keep = None
    if p > 0:
        rng, off = at.LAST_RNG[torch.device(gpu)]  # the state + offset this call used
        keep = at.dropout_mask((bt, H, t, t), p, rng, off).cpu()
    gout = torch.randn(bt, t, H * d, generator=torch.Generator().manual_seed(7))
    ctx.backward(gout.to(gpu))

    ref_in = [x.double().requires_grad_() for x in (q, k, v, pos, u, vb)]
    rctx, _ = _ref(*ref_in, lens_t, H, keep=keep, p=p)
    rctx.backward(gout.double())
    _close(ctx.detach(), rctx.detach(), 1e-5, 1e-6, "ctx")
    for name, a, b in zip(("dq", "dk", "dv", "dpos", "du", "dvb"), dev, ref_in):
        _close(a.grad, b.grad, 1e-4, 1e-6, name)


def test_relattn_probs_and_determinism(gpu):
    from onebit_asr import _lib

    bt, P, t, H, d = 4, 2, 249, 4, 36
    q, k, v, pos, u, vb = (x.to(gpu) for x in _inputs(bt, P, t, H, d, seed=3))
    lens = torch.tensor([249, 120, 0, 249], dtype=torch.int32)
    lib = _lib.load()
    from onebit_asr.attention import probs_dense

    outs = []
    for _ in range(2):
        probs = torch.full((lib.ob_relattn_probs_elems(bt, t, H),), float("nan"), device=gpu)
        ctx = torch.empty_like(q)
        _lib.check(lib.ob_relattn_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), pos.data_ptr(),
                                      u.data_ptr(), vb.data_ptr(), lens.to(gpu).data_ptr(), bt, P,
                                      t, H, d, 0.0, None, 0, None, probs.data_ptr(),
                                      ctx.data_ptr(), _lib.stream_of(q)), "fwd")
        # every padding slot of the fragment tiles is written (zero)
        assert torch.isfinite(probs).all().item()
        outs.append((probs_dense(probs, bt, H, t).clone(), ctx.clone()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    _, rprobs = _ref(*(x.double().cpu() for x in (q, k, v, pos, u, vb)), lens.long(), H)
    _close(outs[0][0], rprobs, 0.0, 1e-6, "probs")
    assert torch.count_nonzero(outs[0][0][2]).item() == 0  # length-0 utterance


def test_relattn_dropout_mask_rate(gpu):
    from onebit_asr import attention as at

    rng = torch.tensor([12345, 7], dtype=torch.int64, device=gpu)
    m = at.dropout_mask((4, 4, 249, 249), 0.1, rng).float()
    assert abs(m.mean().item() - 0.9) < 2e-3
    rng2 = torch.tensor([12345, 8], dtype=torch.int64, device=gpu)
    m2 = at.dropout_mask((4, 4, 249, 249), 0.1, rng2).float()
    assert (m != m2).float().mean().item() > 0.1  # the counter changes the mask
    # the host offset is added to the device counter: (7, +1) draws (8, +0)'s mask
    assert torch.equal(at.dropout_mask((4, 4, 249, 249), 0.1, rng, 1).float(), m2)


def test_mhsa_fused_matches_torch_path(gpu, monkeypatch):
    """MHSA.forward with the fused core == the reference op sequence (OB_ATTN=torch)."""
    from onebit_asr.conformer import MHSA

    torch.manual_seed(0)
    m = MHSA(144, 4, 0.0).to(gpu)
    x = torch.randn(3, 120, 144, device=gpu)
    km = torch.arange(120, device=gpu)[None] < torch.tensor([120, 80, 0], device=gpu)[:, None]
    mask = km[:, :, None] & km[:, None, :]
    pe = torch.randn(1, 120, 144, device=gpu)
    outs = {}
    for mode in ("fused", "torch"):
        monkeypatch.setenv("OB_ATTN", "" if mode == "fused" else "torch")
        xi = x.clone().requires_grad_()
        m.zero_grad(set_to_none=True)
        y = m(xi, mask, 2, pe)
        y.backward(torch.ones_like(y))
        outs[mode] = (y.detach(), xi.grad.detach(), m.pos_bias_u.grad.detach(),
                      m.q_proj.weight.grad.detach())
    for a, b in zip(outs["fused"], outs["torch"]):
        err = (a - b).abs().max().item()
        assert err <= 1e-4 * b.abs().max().item() + 1e-6, err


def test_backward_refuses_saved_state_of_the_other_mode(gpu):
    """The backward mode is process-wide: a backward whose forward saved its state
    under the other mode is refused (OB_ERR_SHAPE from the saved-size check), not run on a
    buffer of the wrong layout."""
    from onebit_asr import attention as at

    bt, P, t, H, d = 2, 1, 249, 4, 36
    dev = [x.to(gpu).requires_grad_() for x in _inputs(bt, P, t, H, d, seed=11)]
    lens = torch.tensor([249, 100], device=gpu)
    prev = at.set_backward_mode("probs")
    try:
        ctx = at.rel_pos_attention(*dev, lens, H)
        at.set_backward_mode("flash")
        with pytest.raises(RuntimeError, match="ob_relattn_bwd"):
            ctx.backward(torch.ones_like(ctx))
    finally:
        at.set_backward_mode(prev)
