"""GPU parity of the fused decoder losses (csrc/seqloss.hip, onebit_asr/seqloss.py) against
the reference's torch expressions in float64: label-smoothed attention CE with its
scalar-mean quirk (losses.py:22-35) per pass and KL(stopgrad softmax(teacher) || softmax(
student)) over non-pad positions (losses.py:50-59), combined as train.py:82-111 does
(pass 0 = teacher). Bars: losses rel <= 2e-6; logits gradient max|err| <= 2e-6 * max|ref|
(fp32 row reductions over V <= 5004 terms); bit-identical on a repeat (fixed-order sums)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

PAD = 0


def _ref(logits, t_out, t_pad, P, ls):
    """train.py:82-111's combination of losses.py:22-35 and :50-59, float64."""
    x = logits.double()
    bsz = x.size(0) // P
    v = x.size(-1)
    logp = F.log_softmax(x, -1).view(P, bsz, -1, v)
    off = ls / (v - 1)
    tgt_logp = logp.gather(-1, t_out.unsqueeze(0).expand(P, -1, -1).unsqueeze(-1)).squeeze(-1)
    per_pos = -(off * logp.sum(-1) + (1.0 - ls - off) * tgt_logp)
    m = (t_out != PAD).double()
    l_att = per_pos.reshape(P, -1).mean(1) * m.sum() / m.sum().clamp_min(1.0)
    p_t = F.softmax(x[:bsz].detach(), -1)
    kl = F.kl_div(logp[1:], p_t.unsqueeze(0).expand(P - 1, -1, -1, -1), reduction="none").sum(-1)
    keep = (~t_pad).double()
    l_kl = (kl * keep).sum(dim=(1, 2)) / keep.sum().clamp_min(1.0)
    return l_att, l_kl


def _case(P, B, U, V, seed, all_pad=False):
    g = torch.Generator().manual_seed(seed)
    logits = torch.randn(P * B, U, V, generator=g) * 3
    lens = torch.randint(1, U + 1, (B,), generator=g)
    t_out = torch.randint(1, V, (B, U), generator=g)
    t_inp = torch.randint(1, V, (B, U), generator=g)
    for b in range(B):
        t_out[b, lens[b]:] = PAD
        t_inp[b, lens[b] + 1:] = PAD
    if all_pad:
        t_out[:] = PAD
        t_inp[:] = PAD
    return logits, t_out, t_inp == PAD


@pytest.mark.parametrize("case", [
    dict(P=3, B=4, U=41, V=5004, seed=0),   # Conformer-S vocabulary
    dict(P=3, B=3, U=7, V=64, seed=1),
    dict(P=2, B=2, U=5, V=8, seed=2),
    dict(P=1, B=2, U=3, V=12, seed=3),      # teacher only: no KL
    dict(P=3, B=2, U=4, V=32, seed=4, all_pad=True),  # every position padded
])
def test_att_kl_matches_reference(gpu, case):
    from onebit_asr.seqloss import att_kl_losses

    P, ls = case["P"], 0.1
    logits, t_out, t_pad = _case(**case)
    lr = logits.clone().double().requires_grad_()
    ra, rk = _ref(lr, t_out, t_pad, P, ls)
    ga = torch.linspace(0.5, 1.5, P, dtype=torch.float64)
    gk = torch.linspace(0.7, 1.3, max(P - 1, 1), dtype=torch.float64)[: P - 1]
    ((ra * ga).sum() + (rk * gk).sum()).backward()

    lg = logits.to(gpu).requires_grad_()
    a, k = att_kl_losses(lg, t_out.to(gpu), t_pad.to(gpu), P, PAD, ls)
    assert a.shape == (P,) and k.shape == (P - 1,)
    torch.testing.assert_close(a.double().cpu(), ra.detach(), rtol=2e-6, atol=1e-7)
    torch.testing.assert_close(k.double().cpu(), rk.detach(), rtol=2e-6, atol=1e-7)
    ((a * ga.float().to(gpu)).sum() + (k * gk.float().to(gpu)).sum()).backward()
    gref = lr.grad
    err = (lg.grad.double().cpu() - gref).abs().max().item()
    assert err <= 2e-6 * gref.abs().max().item() + 1e-12, err
    # deterministic: the same bits on a repeat
    a2, k2 = att_kl_losses(lg, t_out.to(gpu), t_pad.to(gpu), P, PAD, ls)
    assert torch.equal(a2, a) and torch.equal(k2, k)


def test_att_kl_rejects_bad_shapes(gpu):
    from onebit_asr import _lib
    from onebit_asr.seqloss import att_kl_losses, att_kl_supported

    x = torch.randn(6, 3, 10, device=gpu)  # V % 4 != 0: not supported -> torch path
    assert not att_kl_supported(x, 0.1)
    assert not att_kl_supported(torch.randn(6, 3, 8, device=gpu), 0.0)
    with pytest.raises(Exception):
        att_kl_losses(torch.randn(6, 3, 8, device=gpu), torch.ones(2, 4, dtype=torch.long,
                                                                     device=gpu),
                      torch.zeros(2, 4, dtype=torch.bool, device=gpu), 3, PAD, 0.1)
    lib = _lib.load()
    assert lib.ob_att_kl_loss_fwd(0, 0, 0, 3, 4, 10, 0, 0.1, 0, 0, 0, 0, 0) != 0


def test_loss_combine_equals_torch_expression(gpu):
    """ob_loss_combine_fwd / _bwd (train_step._LossCombine) against the torch expression it
    replaces (train.py:95-111 in the stacked form): loss, the eight parts and the gradients of
    l_att, l_ctc, l_kl bit for bit (same rounding sequence), for a unit and a non-unit seed."""
    from onebit_asr.train_step import _LossCombine

    g = torch.Generator().manual_seed(5)
    gam, lam1, lam2 = 0.2, 0.5, 1.0
    for seed in (1.0, 0.37):
        base = [torch.rand(n, generator=g) * 5 for n in (3, 3, 2)]
        la, lc, lk = (t.to(gpu).requires_grad_() for t in base)
        loss, parts = _LossCombine.apply(la, lc, lk, gam, lam1, lam2)
        loss.backward(torch.tensor(seed, device=gpu))
        ta, tc, tk = (t.to(gpu).requires_grad_() for t in base)
        li = (1 - gam) * ta + gam * tc
        tl = li[0] + lam1 * (li[1] + li[2]) + lam2 * (tk[0] + tk[1])
        tp = torch.stack([li[0], li[1], li[2], tk[0], tk[1], tc[0], tc[1], tc[2]])
        tl.backward(torch.tensor(seed, device=gpu))
        assert torch.equal(loss, tl.detach()) and torch.equal(parts, tp.detach())
        for a, b in ((la, ta), (lc, tc), (lk, tk)):
            assert torch.equal(a.grad, b.grad), (a.grad, b.grad)
