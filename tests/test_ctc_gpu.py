"""GPU parity of the HIP CTC loss (device-side lengths) against torch's nn.CTCLoss on CPU
(reference losses.py:41-47: blank 3, zero_infinity, 'mean'). The reference value is torch's
CTC in float64 (torch's fp32 CTC itself is off by ~1e-5 of max|grad| over T=249 steps).
Bars: loss rel <= 1e-5, logits-gradient (through log_softmax) max|err| <= max(2e-5 *
max|ref|, 2x torch-fp32's own error) + 1e-7; deterministic."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _case(B, T, V, in_lens, tg_lens, seed, repeat=False):
    g = torch.Generator().manual_seed(seed)
    logits = torch.randn(B, T, V, generator=g) * 2
    S = max(max(tg_lens), 1)
    tg = torch.zeros(B, S, dtype=torch.long)
    for b, L in enumerate(tg_lens):
        if L:
            vals = torch.randint(4, V, (L,), generator=g)
            if repeat:
                vals[1::2] = vals[0::2][: len(vals[1::2])]  # adjacent repeats
            tg[b, :L] = vals
    return logits, tg, torch.tensor(in_lens), torch.tensor(tg_lens)


@pytest.mark.parametrize("case", [
    dict(B=2, T=50, V=30, in_lens=[50, 37], tg_lens=[10, 4], seed=0),
    dict(B=3, T=40, V=20, in_lens=[40, 40, 30], tg_lens=[6, 8, 5], seed=1, repeat=True),
    dict(B=2, T=12, V=10, in_lens=[12, 5], tg_lens=[4, 9], seed=2),           # sample 1 infeasible
    dict(B=2, T=20, V=10, in_lens=[20, 20], tg_lens=[0, 3], seed=3),          # empty target
    dict(B=4, T=249, V=5004, in_lens=[249, 249, 200, 100], tg_lens=[40, 27, 12, 40], seed=4),
])
def test_ctc_matches_torch(gpu, case):
    from onebit_asr.ctc import ctc_loss_mean

    logits, tg, il, tl = _case(**case)
    lr = logits.clone().double().requires_grad_()
    ref = torch.nn.CTCLoss(blank=3, zero_infinity=True)(
        F.log_softmax(lr, -1).transpose(0, 1), tg, il, tl)
    ref.backward()
    l32 = logits.clone().requires_grad_()
    torch.nn.CTCLoss(blank=3, zero_infinity=True)(
        F.log_softmax(l32, -1).transpose(0, 1), tg, il, tl).backward()
    err32 = (l32.grad.double() - lr.grad).abs().max().item()
    lg = logits.to(gpu).requires_grad_()
    out = ctc_loss_mean(F.log_softmax(lg, -1), tg.to(gpu), il.to(gpu), tl.to(gpu), 3)
    out.backward()
    assert abs(out.item() - ref.item()) <= 1e-5 * abs(ref.item()) + 1e-6, (out.item(), ref.item())
    err = (lg.grad.cpu().double() - lr.grad).abs().max().item()
    # the fp32 log_softmax input already limits both fp32 CTCs (case4: ~1e-3 of max|grad|)
    assert err <= max(2e-5 * lr.grad.abs().max().item(), 2 * err32) + 1e-7, (err, err32)
    g1 = lg.grad.clone()
    lg.grad = None
    ctc_loss_mean(F.log_softmax(lg, -1), tg.to(gpu), il.to(gpu), tl.to(gpu), 3).backward()
    assert torch.equal(g1, lg.grad)


def test_ctc_groups_equal_per_group_calls(gpu):
    """ctc_loss_mean_groups over 3 stacked groups == three ctc_loss_mean calls (losses and
    log-prob gradients), incl. a ragged input length and an infeasible sample (zero_infinity)."""
    from onebit_asr.ctc import ctc_loss_mean, ctc_loss_mean_groups

    torch.manual_seed(3)
    G, B, T, V, S = 3, 4, 30, 12, 6
    lp = torch.randn(G * B, T, V, device=gpu).log_softmax(-1).requires_grad_(True)
    tg = torch.randint(1, V, (G * B, S), device=gpu)
    il = torch.tensor([30, 25, 30, 4] * G, device=gpu)  # 4 frames < 6 labels: infeasible
    tl = torch.tensor([6, 5, 3, 6] * G, device=gpu)
    w = torch.tensor([0.7, -1.3, 2.0], device=gpu)
    loss = ctc_loss_mean_groups(lp, tg, il, tl, 0, G)
    (loss * w).sum().backward()
    g_grp = lp.grad.clone()
    lp.grad = None
    ref = torch.stack([ctc_loss_mean(lp[g * B:(g + 1) * B], tg[g * B:(g + 1) * B],
                                     il[g * B:(g + 1) * B], tl[g * B:(g + 1) * B], 0)
                       for g in range(G)])
    (ref * w).sum().backward()
    assert torch.allclose(loss, ref, rtol=1e-6, atol=0)
    assert torch.allclose(g_grp, lp.grad, rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("case", [
    dict(B=2, T=50, V=30, in_lens=[50, 37], tg_lens=[10, 4], seed=0),
    dict(B=3, T=40, V=20, in_lens=[40, 40, 30], tg_lens=[6, 8, 5], seed=1, repeat=True),
    dict(B=2, T=12, V=10, in_lens=[12, 5], tg_lens=[4, 9], seed=2),           # sample 1 infeasible
    dict(B=2, T=20, V=10, in_lens=[20, 20], tg_lens=[0, 3], seed=3),          # empty target
    dict(B=3, T=33, V=13, in_lens=[33, 0, 20], tg_lens=[5, 2, 7], seed=6),    # zero-length input
    dict(B=4, T=249, V=5004, in_lens=[249, 249, 200, 100], tg_lens=[40, 27, 12, 40], seed=4),
])
def test_ctc_from_logits_matches_torch(gpu, case):
    """ctc_loss_logits_groups (lse pass + compact label log-probs + d/dlogits, no log_softmax
    tensor) vs float64 torch log_softmax + nn.CTCLoss: the same bars as the log-prob path;
    bitwise repeatable."""
    from onebit_asr.ctc import ctc_loss_logits_groups

    logits, tg, il, tl = _case(**case)
    lr = logits.clone().double().requires_grad_()
    ref = torch.nn.CTCLoss(blank=3, zero_infinity=True)(
        F.log_softmax(lr, -1).transpose(0, 1), tg, il, tl)
    ref.backward()
    l32 = logits.clone().requires_grad_()
    torch.nn.CTCLoss(blank=3, zero_infinity=True)(
        F.log_softmax(l32, -1).transpose(0, 1), tg, il, tl).backward()
    err32 = (l32.grad.double() - lr.grad).abs().max().item()
    lg = logits.to(gpu).requires_grad_()
    out = ctc_loss_logits_groups(lg, tg.to(gpu), il.to(gpu), tl.to(gpu), 3, 1)[0]
    out.backward()
    assert abs(out.item() - ref.item()) <= 1e-5 * abs(ref.item()) + 1e-6, (out.item(), ref.item())
    err = (lg.grad.cpu().double() - lr.grad).abs().max().item()
    assert err <= max(2e-5 * lr.grad.abs().max().item(), 2 * err32) + 1e-7, (err, err32)
    g1 = lg.grad.clone()
    lg.grad = None
    ctc_loss_logits_groups(lg, tg.to(gpu), il.to(gpu), tl.to(gpu), 3, 1)[0].backward()
    assert torch.equal(g1, lg.grad)


def test_ctc_from_logits_groups(gpu):
    """Grouped losses == per-group log-prob-path losses (weighted backward), with a ragged
    length and an infeasible sample (targets never contain blank: torch's CTC contract)."""
    from onebit_asr.ctc import ctc_loss_logits_groups, ctc_loss_mean

    torch.manual_seed(5)
    G, B, T, V, S = 3, 4, 30, 12, 6
    x = torch.randn(G * B, T, V, device=gpu).requires_grad_(True)
    tg = torch.randint(1, V, (G * B, S), device=gpu)
    il = torch.tensor([30, 25, 30, 4] * G, device=gpu)
    tl = torch.tensor([6, 5, 3, 6] * G, device=gpu)
    w = torch.tensor([0.7, -1.3, 2.0], device=gpu)
    loss = ctc_loss_logits_groups(x, tg, il, tl, 0, G)
    (loss * w).sum().backward()
    g_grp = x.grad.clone()
    x.grad = None
    lp = F.log_softmax(x, -1)
    ref = torch.stack([ctc_loss_mean(lp[g * B:(g + 1) * B], tg[g * B:(g + 1) * B],
                                     il[g * B:(g + 1) * B], tl[g * B:(g + 1) * B], 0)
                       for g in range(G)])
    (ref * w).sum().backward()
    assert torch.allclose(loss, ref, rtol=1e-5, atol=1e-6), (loss, ref)
    # (torch's log_softmax + its backward's sum term vs the fused lse pass: ~1e-5 of max)
    assert (g_grp - x.grad).abs().max().item() <= 2e-5 * x.grad.abs().max().item() + 1e-7
