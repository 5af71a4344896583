"""GPU parity of the fused clip_grad_norm_ + AdamW tail (ob_adamw_clip_step) against torch
(reference train.py:116-118, 259: clip 5.0, AdamW betas (0.9, 0.98), wd 1e-2, eps 1e-8).
Reference: torch.optim.AdamW(foreach=False) after torch.nn.utils.clip_grad_norm_ on CPU
fp32. Bars: params / exp_avg / exp_avg_sq max|err| <= 2e-6 * max|ref| + 2e-8 per tensor
(2e-8 ~ 1e-5 of the summed learning rates: the device lr is fp32, torch's a double),
global norm rel <= 1e-5; a parameter without a gradient is untouched."""
import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = [(1,), (144,), (576, 144), (5004, 144), (4097,), (3, 31)]


def _make(seed):
    g = torch.Generator().manual_seed(seed)
    ps = [torch.randn(s, generator=g) * 0.1 for s in SHAPES]
    grads = [[torch.randn(s, generator=g) * sc for s in SHAPES] for sc in (0.05, 2.0, 0.5)]
    return ps, grads


@pytest.mark.parametrize("max_norm", [5.0, 0.0])
def test_fused_adamw_matches_torch(gpu, max_norm):
    from onebit_asr.optim import FusedAdamW
    from onebit_asr.train_step import WarmupCosine

    ps, grads = _make(0)
    ref = [torch.nn.Parameter(p.clone()) for p in ps]
    opt_ref = torch.optim.AdamW(ref, lr=5e-4, betas=(0.9, 0.98), weight_decay=1e-2, foreach=False)
    sch_ref = WarmupCosine(opt_ref, 2, 10)
    dev = [torch.nn.Parameter(p.clone().to(gpu)) for p in ps]
    opt = FusedAdamW(dev, lr=5e-4, max_norm=max_norm)
    sch = WarmupCosine(opt, 2, 10)
    for step_grads in grads:
        norms = []
        for p, g in zip(ref, step_grads):
            p.grad = g.clone()
        if max_norm > 0:
            norms.append(torch.nn.utils.clip_grad_norm_(ref, max_norm).item())
        opt_ref.step()
        sch_ref.step()
        for p, g in zip(dev, step_grads):
            p.grad = g.to(gpu)
        opt.step()
        sch.step()
        if max_norm > 0:
            assert abs(opt.total_norm.item() - norms[0]) <= 1e-5 * norms[0]
    for i, (a, b) in enumerate(zip(dev, ref)):
        st = opt_ref.state[b]
        for x, y in ((a.detach().cpu(), b.detach()), (opt.exp_avg[i].cpu(), st["exp_avg"]),
                     (opt.exp_avg_sq[i].cpu(), st["exp_avg_sq"])):
            err = (x - y).abs().max().item()
            assert err <= 2e-6 * y.abs().max().item() + 2e-8, (i, err)
    assert opt.step_t.item() == 3.0


def test_fused_adamw_skips_param_without_grad(gpu):
    from onebit_asr.optim import FusedAdamW

    a = torch.nn.Parameter(torch.ones(10, device=gpu))
    b = torch.nn.Parameter(torch.ones(10, device=gpu))
    opt = FusedAdamW([a, b], lr=1e-2)
    a.grad = torch.full((10,), 0.5, device=gpu)
    opt.step()
    assert torch.equal(b.detach(), torch.ones(10, device=gpu))
    assert (a.detach() < 1).all()


def test_fused_adamw_in_graph(gpu):
    """Captured once, replayed: same result as eager steps (lr changes between replays)."""
    from onebit_asr.optim import FusedAdamW

    ps, grads = _make(1)
    eager = [torch.nn.Parameter(p.clone().to(gpu)) for p in ps]
    graphed = [torch.nn.Parameter(p.clone().to(gpu)) for p in ps]
    oe, og = FusedAdamW(eager), FusedAdamW(graphed)
    static = [g.to(gpu) for g in grads[0]]
    for p, g in zip(graphed, static):
        p.grad = g
    og.step()  # plan + table outside capture
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        og.step()
    for p, g in zip(eager, static):
        p.grad = g
    oe.step()
    for k, step_grads in enumerate(grads[1:]):
        lr = 1e-3 * (k + 1)
        for o in (oe, og):
            o.lr.fill_(lr)
        for s, g in zip(static, step_grads):
            s.copy_(g.to(gpu))
        graph.replay()
        oe.step()
    for a, b in zip(eager, graphed):
        assert torch.equal(a.detach(), b.detach())
