"""HIP LayerNorm (csrc/layernorm.hip) vs a float64 torch reference of nn.LayerNorm:
y, dx max|err| <= 1e-5 * max|ref| + 1e-6; dgamma, dbeta rel-L2 <= 1e-5; deterministic."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("rows,d", [(1, 1), (7, 64), (23904, 144), (333, 144), (50, 256),
                                    (3, 500), (1000, 17)])
def test_layernorm_fwd_bwd(gpu, rows, d):
    from onebit_asr.layernorm import layer_norm

    g = torch.Generator(device=gpu).manual_seed(rows + d)
    x = (torch.randn(rows, d, device=gpu, generator=g) * 3 + 1).requires_grad_(True)
    w = (torch.randn(d, device=gpu, generator=g) * 0.5 + 1).requires_grad_(True)
    b = torch.randn(d, device=gpu, generator=g).requires_grad_(True)
    dy = torch.randn(rows, d, device=gpu, generator=g)
    y = layer_norm(x, w, b, 1e-5)
    y.backward(dy)
    xd, wd, bd = (t.detach().double().requires_grad_(True) for t in (x, w, b))
    yr = torch.nn.functional.layer_norm(xd, (d,), wd, bd, 1e-5)
    yr.backward(dy.double())

    def close(a, r):
        assert (a.double() - r).abs().max().item() <= 1e-5 * r.abs().max().item() + 1e-6

    close(y.detach(), yr.detach())
    close(x.grad, xd.grad)
    for a, r in ((w.grad, wd.grad), (b.grad, bd.grad)):
        rel = (a.double() - r).norm() / r.norm().clamp_min(1e-30)
        assert rel.item() <= 1e-5, rel.item()
    # deterministic
    gw1 = w.grad.clone()
    w.grad = None
    x.grad = None
    layer_norm(x, w, b, 1e-5).backward(dy)
    assert torch.equal(w.grad, gw1)


def test_layernorm_module_uses_hip(gpu):
    from onebit_asr.conformer import LayerNorm

    m = LayerNorm(144).to(gpu)
    x = torch.randn(4, 9, 144, device=gpu, requires_grad=True)
    y = m(x)
    assert y.grad_fn is not None and "LayerNormFn" in type(y.grad_fn).__name__


def _dropout_step(gpu, gscale: bool, monkeypatch):
    """One training forward+backward of the cfg1 model with dropout 0.1 and padded
    utterances; every fused dropout stream reset so both runs draw the same masks."""
    from _steputil import StepRunner, build

    from onebit_asr import fused, layernorm
    from onebit_asr.data import CFG1, synthetic_batch

    monkeypatch.setattr(layernorm, "_GSCALE", gscale)
    fused._STATE.pop(torch.device(gpu), None)
    model = build(CFG1, gpu, dropout=0.1).train()
    batch = synthetic_batch([734, 349], [27, 12], seed=3, device=gpu)
    run = StepRunner(model, CFG1["enc_layers"], batch, [1, 0], stacked=True)
    torch.manual_seed(11)
    return run.eager()


def test_ln_grad_scale_handoff_bit_exact(gpu, monkeypatch):
    """The residual tails' dropout/pad/scale backward formed by the next LN's backward
    (ob_layernorm_bwd_ex, layernorm.GradScale) equals the separate ob_drop_scale_bwd pass
    bit for bit: loss, parts and every parameter gradient, dropout 0.1, padded rows."""
    l0, p0, g0 = _dropout_step(gpu, False, monkeypatch)
    l1, p1, g1 = _dropout_step(gpu, True, monkeypatch)
    assert torch.equal(l0, l1) and torch.equal(p0, p1)
    for k in g0:
        assert (g0[k] is None) == (g1[k] is None), k
        if g0[k] is not None:
            assert torch.equal(g0[k], g1[k]), k


def test_layernorm_bwd_ex_matches_drop_scale(gpu):
    """ob_layernorm_bwd_ex's dy2 == ob_drop_scale_bwd(dx) element for element (rscale 0.5,
    p 0.1, lens), and its dx == ob_layernorm_bwd_res's."""
    from onebit_asr import _lib

    lib = _lib.load()
    g = torch.Generator(device=gpu).manual_seed(5)
    B, T, d = 3, 37, 144
    rows = B * T
    x, dy, dres = (torch.randn(rows, d, device=gpu, generator=g) for _ in range(3))
    w, b = torch.randn(d, device=gpu), torch.randn(d, device=gpu)
    mean = x.mean(1)
    rstd = 1.0 / torch.sqrt(x.var(1, unbiased=False) + 1e-5)
    lens = torch.tensor([37, 20, 1], dtype=torch.int32, device=gpu)
    rng = torch.tensor([77, 5], dtype=torch.int64, device=gpu)
    wsb = lib.ob_layernorm_bwd_workspace(rows, d)
    ws = torch.empty(wsb, dtype=torch.uint8, device=gpu)
    s = _lib.stream_of(x)
    dx0, dw0, db0 = torch.empty_like(x), torch.empty(d, device=gpu), torch.empty(d, device=gpu)
    assert lib.ob_layernorm_bwd_res(dy.data_ptr(), x.data_ptr(), w.data_ptr(), mean.data_ptr(),
                                    rstd.data_ptr(), rows, d, dres.data_ptr(), dx0.data_ptr(),
                                    dw0.data_ptr(), db0.data_ptr(), ws.data_ptr(), wsb, s) == 0
    ref = torch.empty_like(x)
    assert lib.ob_drop_scale_bwd(dx0.data_ptr(), rows, d, 0.5, 0.1, rng.data_ptr(), 9,
                                 lens.data_ptr(), T, ref.data_ptr(), s) == 0
    dx1, dw1, db1 = torch.empty_like(x), torch.empty(d, device=gpu), torch.empty(d, device=gpu)
    dy2 = torch.empty_like(x)
    assert lib.ob_layernorm_bwd_ex(dy.data_ptr(), x.data_ptr(), w.data_ptr(), mean.data_ptr(),
                                   rstd.data_ptr(), rows, d, dres.data_ptr(), dx1.data_ptr(),
                                   dw1.data_ptr(), db1.data_ptr(), ws.data_ptr(), wsb,
                                   dy2.data_ptr(), 0.5, 0.1, rng.data_ptr(), 9, lens.data_ptr(),
                                   T, s) == 0
    torch.cuda.synchronize()
    assert torch.equal(dx0, dx1) and torch.equal(dw0, dw1) and torch.equal(db0, db1)
    assert torch.equal(dy2, ref)
    assert (dy2.view(B, T, d)[1, 20:] == 0).all()
