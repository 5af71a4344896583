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
