"""The registered operator torch.ops.onebit.bitlinear equals QuantizedLinear (same kernels)
in forward and every gradient, passes torch.library.opcheck's schema / fake / autograd
registration checks, and runs under torch.compile."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("bits", [2, 1])
def test_op_matches_module(gpu, bits):
    from onebit_asr.ops import bitlinear
    from onebit_asr.quant import QuantizedLinear

    torch.manual_seed(bits)
    lin = QuantizedLinear(144, 576).to(gpu)
    with torch.no_grad():
        lin.bias.uniform_(-0.1, 0.1)
    x = torch.randn(4, 37, 144, device=gpu)
    g = torch.randn(4, 37, 576, device=gpu)
    outs = []
    for use_op in (False, True):
        lin.zero_grad()
        xx = x.clone().requires_grad_(True)
        y = bitlinear(xx, lin.weight, lin.alpha, lin.bias, bits) if use_op else lin(xx, bits)
        (y * g).sum().backward()
        outs.append([y.detach(), xx.grad, lin.weight.grad.clone(), lin.alpha.grad.clone(),
                     lin.bias.grad.clone()])
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_opcheck_and_compile(gpu):
    import onebit_asr.ops  # noqa: F401

    torch.manual_seed(0)
    x = torch.randn(3, 64, device=gpu, requires_grad=True)
    w = torch.randn(48, 64, device=gpu, requires_grad=True) * 0.1
    w = w.detach().requires_grad_(True)
    a = torch.tensor(0.05, device=gpu, requires_grad=True)
    b = torch.randn(48, device=gpu, requires_grad=True)
    torch.library.opcheck(torch.ops.onebit.bitlinear.default, (x, w, a, b, 2),
                          test_utils=("test_schema", "test_faketensor",
                                      "test_autograd_registration"))
    f = torch.compile(lambda t: torch.ops.onebit.bitlinear(t, w, a, b, 2).sum(), fullgraph=True)
    y = f(x)
    ref = torch.ops.onebit.bitlinear(x, w, a, b, 2).sum()
    assert torch.equal(y, ref)
