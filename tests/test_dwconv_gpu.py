"""GPU parity of the conv-module depthwise Conv1d HIP kernel against torch's fp32 conv1d on
CPU (the op is full precision in the reference, conformer.py:147). Bar: max|err| <= 1e-5 *
max|ref| + 1e-6 for y, dx, dw, db; deterministic."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B,C,T,K", [(2, 8, 37, 31), (32, 144, 249, 31), (1, 4, 600, 31),
                                     (3, 5, 7, 31), (2, 6, 50, 3), (2, 6, 50, 1), (1, 2, 300, 63)])
def test_dwconv_matches_torch(gpu, B, C, T, K):
    from onebit_asr.conv import depthwise_conv1d

    g = torch.Generator().manual_seed(B * 1000 + C * 10 + T + K)
    conv = torch.nn.Conv1d(C, C, K, padding=K // 2, groups=C)
    with torch.no_grad():
        conv.weight.copy_(torch.randn(conv.weight.shape, generator=g) * 0.2)
        conv.bias.copy_(torch.randn(C, generator=g))
    x = torch.randn(B, C, T, generator=g)
    dy = torch.randn(B, C, T, generator=g)
    xr = x.clone().requires_grad_()
    ref = conv(xr)
    ref.backward(dy)
    convg = torch.nn.Conv1d(C, C, K, padding=K // 2, groups=C).to(gpu)
    convg.load_state_dict(conv.state_dict())
    xg = x.to(gpu).requires_grad_()
    y = depthwise_conv1d(xg, convg)
    y.backward(dy.to(gpu))

    def close(a, b):
        a = a.detach().cpu().double()
        b = b.detach().double()
        err = (a - b).abs().max().item()
        assert err <= 1e-5 * b.abs().max().item() + 1e-6, err

    close(y, ref)
    close(xg.grad, xr.grad)
    close(convg.weight.grad, conv.weight.grad)
    close(convg.bias.grad, conv.bias.grad)
    # deterministic backward
    w1 = convg.weight.grad.clone()
    convg.zero_grad()
    depthwise_conv1d(xg, convg).backward(dy.to(gpu))
    assert torch.equal(w1, convg.weight.grad)
