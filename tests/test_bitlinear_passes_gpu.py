"""Stacked-pass BitLinear (ob_bitlinear_*_passes): P passes of one layer in one call each.

Checked two ways:
* against the single-pass entries run once per pass (the reference's three separate
  QuantizedLinear calls, quant.py:120-127) with autograd summing their gradients:
  Y and dX bit-identical (same kernel per pass), dW / db rel <= 1e-6 and dalpha
  <= 1e-6 * sum|G*term| (only the order of the cross-pass sum differs);
* against the float64 oracle: sum over passes of the per-pass oracle gradients, with the
  single-pass bars of test_bitlinear_gpu.py.
"""
import numpy as np
import pytest
import torch

from oracle import quant_oracle as qo

pytestmark = pytest.mark.gpu

CASES = [  # (M per pass, K, N, pass bits)
    (364, 64, 256, [2, 1, 1]),
    (364, 256, 64, [2, 1, 2]),
    (7968, 144, 576, [2, 1, 1]),
    (7968, 576, 144, [2, 1, 2]),
    (249, 144, 144, [2, 1, 1]),
    (33, 13, 130, [1, 2, 1]),
    (100, 100, 37, [2, 2]),
]


def _layer(K, N, seed, device):
    from onebit_asr.quant import QuantizedLinear

    torch.manual_seed(seed)
    m = QuantizedLinear(K, N).to(device)
    with torch.no_grad():
        m.bias.uniform_(-0.1, 0.1)
    return m


@pytest.mark.parametrize("M,K,N,bits", CASES)
def test_passes_match_separate_calls(gpu, M, K, N, bits):
    from onebit_asr.quant import PassBits

    P = len(bits)
    g = torch.Generator(device=gpu).manual_seed(M + K + N)
    x = torch.randn(P, M, K, device=gpu, generator=g)
    dy = torch.randn(P, M, N, device=gpu, generator=g)
    lay = _layer(K, N, 0, gpu)

    xs = x.clone().requires_grad_()
    ys = torch.cat([lay(xs[p], bits[p]) for p in range(P)])
    ys.backward(dy.reshape(P * M, N))
    ref = {k: p.grad.clone() for k, p in lay.named_parameters()}
    for p in lay.parameters():
        p.grad = None

    xp = x.clone().reshape(P * M, K).requires_grad_()
    pb = PassBits(torch.tensor(bits, dtype=torch.int32, device=gpu))
    yp = lay(xp, pb)
    yp.backward(dy.reshape(P * M, N))
    assert torch.equal(yp, ys)
    assert torch.equal(xp.grad, xs.grad.reshape(P * M, K))
    for k, p in lay.named_parameters():
        got, want = p.grad.double(), ref[k].double()
        if k == "alpha":
            continue
        rel = ((got - want).norm() / want.norm().clamp_min(1e-30)).item()
        assert rel <= 1e-6, (k, rel)

    # dalpha against the float64 oracle (condition-aware bar)
    W = lay.weight.detach().cpu().numpy()
    araw = float(lay.alpha.item())
    a = qo.np_effective_alpha(araw)
    wa = (W / a).astype(np.float32)
    X = x.cpu().numpy().astype(np.float64)
    DY = dy.cpu().numpy().astype(np.float64)
    dal = scale = 0.0
    for p in range(P):
        G = DY[p].T @ X[p]
        term = qo.np_term(wa, bits[p]).astype(np.float64)
        dal += float((G * term).sum())
        scale += float(np.abs(G * term).sum())
    dal *= float(np.sign(np.float32(araw)))
    assert abs(lay.alpha.grad.item() - dal) <= 1e-5 * scale + 1e-6


def test_passes_against_oracle(gpu):
    from onebit_asr.quant import PassBits

    M, K, N, bits = 364, 64, 256, [2, 1, 1]
    P = len(bits)
    lay = _layer(K, N, 3, gpu)
    rng = np.random.default_rng(7)
    X = rng.standard_normal((P, M, K)).astype(np.float32)
    DY = rng.standard_normal((P, M, N)).astype(np.float32)
    xp = torch.tensor(X.reshape(P * M, K), device=gpu, requires_grad=True)
    y = lay(xp, PassBits(torch.tensor(bits, dtype=torch.int32, device=gpu)))
    y.backward(torch.tensor(DY.reshape(P * M, N), device=gpu))
    W = lay.weight.detach().cpu().numpy()
    araw = float(lay.alpha.item())
    b = lay.bias.detach().cpu().numpy().astype(np.float64)
    a = qo.np_effective_alpha(araw)
    dW = np.zeros((N, K))
    db = np.zeros(N)
    for p in range(P):
        w_hat = (a * qo.np_quant_q(W, araw, bits[p])).astype(np.float64)
        y_ref = X[p].astype(np.float64) @ w_hat.T + b
        got = y[p * M:(p + 1) * M].detach().cpu().numpy()
        assert np.abs(got - y_ref).max() <= 1e-5 * np.abs(y_ref).max() + 1e-6
        dx_ref = DY[p].astype(np.float64) @ w_hat
        gx = xp.grad[p * M:(p + 1) * M].cpu().numpy()
        assert np.abs(gx - dx_ref).max() <= 1e-5 * np.abs(dx_ref).max() + 1e-6
        wa = (W / a).astype(np.float32)
        dW += (DY[p].astype(np.float64).T @ X[p].astype(np.float64)) * (np.abs(wa) <= 1)
        db += DY[p].astype(np.float64).sum(0)
    gw = lay.weight.grad.cpu().numpy().astype(np.float64)
    assert np.linalg.norm(gw - dW) <= 1e-5 * np.linalg.norm(dW)
    assert np.abs(lay.bias.grad.cpu().numpy() - db).max() <= 1e-5 * np.abs(db).max() + 1e-6


def test_passes_device_bits_change_without_host(gpu):
    """The pass bitwidths are read on device: rewriting the tensor changes the result."""
    from onebit_asr.quant import PassBits

    lay = _layer(144, 144, 5, gpu)
    x = torch.randn(3 * 50, 144, device=gpu)
    t = torch.tensor([2, 1, 2], dtype=torch.int32, device=gpu)
    y_a = lay(x, PassBits(t)).clone()
    t[2] = 1
    y_b = lay(x, PassBits(t))
    assert torch.equal(y_a[:100], y_b[:100])
    assert torch.equal(y_b[100:], lay(x[100:], 1))
    assert not torch.equal(y_a[100:], y_b[100:])
