"""GPU parity of the BitLinear HIP kernels (through the C ABI) against the CPU oracle.

Bars (written here, per the task): quantizer codes, STE masks, the hand-derived KATs and
determinism are bit-exact; float outputs are compared with a float64 oracle:
  Y, dX       : max|err| <= 1e-5 * max|ref| + 1e-6       (fp32 sum-order only)
  G = dY^T X  : rel-L2(dW) <= 1e-5
  dalpha      : |err| <= 1e-5 * sum|G * term| + 1e-6      (condition-aware)
  db          : max|err| <= 1e-5 * max|ref| + 1e-6
"""
import json

import numpy as np
import pytest
import torch

from oracle import quant_oracle as qo

pytestmark = pytest.mark.gpu

SHAPES = [  # (M, K, N)
    (1, 3, 2), (5, 7, 37), (16, 16, 16), (100, 100, 37), (364, 64, 256), (364, 256, 64),
    (249, 144, 144), (7968, 144, 144), (7968, 144, 576), (7968, 576, 144), (33, 13, 130),
    # the K = 576 byte-image launches (all 144 columns of a row tile in one block) with
    # ragged row counts: forward at N = 288 and at K = 560 (padded to 576), dX of K = 144
    (65, 576, 288), (130, 560, 144), (65, 144, 576),
]


def _ql_module(W, alpha_raw_value, bias, device):
    from onebit_asr.quant import QuantizedLinear

    n, k = W.shape
    m = QuantizedLinear(k, n, bias=bias is not None).to(device)
    with torch.no_grad():
        m.weight.copy_(torch.as_tensor(W))
        m.alpha.fill_(alpha_raw_value)
        if bias is not None:
            m.bias.copy_(torch.as_tensor(bias))
    return m


def _oracle_grads(X, W, alpha_raw, dY, bits):
    """float64 reference for (dX, dW, dalpha_raw, db)."""
    a = qo.np_effective_alpha(alpha_raw)
    w_hat = (a * qo.np_quant_q(W, alpha_raw, bits)).astype(np.float64)
    dY64 = dY.astype(np.float64)
    dX = dY64 @ w_hat
    G = dY64.T @ X.astype(np.float64)
    wa = (W / a).astype(np.float32)
    ind = (np.abs(wa) <= 1).astype(np.float64)
    term = qo.np_term(wa, bits).astype(np.float64)
    chain = float(np.sign(np.float32(alpha_raw)))
    dalpha = float((G * term).sum()) * chain
    scale = float(np.abs(G * term).sum())
    return dX, G * ind, dalpha, scale, dY64.sum(0)


def _close(got, ref, rtol=1e-5, atol=1e-6):
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    err = np.abs(got - ref).max() if ref.size else 0.0
    bound = rtol * (np.abs(ref).max() if ref.size else 0.0) + atol
    assert err <= bound, f"max err {err:.3e} > {bound:.3e}"


def test_kat_layer_exact(gpu, golden_dir):
    kat = json.loads((golden_dir / "quant_kat.json").read_text())
    L = kat["layer_2x3"]
    for bits in (1, 2):
        exp = L[f"bits{bits}"]
        m = _ql_module(np.array(L["W"], np.float32), -0.5, np.array(L["bias"], np.float32), gpu)
        x = torch.tensor(L["X"], device=gpu, requires_grad=True)
        y = m(x, bits)
        assert torch.equal(y.cpu(), torch.tensor(exp["Y"]))
        y.backward(torch.tensor(L["dY"], device=gpu))
        assert torch.equal(x.grad.cpu(), torch.tensor(exp["dX"]))
        assert torch.equal(m.weight.grad.cpu(), torch.tensor(exp["dW"]))
        assert m.alpha.grad.item() == pytest.approx(-exp["dalpha_eff"], abs=1e-6)
        assert torch.equal(m.bias.grad.cpu(), torch.tensor(exp["db"]))


def test_threshold_codes_exact(gpu, golden_dir):
    """Weights sitting exactly on |W/a| in {0, 0.5, 1} and one ulp either side."""
    from onebit_asr.quant import pack_codes

    a = np.float32(0.0731)  # raw alpha; a_eff = |a| + 1e-8
    ae = qo.np_effective_alpha(a)
    base = np.array([0.0, 0.5, 1.0, 0.25, 0.75, 2.0], np.float32)
    vals = []
    for v in base:
        w = np.float32(v) * ae
        for d in (-2, -1, 0, 1, 2):
            x = w
            for _ in range(abs(d)):
                x = np.nextafter(x, np.float32(np.inf if d > 0 else -np.inf), dtype=np.float32)
            vals += [x, -x]
    W = np.array(vals, np.float32)
    W = np.resize(W, (7, 19)).astype(np.float32)
    for bits in (1, 2):
        codes, codes_t = pack_codes(torch.from_numpy(W).to(gpu), torch.tensor(a, device=gpu), bits)
        c_ref, ct_ref = qo.c_codes(W, a, bits)
        assert np.array_equal(codes.cpu().numpy().view(np.uint32), c_ref)
        assert np.array_equal(codes_t.cpu().numpy().view(np.uint32), ct_ref)


@pytest.mark.parametrize("bits", [1, 2])
@pytest.mark.parametrize("shape", SHAPES)
def test_layer_parity(gpu, bits, shape):
    M, K, N = shape
    g = torch.Generator().manual_seed(M * 7919 + K * 31 + N + bits)
    W, alpha, _ = qo.ref_layer_init(K, N, g)
    W = W.numpy()
    alpha = float(alpha) * (-1 if (M % 2) else 1)  # exercise the sign chain
    bias = (torch.randn(N, generator=g) * 0.1).numpy()
    X = torch.randn(M, K, generator=g).numpy()
    dY = torch.randn(M, N, generator=g).numpy()

    m = _ql_module(W, alpha, bias, gpu)
    from onebit_asr.quant import pack_codes

    codes, codes_t = pack_codes(m.weight, m.alpha, bits)
    c_ref, ct_ref = qo.c_codes(W, alpha, bits)
    assert np.array_equal(codes.cpu().numpy().view(np.uint32), c_ref)
    assert np.array_equal(codes_t.cpu().numpy().view(np.uint32), ct_ref)

    x = torch.from_numpy(X).to(gpu).requires_grad_()
    y = m(x, bits)
    _close(y.detach().cpu().numpy(), qo.np_bitlinear_fwd(X, W, alpha, bias, bits))
    y.backward(torch.from_numpy(dY).to(gpu))
    dX, dW, dalpha, scale, db = _oracle_grads(X, W, alpha, dY, bits)
    _close(x.grad.cpu().numpy(), dX)
    gw = m.weight.grad.cpu().numpy().astype(np.float64)
    if np.abs(dW).max() > 0:
        rel = np.linalg.norm(gw - dW) / np.linalg.norm(dW)
        assert rel <= 1e-5, rel
    # STE mask is exact: masked entries are exactly zero
    wa = (W / qo.np_effective_alpha(alpha)).astype(np.float32)
    assert np.all(gw[np.abs(wa) > 1] == 0)
    assert abs(m.alpha.grad.item() - dalpha) <= 1e-5 * scale + 1e-6
    _close(m.bias.grad.cpu().numpy(), db)


def test_backward_deterministic(gpu):
    g = torch.Generator().manual_seed(5)
    W, alpha, _ = qo.ref_layer_init(144, 576, g)
    m = _ql_module(W.numpy(), float(alpha), np.zeros(576, np.float32), gpu)
    x = torch.randn(7968, 144, generator=g).to(gpu).requires_grad_()
    dy = torch.randn(7968, 576, generator=g).to(gpu)
    outs = []
    for _ in range(2):
        m.zero_grad(set_to_none=True)
        x.grad = None
        m(x, 2).backward(dy)
        outs.append([t.detach().clone() for t in (x.grad, m.weight.grad, m.alpha.grad, m.bias.grad)])
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_no_bias_and_3d_input(gpu):
    g = torch.Generator().manual_seed(11)
    W, alpha, _ = qo.ref_layer_init(64, 48, g)
    m = _ql_module(W.numpy(), float(alpha), None, gpu)
    X = torch.randn(2, 31, 64, generator=g)
    y = m(X.to(gpu), 1)
    assert y.shape == (2, 31, 48)
    _close(y.detach().cpu().numpy().reshape(-1, 48),
           qo.np_bitlinear_fwd(X.reshape(-1, 64).numpy(), W.numpy(), float(alpha), None, 1))


def test_empty_rows(gpu):
    g = torch.Generator().manual_seed(2)
    W, alpha, _ = qo.ref_layer_init(32, 16, g)
    m = _ql_module(W.numpy(), float(alpha), np.ones(16, np.float32), gpu)
    x = torch.zeros(0, 32, device=gpu, requires_grad=True)
    y = m(x, 2)
    assert y.shape == (0, 16)
    y.sum().backward()
    assert torch.count_nonzero(m.weight.grad) == 0 and m.alpha.grad.item() == 0.0
    assert torch.count_nonzero(m.bias.grad) == 0


@pytest.mark.parametrize("bits", [1, 2, 32])
def test_quantize_weight_api(gpu, bits):
    from onebit_asr.quant import quantize_weight

    g = torch.Generator().manual_seed(bits)
    W, alpha, _ = qo.ref_layer_init(100, 37, g)
    gr = torch.randn(37, 100, generator=g)
    Wg = W.to(gpu).requires_grad_()
    ag = torch.tensor(float(alpha), device=gpu, requires_grad=True)
    out = quantize_weight(Wg, ag, bits)
    Wc = W.clone().requires_grad_()
    ac = torch.tensor(float(alpha), requires_grad=True)
    ref = qo.ref_quantize_weight(Wc, ac, bits)
    assert torch.equal(out.detach().cpu(), ref.detach())
    out.backward(gr.to(gpu))
    ref.backward(gr)
    assert torch.equal(Wg.grad.cpu(), Wc.grad)
    assert ag.grad.item() == pytest.approx(ac.grad.item(), rel=1e-5, abs=1e-5)


def test_errors(gpu):
    from onebit_asr.quant import QuantizedLinear

    m = QuantizedLinear(8, 4).to(gpu)
    with pytest.raises(ValueError, match=r"bitwidth must be one of \{1,2,32\}"):
        m(torch.zeros(2, 8, device=gpu), 3)
    with pytest.raises(RuntimeError, match="ROCm device"):
        QuantizedLinear(8, 4)(torch.zeros(2, 8), 2)
    y32 = m(torch.ones(2, 8, device=gpu), 32)
    assert torch.allclose(y32, torch.nn.functional.linear(torch.ones(2, 8, device=gpu), m.weight, m.bias))


def test_alpha_zero_chain(gpu):
    """alpha = 0: a = 1e-8, every |W/a| > 1 -> dW = 0; d|alpha|/dalpha = sgn(0) = 0."""
    g = torch.Generator().manual_seed(3)
    W, _, _ = qo.ref_layer_init(16, 16, g)
    m = _ql_module(W.numpy(), 0.0, np.zeros(16, np.float32), gpu)
    x = torch.randn(8, 16, device=gpu)
    m(x, 2).sum().backward()
    assert torch.count_nonzero(m.weight.grad) == 0
    assert m.alpha.grad.item() == 0.0


def test_pack_group_matches_oracle(gpu):
    """ob_quant_pack_group (one launch for every layer and bitwidth) == the oracle's codes,
    for layers of ragged shapes (K, N not multiples of 16, a 1x1 layer), and the layers'
    forwards then use those codes without packing again."""
    import torch.nn as nn
    from onebit_asr.quant import PackGroup, QuantizedLinear

    torch.manual_seed(5)
    shapes = [(144, 576), (576, 144), (7, 37), (1, 1), (33, 130), (144, 144)]
    mod = nn.ModuleList([QuantizedLinear(k, n) for k, n in shapes]).to(gpu)
    with torch.no_grad():
        mod[1].alpha.fill_(-0.03)  # negative raw alpha: |alpha| + 1e-8 is what quantizes
    grp = PackGroup(mod, bits=(2, 1))
    grp.run()
    for m, per in zip(mod, grp.codes):
        W = m.weight.detach().cpu().numpy()
        a = np.float32(m.alpha.item())
        for bits, (c, ct) in per.items():
            c_ref, ct_ref = qo.np_codes(W, a, bits)
            assert np.array_equal(c.cpu().numpy().view(np.uint32), c_ref)
            assert np.array_equal(ct.cpu().numpy().view(np.uint32), ct_ref)
            got = m._codes(bits)
            assert got[0].data_ptr() == c.data_ptr()  # cache hit: no per-layer pack
    # after an in-place update the cache is stale until the next run()
    with torch.no_grad():
        mod[0].weight.mul_(-1.0)
    assert mod[0]._codes(2)[0].data_ptr() != grp.codes[0][2][0].data_ptr()
    grp.run()
    c_ref, _ = qo.np_codes(mod[0].weight.detach().cpu().numpy(), np.float32(mod[0].alpha.item()), 2)
    assert np.array_equal(grp.codes[0][2][0].cpu().numpy().view(np.uint32), c_ref)


@pytest.mark.parametrize("bits", [1, 2])
@pytest.mark.parametrize("shape", [(7, 144, 576), (130, 576, 144), (64, 16, 20), (1, 4, 4),
                                   (0, 144, 144)])
def test_signacc_forward_matches_oracle(gpu, bits, shape):
    """The VALU sign-accumulate forward (ob_bitlinear_fwd_signacc, the north-star inner-product
    A/B partner of the MFMA kernel) vs the float64 oracle at the module path's bar; ragged
    M / N (tile edges), K % 16 != 0 (a partial code word), no rows; misaligned K refused."""
    from onebit_asr import _lib
    from onebit_asr.quant import pack_codes

    M, K, N = shape
    g = torch.Generator().manual_seed(M * 131 + K * 7 + N + bits)
    W, alpha, _ = qo.ref_layer_init(K, N, g)
    bias = torch.randn(N, generator=g) * 0.1
    X = torch.randn(M, K, generator=g)
    lib = _lib.load()
    w, a = W.to(gpu), alpha.reshape(()).to(gpu)
    codes, _ = pack_codes(w, a, bits)
    x, b = X.to(gpu), bias.to(gpu)
    y = torch.full((M, N), float("nan"), device=gpu)
    _lib.check(lib.ob_bitlinear_fwd_signacc(x.data_ptr() if M else None, M, K, codes.data_ptr(),
                                            a.data_ptr(), 1, b.data_ptr(), N,
                                            y.data_ptr() if M else None, _lib.stream_of(y)),
               "ob_bitlinear_fwd_signacc")
    torch.cuda.synchronize()
    if M:
        _close(y.cpu().numpy(), qo.np_bitlinear_fwd(X.numpy(), W.numpy(), float(alpha), bias.numpy(),
                                                     bits))
    if K % 4 == 0 and M:
        assert lib.ob_bitlinear_fwd_signacc(x.data_ptr(), M, K - 1, codes.data_ptr(), a.data_ptr(), 1,
                                            None, N, y.data_ptr(), None) == -2  # K % 4 != 0
