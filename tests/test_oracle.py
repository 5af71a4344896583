"""CPU: pin the oracle against the hand-derived known answers, and the three oracle
restatements (numpy, C, torch fp32) against each other."""
import json

import numpy as np
import pytest
import torch

from oracle import quant_oracle as qo

F32 = np.float32


def _term(expr: str, wa: float) -> float:
    wa = F32(wa)
    return float({"0": F32(0), "1": F32(1), "-1": F32(-1), "-wa": -wa,
                  "-wa+1": (-wa) + F32(1), "-wa-1": (-wa) - F32(1)}[expr])


@pytest.fixture(scope="module")
def kat(golden_dir):
    return json.loads((golden_dir / "quant_kat.json").read_text())


@pytest.fixture(scope="module", autouse=True)
def _c_oracle_built():
    import subprocess
    from pathlib import Path

    subprocess.run(["make", "-s", "-C", str(Path(qo.__file__).parent)], check=True)


def test_threshold_kats_numpy_c_torch(kat):
    a = kat["alpha_eff"]
    rows = kat["thresholds"]["rows"]
    wa = np.array([r[0] for r in rows], F32)
    W = (wa * F32(a)).astype(F32)  # exact: a = 0.5
    assert np.array_equal((W / F32(a)).astype(F32), wa)
    for bits, col in ((1, 1), (2, 2)):
        want = np.array([r[col] for r in rows], F32)
        assert np.array_equal(qo.np_quant_q(W, a, bits, alpha_raw=False), want)
        assert np.array_equal(qo.c_quant_q(W, a, bits, alpha_raw=False).astype(F32), want)
        tq = qo.ref_quantize_weight(torch.from_numpy(W), torch.tensor(a), bits) / a
        assert np.array_equal(tq.numpy(), want)
    ind = np.array([r[3] for r in rows], F32)
    for bits, col in ((1, 4), (2, 5)):
        term = np.array([_term(r[col], r[0]) for r in rows], F32)
        g = np.ones_like(W)
        gw, _ = qo.np_ste_bwd(g, W, a, bits, alpha_raw=False)
        assert np.array_equal(gw, ind)
        assert np.array_equal(qo.np_term(wa, bits), term)
        # one-hot gradients isolate each element's term in the alpha gradient
        for i in range(len(rows)):
            gi = np.zeros_like(W)
            gi[i] = 1.0
            _, ga = qo.np_ste_bwd(gi, W, a, bits, alpha_raw=False)
            cw, c64, c32 = qo.c_ste_bwd(gi, W, a, bits, alpha_raw=False)
            assert ga == pytest.approx(float(term[i]), abs=0) and c32 == term[i]
        Wt = torch.from_numpy(W).requires_grad_()
        at = torch.tensor(a, requires_grad=True)
        qo.ref_quantize_weight(Wt, at, bits).sum().backward()
        assert np.array_equal(Wt.grad.numpy(), ind)
        assert at.grad.item() == pytest.approx(float(term.astype(np.float64).sum()), rel=1e-6)


@pytest.mark.parametrize("bits", [1, 2])
def test_layer_kat(kat, bits):
    L = kat["layer_2x3"]
    exp = L[f"bits{bits}"]
    W = np.array(L["W"], F32)
    X = np.array(L["X"], F32)
    b = np.array(L["bias"], F32)
    a = kat["alpha_eff"]
    assert np.array_equal(qo.np_quant_q(W, a, bits, alpha_raw=False), np.array(exp["Q"], F32))
    np.testing.assert_allclose(qo.np_bitlinear_fwd(X, W, a, b, bits, alpha_raw=False), exp["Y"], atol=1e-6)
    np.testing.assert_allclose(qo.c_bitlinear_fwd(X, W, a, b, bits, alpha_raw=False), exp["Y"], atol=1e-6)
    gw, ga = qo.np_ste_bwd(X, W, a, bits, alpha_raw=False)  # dW_hat = X when dY = I
    np.testing.assert_array_equal(gw, exp["dW"])
    assert ga == pytest.approx(exp["dalpha_eff"], abs=1e-6)
    # torch fp32 reference of the whole layer, raw alpha = -0.5 -> a = 0.5, sign chain -1
    x = torch.tensor(L["X"], requires_grad=True)
    Wt = torch.tensor(L["W"], requires_grad=True)
    al = torch.tensor(-0.5, requires_grad=True)
    bt = torch.tensor(L["bias"], requires_grad=True)
    y = qo.ref_quantized_linear(x, Wt, al, bt, bits)
    np.testing.assert_allclose(y.detach().numpy(), exp["Y"], atol=1e-6)
    y.backward(torch.tensor(L["dY"]))
    np.testing.assert_allclose(x.grad.numpy(), exp["dX"], atol=1e-6)
    np.testing.assert_allclose(Wt.grad.numpy(), exp["dW"], atol=1e-6)
    assert al.grad.item() == pytest.approx(-exp["dalpha_eff"], abs=1e-5)
    np.testing.assert_allclose(bt.grad.numpy(), exp["db"], atol=0)


@pytest.mark.parametrize("bits", [1, 2])
@pytest.mark.parametrize("shape", [(7, 5), (64, 256), (144, 576), (37, 100)])
def test_restatements_agree(bits, shape):
    g = torch.Generator().manual_seed(hash((bits,) + shape) & 0xFFFF)
    W, alpha, _ = qo.ref_layer_init(shape[1], shape[0], g)
    W = W.numpy()
    alpha = float(alpha)
    qn = qo.np_quant_q(W, alpha, bits)
    assert np.array_equal(qn, qo.c_quant_q(W, alpha, bits).astype(F32))
    cn, ctn = qo.np_codes(W, alpha, bits)
    cc, ctc = qo.c_codes(W, alpha, bits)
    assert np.array_equal(cn, cc) and np.array_equal(ctn, ctc)
    gr = torch.randn(shape, generator=g).numpy()
    gw_n, ga_n = qo.np_ste_bwd(gr, W, alpha, bits)
    gw_c, ga_c64, ga_c32 = qo.c_ste_bwd(gr, W, alpha, bits)
    assert np.array_equal(gw_n, gw_c)
    assert ga_n == pytest.approx(ga_c64, rel=1e-12, abs=1e-12)
    Wt = torch.from_numpy(W).requires_grad_()
    at = torch.tensor(alpha, requires_grad=True)
    out = qo.ref_quantize_weight(Wt, at.abs() + 1e-8, bits)
    np.testing.assert_array_equal(out.detach().numpy(),
                                  (qo.np_effective_alpha(alpha) * qn).astype(F32))
    out.backward(torch.from_numpy(gr))
    assert np.array_equal(Wt.grad.numpy(), gw_n)
    assert at.grad.item() == pytest.approx(ga_n, rel=1e-4, abs=1e-4)


def test_init_distribution_matches_reference_recipe():
    """quant.py:104-113: U(-2/sqrt(in), 2/sqrt(in)) and alpha = mean|W| -> ~25% zeros (2-bit)."""
    g = torch.Generator().manual_seed(0)
    W, alpha, b = qo.ref_layer_init(144, 576, g)
    assert float(W.abs().max()) <= 2 / 12 + 1e-6
    q = qo.np_quant_q(W.numpy(), float(alpha), 2)
    assert 0.20 < float((q == 0).mean()) < 0.30
    assert torch.count_nonzero(b) == 0


def test_bad_bitwidth():
    W = np.zeros((2, 2), F32)
    with pytest.raises(ValueError, match=r"bitwidth must be one of \{1,2,32\}"):
        qo.np_quant_q(W, 1.0, 3)
    with pytest.raises(ValueError, match=r"bitwidth must be one of \{1,2,32\}"):
        qo.c_quant_q(W, 1.0, 4)
    with pytest.raises(ValueError, match=r"bitwidth must be one of \{1,2,32\}"):
        qo.ref_quantize_weight(torch.zeros(2, 2), torch.tensor(1.0), 8)


def test_i8_mode_kat():
    """Hand-derived known answer for the opt-in int8 activation restatement: gamma = 127 so
    sx = 1 and rint's half-to-even ties are visible (-63.5 -> -64, 2.5 -> 2, 0.5 -> 0)."""
    X = np.array([[127.0, -63.5, 31.75, 2.5, 0.5]], np.float32)
    xq, gam = qo.np_act_quant_i8(X)
    assert gam == np.float32(127.0)
    assert xq.tolist() == [[127, -64, 32, 2, 0]]
    W = np.array([[1.0, -1.0, 0.1, 1.0, 1.0], [0.0, 0.6, -0.7, 0.2, -1.0]], np.float32)
    b = np.array([0.5, -0.25], np.float32)
    y = qo.np_bitlinear_fwd_i8(X, W, 1.0, b, 2)  # a = fp32(1 + 1e-8) = 1; Q2 = [1,-1,0,1,1], [0,1,-1,0,-1]
    acc = np.array([127 + 64 + 2 + 0, -64 - 32 - 0], np.float32)
    expect = (acc * np.float32(np.float32(1.0) * np.float32(np.float32(127.0) / np.float32(127.0)))).astype(np.float32) + b
    np.testing.assert_array_equal(y[0], expect)
    # all-zero input: gamma clamps to 1e-5, every code is 0, y = bias
    np.testing.assert_array_equal(qo.np_bitlinear_fwd_i8(np.zeros((2, 5), np.float32), W, 1.0, b, 1),
                                  np.broadcast_to(b, (2, 2)))
    deq = qo.np_act_dequant_i8(X)
    np.testing.assert_array_equal(deq, np.array([[127, -64, 32, 2, 0]], np.float32))
