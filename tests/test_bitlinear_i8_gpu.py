"""GPU parity of the opt-in int8-activation BitLinear mode (csrc/tgemm_i8.hip) through the
C ABI, against oracle/quant_oracle.py's restatement of the mode.

This mode is NOT the reference's arithmetic (the reference keeps activations fp32,
quant.py:126), so it has its own bars, written here:
  absmax, dequantized activations, forward Y   : bit-exact vs the numpy fp32 restatement
                                                  (integer accumulation, then one rounded
                                                  mul and one rounded add per output);
  dX  (STE)                                    : max|err| <= 1e-5 * max|ref| + 1e-6 vs float64
  dW  (= dY^T X_deq masked)                    : rel-L2 <= 1e-5 vs float64;
  whole model (cfg1, 2-bit): CTC loss rel <= 3e-2 and logits cosine >= 0.99 vs the fp32
  activation path (the north-star tolerance SURVEY.md §8c proposes).
"""
import numpy as np
import pytest
import torch

from oracle import quant_oracle as qo

pytestmark = pytest.mark.gpu

SHAPES = [  # (M, K, N): Conformer widths plus ragged rows / narrow N
    (1, 16, 16), (5, 64, 37), (100, 144, 144), (249, 144, 576), (364, 256, 64),
    (1000, 576, 144), (7968, 144, 576), (63, 48, 130),
]


def _data(M, K, N, seed):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((M, K)).astype(np.float32)
    X[rng.random((M, K)) < 0.05] = 0.0
    W = ((rng.random((N, K)) * 2 - 1) * (2 / np.sqrt(K))).astype(np.float32)
    alpha = float(np.abs(W).mean())
    b = rng.standard_normal(N).astype(np.float32)
    return X, W, alpha, b


def _lib():
    from onebit_asr import _lib

    return _lib, _lib.load()


@pytest.mark.parametrize("M,K,N", SHAPES)
@pytest.mark.parametrize("bits", [2, 1])
def test_fwd_i8_bit_exact(gpu, M, K, N, bits):
    from onebit_asr.quant import pack_codes

    X, W, alpha, b = _data(M, K, N, M * 7 + K + N + bits)
    L, lib = _lib()
    Xd = torch.from_numpy(X).to(gpu)
    Wd = torch.from_numpy(W).to(gpu)
    ad = torch.tensor(alpha, device=gpu)
    bd = torch.from_numpy(b).to(gpu)
    codes, _ = pack_codes(Wd, ad, bits)
    from onebit_asr.quant import act_absmax

    amax = act_absmax(Xd)
    s = L.stream_of(Xd)
    Y = torch.empty(M, N, device=gpu)
    L.check(lib.ob_bitlinear_fwd_i8(Xd.data_ptr(), 1, M, K, codes.data_ptr(), None, None,
                                    ad.data_ptr(), 1, amax.data_ptr(), bd.data_ptr(), N,
                                    Y.data_ptr(), s), "fwd_i8")
    torch.cuda.synchronize()
    assert amax.item() == float(np.abs(X).max())
    ref = qo.np_bitlinear_fwd_i8(X, W, alpha, b, bits)
    got = Y.cpu().numpy()
    bad = np.argwhere(got != ref)
    assert bad.size == 0, f"{len(bad)} mismatches, first {bad[:3].tolist()}: {got[tuple(bad[0])]} vs {ref[tuple(bad[0])]}"


def test_fwd_i8_stacked_passes(gpu):
    """P = 3 passes with bitwidths [2, 1, 1] and their own absmax each."""
    from onebit_asr.quant import pack_codes

    P, M, K, N = 3, 333, 144, 144
    rng = np.random.default_rng(5)
    X = (rng.standard_normal((P, M, K)) * np.array([1.0, 3.0, 0.25])[:, None, None]).astype(np.float32)
    _, W, alpha, b = _data(M, K, N, 9)
    L, lib = _lib()
    Xd = torch.from_numpy(X.reshape(P * M, K)).to(gpu)
    Wd, ad, bd = torch.from_numpy(W).to(gpu), torch.tensor(alpha, device=gpu), torch.from_numpy(b).to(gpu)
    c2, _ = pack_codes(Wd, ad, 2)
    c1, _ = pack_codes(Wd, ad, 1)
    pbits = torch.tensor([2, 1, 1], dtype=torch.int32, device=gpu)
    from onebit_asr.quant import act_absmax

    amax = act_absmax(Xd, P)
    s = L.stream_of(Xd)
    Y = torch.empty(P * M, N, device=gpu)
    L.check(lib.ob_bitlinear_fwd_i8(Xd.data_ptr(), P, M, K, c2.data_ptr(), c1.data_ptr(),
                                    pbits.data_ptr(), ad.data_ptr(), 1, amax.data_ptr(),
                                    bd.data_ptr(), N, Y.data_ptr(), s), "fwd_i8")
    got = Y.cpu().numpy().reshape(P, M, N)
    for p, bits in enumerate([2, 1, 1]):
        assert amax[p].item() == float(np.abs(X[p]).max())
        np.testing.assert_array_equal(got[p], qo.np_bitlinear_fwd_i8(X[p], W, alpha, b, bits))


def test_dequant_and_zero_input(gpu):
    L, lib = _lib()
    X = np.random.default_rng(1).standard_normal((77, 64)).astype(np.float32)
    for arr in (X, np.zeros_like(X)):
        Xd = torch.from_numpy(arr).to(gpu)
        from onebit_asr.quant import act_absmax

        amax = act_absmax(Xd)
        out = torch.empty_like(Xd)
        s = L.stream_of(Xd)
        L.check(lib.ob_act_dequant_i8(Xd.data_ptr(), 1, arr.size, amax.data_ptr(),
                                      out.data_ptr(), s), "dequant")
        np.testing.assert_array_equal(out.cpu().numpy(), qo.np_act_dequant_i8(arr))


def test_unsupported_shape_raises(gpu):
    from onebit_asr.quant import QuantizedLinear

    layer = QuantizedLinear(20, 8, act_quant="absmax_int8").to(gpu)  # K % 16 != 0
    with pytest.raises(RuntimeError, match="invalid shape"):
        layer(torch.randn(4, 20, device=gpu), 2)
    with pytest.raises(ValueError):
        QuantizedLinear(16, 8, act_quant="int4")


@pytest.mark.parametrize("stacked", [False, True])
def test_module_i8_backward(gpu, stacked):
    from onebit_asr.quant import PassBits, QuantizedLinear

    torch.manual_seed(3)
    K, N, M = 144, 576, 249
    layer = QuantizedLinear(K, N, act_quant="absmax_int8").to(gpu)
    P = 3 if stacked else 1
    pass_bits = [2, 1, 2]
    x = torch.randn(P * M, K, device=gpu, requires_grad=True)
    dy = torch.randn(P * M, N, device=gpu)
    bw = PassBits(torch.tensor(pass_bits, dtype=torch.int32, device=gpu)) if stacked else 2
    y = layer(x, bw)
    y.backward(dy)
    W = layer.weight.detach().cpu().numpy()
    alpha = float(layer.alpha.item())
    X = x.detach().cpu().numpy().reshape(P, M, K)
    DY = dy.cpu().numpy().astype(np.float64).reshape(P, M, N)
    a = qo.np_effective_alpha(alpha)
    wa = (W / a).astype(np.float32)
    dX = np.zeros((P, M, K))
    dW = np.zeros((N, K))
    for p in range(P):
        bits = pass_bits[p] if stacked else 2
        np.testing.assert_array_equal(
            y.detach().cpu().numpy().reshape(P, M, N)[p],
            qo.np_bitlinear_fwd_i8(X[p], W, alpha, layer.bias.detach().cpu().numpy(), bits))
        w_hat = (a * qo.np_quant_q(W, alpha, bits)).astype(np.float64)
        dX[p] = DY[p] @ w_hat
        G = DY[p].T @ qo.np_act_dequant_i8(X[p]).astype(np.float64)
        dW += G * (np.abs(wa) <= 1)
    got_dx = x.grad.cpu().numpy().reshape(P, M, K)
    assert np.abs(got_dx - dX).max() <= 1e-5 * np.abs(dX).max() + 1e-6
    rel = np.linalg.norm(layer.weight.grad.cpu().numpy() - dW) / np.linalg.norm(dW)
    assert rel <= 1e-5, rel


def test_model_i8_close_to_fp32_acts(gpu):
    """cfg1 Conformer, 2-bit weights: int8 activations vs the reference's fp32 activations."""
    from onebit_asr.conformer import ConformerASR
    from onebit_asr.data import CFG1, synthetic_batch
    from onebit_asr.losses import ctc_loss_from_logits
    from onebit_asr.quant import set_act_quant

    torch.manual_seed(0)
    model = ConformerASR(80, 5004, **CFG1).to(gpu).eval()
    batch = synthetic_batch([734, 349], [27, 12], seed=0, device=gpu)
    with torch.no_grad():
        _, mask, ref = model(batch, precision=2)
        set_act_quant(model, "absmax_int8")
        _, _, got = model(batch, precision=2)
        set_act_quant(model, None)
        lens = mask.sum(1).long()
        l_ref = ctc_loss_from_logits(ref, lens, batch["tokens"], batch["token_lens"], 3).item()
        l_got = ctc_loss_from_logits(got, lens, batch["tokens"], batch["token_lens"], 3).item()
    cos = torch.nn.functional.cosine_similarity(got.flatten(), ref.flatten(), dim=0).item()
    assert abs(l_got - l_ref) <= 3e-2 * abs(l_ref), (l_got, l_ref)
    assert cos >= 0.99, cos
