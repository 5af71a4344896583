"""ob_dw_grouped: every deferred weight gradient of a backward in one stream-K launch
(csrc/dw.hip dw_grouped_kernel), through the C ABI.

One launch holds a mix of gemms -- BitLinear (quant.py:72-92 + the autograd of quant.py:126:
STE-masked dW, dalpha at each stacked pass's bitwidth, db) and dense ones (W = NULL) -- with
ragged pass lengths (rows not a multiple of the 32-row step, a 1-row pass), several tiles per
gemm (N or K = 576) and passes of different bitwidths, so segments cross pass boundaries and
tiles are split between blocks. Checked against:
* the float64 oracle (oracle/quant_oracle.py helpers): dW rel-L2 <= 1e-5, db <= 1e-5 of max,
  dalpha <= 1e-5 * sum|G * term| (the single-layer bars of test_bitlinear_gpu.py);
* the per-layer entry ob_bitlinear_bwd_dw_passes / ob_dense_dw (same products, another
  summation order): dW / db rel <= 2e-6;
* itself: a second launch is bit-identical (static partition, fixed summation order) and the
  ticket words are all zero again after each launch.
"""
import ctypes

import numpy as np
import pytest
import torch

from oracle import quant_oracle as qo

pytestmark = pytest.mark.gpu

# (M per pass, K, N, pass bits or None = dense, bias)
GEMMS = [
    (7968, 144, 576, [2, 1, 1], True),
    (7968, 576, 144, [2, 1, 2], True),
    (249, 144, 144, [1, 1, 2], False),
    (3000, 144, 288, None, True),
    (33, 144, 144, [2, 1, 1], True),
    (1, 288, 144, [1, 2], True),
    (1000, 144, 144, None, False),
    (517, 432, 144, [2], True),
]


def _make(gpu, seed=0):
    g = torch.Generator(device=gpu).manual_seed(seed)
    out = []
    for M, K, N, bits, has_b in GEMMS:
        P = len(bits) if bits else 1
        x = torch.randn(P * M, K, device=gpu, generator=g)
        dy = torch.randn(P * M, N, device=gpu, generator=g)
        W = (torch.rand(N, K, device=gpu, generator=g) * 2 - 1) * (2.0 / K ** 0.5)
        alpha = W.abs().mean().reshape(())
        pb = torch.tensor(bits, dtype=torch.int32, device=gpu) if bits else None
        out.append(dict(M=M, K=K, N=N, P=P, bits=bits, x=x, dy=dy, W=W, alpha=alpha, pb=pb,
                        dW=torch.full((N, K), float("nan"), device=gpu),
                        db=torch.full((N,), float("nan"), device=gpu) if has_b else None,
                        da=torch.full((), float("nan"), device=gpu)))
    return out


def _launch(lib, gpu, gemms, tickets):
    from onebit_asr import _lib
    from onebit_asr.deferred import DwgGemm

    arr = (DwgGemm * len(gemms))(*[
        DwgGemm(e["dy"].data_ptr(), e["x"].data_ptr(), e["W"].data_ptr() if e["bits"] else None,
                e["alpha"].data_ptr(), _lib.ptr(e["pb"]), e["dW"].data_ptr(), _lib.ptr(e["db"]),
                e["da"].data_ptr(), e["N"], e["K"], e["M"], e["P"], 1, 2) for e in gemms])
    ad = ctypes.addressof(arr)
    wsb = lib.ob_dw_grouped_workspace(ad, len(gemms))
    nt = lib.ob_dw_grouped_tickets(ad, len(gemms))
    assert wsb > 0 and 0 < nt <= tickets.numel()
    ws = torch.empty(wsb, dtype=torch.uint8, device=gpu)
    s = torch.cuda.current_stream().cuda_stream
    _lib.check(lib.ob_dw_grouped(ad, len(gemms), ws.data_ptr(), wsb, tickets.data_ptr(),
                                 tickets.numel(), s), "ob_dw_grouped")
    torch.cuda.synchronize()


def test_grouped_against_oracle_and_per_layer(gpu):
    from onebit_asr import _lib

    lib = _lib.load()
    gemms = _make(gpu)
    tickets = torch.zeros(4096, dtype=torch.int32, device=gpu)
    _launch(lib, gpu, gemms, tickets)
    assert int(tickets.abs().sum()) == 0
    s = torch.cuda.current_stream().cuda_stream
    for e in gemms:
        M, K, N, P, bits = e["M"], e["K"], e["N"], e["P"], e["bits"]
        X = e["x"].double().cpu().numpy().reshape(P, M, K)
        DY = e["dy"].double().cpu().numpy().reshape(P, M, N)
        G = sum(DY[p].T @ X[p] for p in range(P))
        got = e["dW"].double().cpu().numpy()
        assert np.isfinite(got).all(), (M, K, N)
        if bits:
            araw = float(e["alpha"].item())
            a = qo.np_effective_alpha(araw)
            wa = (e["W"].cpu().numpy() / a).astype(np.float32)
            want = G * (np.abs(wa) <= 1)
            dal = scale = 0.0
            for p in range(P):
                t = qo.np_term(wa, bits[p]).astype(np.float64) * (DY[p].T @ X[p])
                dal += float(t.sum())
                scale += float(np.abs(t).sum())
            dal *= float(np.sign(np.float32(araw)))
            assert abs(e["da"].item() - dal) <= 1e-5 * scale + 1e-6, (M, K, N, e["da"].item(), dal)
        else:
            want = G
        assert np.linalg.norm(got - want) <= 1e-5 * np.linalg.norm(want), (M, K, N)
        if e["db"] is not None:
            dbw = DY.sum(axis=(0, 1))
            assert np.abs(e["db"].double().cpu().numpy() - dbw).max() <= 1e-5 * np.abs(dbw).max() + 1e-6

        # the per-layer entry points (the path the grouped launch replaces)
        dW2 = torch.empty_like(e["dW"])
        db2 = torch.empty_like(e["db"]) if e["db"] is not None else None
        if bits:
            da2 = torch.empty((), device=gpu)
            wsb = lib.ob_bitlinear_bwd_dw_passes_workspace(P, M, N, K)
            ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=gpu)
            _lib.check(lib.ob_bitlinear_bwd_dw_passes(
                e["dy"].data_ptr(), e["x"].data_ptr(), P, M, N, K, e["W"].data_ptr(),
                e["alpha"].data_ptr(), 1, e["pb"].data_ptr(), dW2.data_ptr(), da2.data_ptr(),
                _lib.ptr(db2), ws.data_ptr(), wsb, s), "ob_bitlinear_bwd_dw_passes")
            assert abs(da2.item() - e["da"].item()) <= 2e-6 * scale + 1e-7
        else:
            wsb = lib.ob_dense_dw_workspace(P * M, N, K)
            ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=gpu)
            _lib.check(lib.ob_dense_dw(e["dy"].data_ptr(), e["x"].data_ptr(), P * M, N, K,
                                       dW2.data_ptr(), _lib.ptr(db2), ws.data_ptr(), wsb, s),
                       "ob_dense_dw")
        torch.cuda.synchronize()
        assert ((dW2 - e["dW"]).norm() / dW2.norm()).item() <= 2e-6, (M, K, N)
        if db2 is not None:
            assert ((db2 - e["db"]).abs().max() / db2.abs().max()).item() <= 2e-6


def test_grouped_deterministic_and_tickets_reset(gpu):
    from onebit_asr import _lib

    lib = _lib.load()
    gemms = _make(gpu, seed=1)
    tickets = torch.zeros(4096, dtype=torch.int32, device=gpu)
    _launch(lib, gpu, gemms, tickets)
    first = [(e["dW"].clone(), None if e["db"] is None else e["db"].clone(), e["da"].clone())
             for e in gemms]
    for e in gemms:
        e["dW"].fill_(float("nan"))
    _launch(lib, gpu, gemms, tickets)
    assert int(tickets.abs().sum()) == 0
    for e, (w, b, a) in zip(gemms, first):
        assert torch.equal(e["dW"], w)
        if b is not None:
            assert torch.equal(e["db"], b)
        if e["bits"]:
            assert torch.equal(e["da"], a)


def test_grouped_small_launch(gpu):
    """Fewer 32-row steps than CUs (one block per step range of one step): still exact."""
    from onebit_asr import _lib

    lib = _lib.load()
    g = torch.Generator(device=gpu).manual_seed(5)
    M, K, N = 40, 144, 144
    x = torch.randn(M, K, device=gpu, generator=g)
    dy = torch.randn(M, N, device=gpu, generator=g)
    e = dict(M=M, K=K, N=N, P=1, bits=None, x=x, dy=dy, W=None, alpha=torch.ones((), device=gpu),
             pb=None, dW=torch.empty(N, K, device=gpu), db=torch.empty(N, device=gpu),
             da=torch.empty((), device=gpu))
    tickets = torch.zeros(64, dtype=torch.int32, device=gpu)
    _launch(lib, gpu, [e], tickets)
    want = dy.double().t() @ x.double()
    assert ((e["dW"].double() - want).norm() / want.norm()).item() <= 1e-5
    assert torch.allclose(e["db"].double(), dy.double().sum(0), rtol=1e-5, atol=1e-5)
    assert int(tickets.abs().sum()) == 0


def test_grouped_rejects_bad_arguments(gpu):
    from onebit_asr import _lib
    from onebit_asr.deferred import DwgGemm

    lib = _lib.load()
    assert lib.ob_dw_grouped_supported(144, 576) == 1
    assert lib.ob_dw_grouped_supported(144, 96) == 0
    x = torch.zeros(64, 96, device=gpu)
    arr = (DwgGemm * 1)(DwgGemm(x.data_ptr(), x.data_ptr(), None, None, None, x.data_ptr(),
                                None, None, 96, 96, 64, 1, 1, 2))
    assert lib.ob_dw_grouped_workspace(ctypes.addressof(arr), 1) == 0
