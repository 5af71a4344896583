"""GPU parity of the fused BitLinear call sites (onebit_asr/fused.py, csrc/tgemm.hip
epilogues, csrc/fused.hip) against the unfused module code they replace
(conformer.py:34-45 FFN, :131-138 MHSA tail).

Bars (written here): dropout off -- forward max|err| <= 1e-6 * max|ref| and every gradient
rel-L2 <= 1e-6 (the same fp32 operations; only torch's own elementwise kernels may contract
differently); dropout on -- against a torch fp32 restatement driven by the kernels' own keep
masks (ob_relattn_dropout_mask on the same {seed, counter + offset}): forward and gradients
within the same bars, plus the kept fraction within 5 sigma of 1 - p.
"""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a = a.detach().double()
    b = b.detach().double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def _maxrel(a, b):
    return float((a.detach() - b.detach()).abs().max() / b.detach().abs().max().clamp_min(1e-30))


def _ffn_pair(gpu, d=144, dff=576, p=0.0):
    from onebit_asr.conformer import FeedForwardModule

    torch.manual_seed(3)
    m = FeedForwardModule(d, dff, p).to(gpu)
    with torch.no_grad():
        for lin in (m.lin1, m.lin2):
            lin.bias.uniform_(-0.1, 0.1)
    return m


def _run(m, x, bits, fused, monkeypatch):
    monkeypatch.setenv("OB_FUSED", "1" if fused else "0")
    for prm in m.parameters():
        prm.grad = None
    xx = x.clone().requires_grad_(True)
    y = m(xx, bits)
    g = torch.randn_like(y, generator=torch.Generator(device=y.device).manual_seed(11))
    (y * g).sum().backward()
    grads = {n: prm.grad.clone() for n, prm in m.named_parameters()}
    return y.detach(), xx.grad.clone(), grads


@pytest.mark.parametrize("bits,bt,t", [(1, 4, 50), (2, 4, 50), (2, 32, 249), (1, 96, 249)])
def test_ffn_fused_equals_unfused(gpu, bits, bt, t, monkeypatch):
    """Small shapes (one row tile per block) and Conformer-S shapes (each block walks several
    row tiles, so the cross-tile A prefetch of csrc/tgemm.hip is exercised)."""
    m = _ffn_pair(gpu).eval()
    x = torch.randn(bt, t, 144, device=gpu)
    y0, gx0, g0 = _run(m, x, bits, False, monkeypatch)
    y1, gx1, g1 = _run(m, x, bits, True, monkeypatch)
    assert _maxrel(y1, y0) <= 1e-6
    assert _rel(gx1, gx0) <= 1e-6
    for n in g0:
        # alpha: one cancellation-prone sum over N*K terms (its own bar, as elsewhere)
        assert _rel(g1[n], g0[n]) <= (1e-5 if n.endswith("alpha") else 1e-6), n


def test_ffn_fused_stacked_passes(gpu, monkeypatch):
    """P = 3 stacked passes (2-bit, 1-bit, 2-bit) == three single-pass calls."""
    from onebit_asr.quant import PassBits

    m = _ffn_pair(gpu).eval()
    x = torch.randn(3 * 2, 40, 144, device=gpu)
    pb = PassBits(torch.tensor([2, 1, 2], dtype=torch.int32, device=gpu))
    y, gx, g = _run(m, x, pb, True, monkeypatch)
    ys, gxs = [], []
    gsum = None
    gg = torch.randn_like(y, generator=torch.Generator(device=gpu).manual_seed(11))
    for p, bits in enumerate([2, 1, 2]):
        for prm in m.parameters():
            prm.grad = None
        xp = x[2 * p:2 * p + 2].clone().requires_grad_(True)
        yp = m(xp, bits)
        (yp * gg[2 * p:2 * p + 2]).sum().backward()
        ys.append(yp.detach())
        gxs.append(xp.grad)
        cur = {n: prm.grad.clone() for n, prm in m.named_parameters()}
        gsum = cur if gsum is None else {n: gsum[n] + cur[n] for n in cur}
    assert _maxrel(y, torch.cat(ys)) <= 1e-6
    assert _rel(gx, torch.cat(gxs)) <= 1e-6
    for n in g:
        assert _rel(g[n], gsum[n]) <= 1e-5, n  # per-pass sums in another order


def _mask(rng_state, off, n, p, gpu):
    from onebit_asr.attention import dropout_mask

    return dropout_mask((n,), p, rng_state, off).bool()


def test_ffn_dropout_matches_torch_restatement(gpu, monkeypatch):
    from onebit_asr import fused

    p = 0.1
    m = _ffn_pair(gpu, p=p).train()
    x = torch.randn(2, 64, 144, device=gpu)
    monkeypatch.setenv("OB_FUSED", "1")
    fused._rng(torch.device(gpu))  # make sure the device state exists
    st = fused._STATE[torch.device(gpu)]
    rng0, off0 = st[0].clone(), st[1]
    xx = x.clone().requires_grad_(True)
    y = m(xx, 2)
    g = torch.randn_like(y)
    (y * g).sum().backward()
    got = {n: prm.grad.clone() for n, prm in m.named_parameters()}
    rows = x.numel() // 144
    k1 = _mask(rng0, off0, rows * 576, p, gpu).view(rows, 576)
    k2 = _mask(rng0, off0 + 1, rows * 144, p, gpu).view(rows, 144)
    frac = k1.float().mean().item()
    assert abs(frac - (1 - p)) < 5 * np.sqrt(p * (1 - p) / k1.numel())
    # torch fp32 restatement with the same masks (layers through the unfused module code)
    monkeypatch.setenv("OB_FUSED", "0")
    for prm in m.parameters():
        prm.grad = None
    xr = x.clone().requires_grad_(True)
    h = m.lin1(m.ln(xr), 2)
    a = F.silu(h) * k1.view(2, 64, 576) / (1 - p)
    o = m.lin2(a, 2) * k2.view(2, 64, 144) / (1 - p)
    yr = xr + 0.5 * o
    (yr * g).sum().backward()
    assert _maxrel(y, yr) <= 1e-6
    assert _rel(xx.grad, xr.grad) <= 1e-6
    for n, prm in m.named_parameters():
        # d alpha is one scalar summed over every weight-gradient element (83k terms, ulp-level
        # differences of the epilogue's silu from torch's feed all of them): 1e-5
        assert _rel(got[n], prm.grad) <= (1e-5 if n.endswith("alpha") else 1e-6), n


def test_linear_residual_padding_and_dropout(gpu):
    """x + pad_zero(dropout(out_proj(ctx))) with ragged lengths and P = 3 passes."""
    from onebit_asr import fused
    from onebit_asr.quant import PassBits, QuantizedLinear

    torch.manual_seed(4)
    lin = QuantizedLinear(144, 144).to(gpu)
    with torch.no_grad():
        lin.bias.uniform_(-0.1, 0.1)
    P, B, T, p = 3, 2, 37, 0.1
    pb = PassBits(torch.tensor([2, 1, 1], dtype=torch.int32, device=gpu))
    lens = torch.tensor([37, 20] * P, dtype=torch.int32, device=gpu)
    ctx = torch.randn(P * B, T, 144, device=gpu, requires_grad=True)
    x = torch.randn(P * B, T, 144, device=gpu, requires_grad=True)
    fused._rng(torch.device(gpu))
    st = fused._STATE[torch.device(gpu)]
    rng0, off0 = st[0].clone(), st[1]
    y = fused.linear_residual(ctx, x, lin, pb, p, 1.0, lens, T)
    g = torch.randn_like(y)
    (y * g).sum().backward()
    got = (ctx.grad.clone(), x.grad.clone(), lin.weight.grad.clone(), lin.alpha.grad.clone(),
           lin.bias.grad.clone())
    keep = _mask(rng0, off0, P * B * T * 144, p, gpu).view(P * B, T, 144)
    valid = (torch.arange(T, device=gpu)[None, :] < lens[:, None]).float()[..., None]
    for prm in (ctx, x, lin.weight, lin.alpha, lin.bias):
        prm.grad = None
    outs = [lin(ctx[q * B:(q + 1) * B], b) for q, b in enumerate([2, 1, 1])]
    yr = x + torch.cat(outs) * keep / (1 - p) * valid
    (yr * g).sum().backward()
    assert _maxrel(y, yr) <= 1e-6
    assert torch.all(y[1, 20:] == x[1, 20:])  # padded rows carry the residual only
    ref = (ctx.grad, x.grad, lin.weight.grad, lin.alpha.grad, lin.bias.grad)
    for a, b, name in zip(got, ref, ["dctx", "dx", "dW", "dalpha", "db"]):
        assert _rel(a, b) <= 1e-5, name


def test_fused_entry_errors(gpu):
    from onebit_asr import _lib

    lib = _lib.load()
    # p_drop out of range and missing rng are rejected, nothing launched
    assert lib.ob_drop_scale_bwd(None, 0, 0, 1.0, 1.5, None, 0, None, 0, None, None) == -2
    assert lib.ob_drop_scale_bwd(16, 1, 4, 1.0, 0.1, None, 0, None, 0, 16, None) == -1


def test_layer_norm_fork_gradient(gpu):
    """(LN(x), x) fork: dx = LN_backward(dy) + d(residual), bit-identical to autograd's
    separate add (the kernel adds the two rounded terms, as the add kernel does)."""
    from onebit_asr.layernorm import layer_norm, layer_norm_fork

    torch.manual_seed(9)
    w = torch.randn(144, device=gpu, requires_grad=True)
    b = torch.randn(144, device=gpu, requires_grad=True)
    x = torch.randn(3, 77, 144, device=gpu, requires_grad=True)
    gy = torch.randn(3, 77, 144, device=gpu)
    gr = torch.randn(3, 77, 144, device=gpu)
    y, xr = layer_norm_fork(x, w, b)
    (y * gy + xr * gr).sum().backward()
    got = (x.grad.clone(), w.grad.clone(), b.grad.clone())
    for t in (x, w, b):
        t.grad = None
    y0 = layer_norm(x, w, b)
    (y0 * gy + x * gr).sum().backward()
    assert torch.equal(y, y0)
    assert torch.equal(got[0], x.grad)
    assert torch.equal(got[1], w.grad) and torch.equal(got[2], b.grad)


def test_subsampling_bias_relu_and_colsum(gpu):
    """conv2d_bias_relu == relu(conv2d(x, w, b)) bit for bit, gradients included; colsum ==
    torch's column sum within fp32 summation order."""
    import torch.nn as nn
    from onebit_asr.conv import colsum, conv2d_bias_relu

    torch.manual_seed(12)
    conv = nn.Conv2d(3, 8, kernel_size=3, stride=2).to(gpu)
    x = torch.randn(2, 3, 37, 21, device=gpu, requires_grad=True)
    y = conv2d_bias_relu(x, conv)
    g = torch.randn_like(y)
    (y * g).sum().backward()
    got = (x.grad.clone(), conv.weight.grad.clone(), conv.bias.grad.clone())
    x.grad = None
    conv.weight.grad = None
    conv.bias.grad = None
    y0 = torch.relu(conv(x))
    (y0 * g).sum().backward()
    assert torch.equal(y, y0)
    assert torch.equal(got[0], x.grad)
    # the weight gradient is MIOpen's (it may pick another algorithm for a bias-free conv)
    assert _rel(got[1], conv.weight.grad) <= 1e-5
    assert _rel(got[2], conv.bias.grad) <= 1e-6
    m = torch.randn(1000, 77, device=gpu)
    assert _rel(colsum(m), m.double().sum(0)) <= 1e-6


@pytest.mark.parametrize("stacked", [False, True])
def test_qkv_projections_match_separate_layers(gpu, stacked):
    """fused.qkv_projections (one autograd node, dX of k / v accumulated in the GEMM
    epilogue) == q_proj(h), k_proj(h), v_proj(h) as three module calls: outputs bit-exact,
    dh and every weight / alpha / bias gradient within fp32 summation-order noise."""
    from onebit_asr.fused import qkv_projections
    from onebit_asr.quant import QuantizedLinear, StackedBits

    torch.manual_seed(0)
    layers = [QuantizedLinear(144, 144).to(gpu) for _ in range(3)]
    with torch.no_grad():
        for m in layers:
            m.bias.normal_()
    if stacked:
        bits = StackedBits(1, gpu)
        bits.set([1])
        bw = bits[0]
    else:
        bw = 1
    rows = (3 if stacked else 1) * 2 * 249
    h = torch.randn(rows, 144, device=gpu, requires_grad=True)
    gouts = [torch.randn(rows, 144, device=gpu) for _ in range(3)]

    def run(fused):
        for m in layers:
            for p in m.parameters():
                p.grad = None
        h.grad = None
        outs = qkv_projections(h, *layers, bw) if fused else [m(h, bw) for m in layers]
        torch.autograd.backward(outs, gouts)
        return ([o.detach().clone() for o in outs], h.grad.clone(),
                [p.grad.clone() for m in layers for p in (m.weight, m.alpha, m.bias)])

    o0, dh0, g0 = run(False)
    o1, dh1, g1 = run(True)
    for a, b in zip(o0, o1):
        assert torch.equal(a, b)
    assert (dh0 - dh1).abs().max().item() <= 1e-6 * dh0.abs().max().item()
    for a, b in zip(g0, g1):
        assert (a - b).abs().max().item() <= 1e-6 * max(a.abs().max().item(), 1e-30), (a, b)
    # stacked: the three dW GEMMs run as one grouped launch (144x144 tiles, one per layer)
    # and one grouped finish: dW / db the same bits as one by one (same chunks, same per-element
    # product order); dalpha sums the same terms in other per-block groupings (rounding only)
    from onebit_asr import fused

    prev, fused._DW_GROUP = fused._DW_GROUP, False
    try:
        _, _, g2 = run(True)
    finally:
        fused._DW_GROUP = prev
    for a, b in zip(g1, g2):
        if a.dim() == 0:
            assert abs(a.item() - b.item()) <= 1e-6 * abs(b.item()) + 1e-12, (a, b)
        else:
            assert torch.equal(a, b)


def test_decoder_residual_dropout(gpu):
    """conformer._residual_dropout (decoder post-norm sublayers): out = x + keep * y / (1-p)
    with a keep rate ~ 1-p, dy = keep / (1-p) * gout and dx = gout -- both directly and with
    the dropout backward formed by the following LayerNorm's backward (GradScale hand-off),
    bit for bit; identity when not training."""
    from onebit_asr.conformer import _residual_dropout
    from onebit_asr.layernorm import layer_norm

    p = 0.1
    g = torch.Generator().manual_seed(3)
    x = torch.zeros(6, 41, 144, device=gpu, requires_grad=True)  # out - x exact
    y = torch.ones(6, 41, 144, device=gpu, requires_grad=True)
    out = _residual_dropout(x, y, p, True)
    d = (out - x).detach()
    scale = torch.tensor(1.0 / (1.0 - p), device=gpu)
    assert bool(((d == 0) | (d == scale)).all())
    keep = (d != 0).float().mean().item()
    assert abs(keep - (1 - p)) < 0.01, keep
    gout = torch.randn(out.shape, generator=g).to(gpu)
    out.backward(gout)
    assert torch.equal(x.grad, gout)
    assert torch.equal(y.grad, torch.where(d != 0, gout * scale, torch.zeros_like(gout)))
    # through the LN hand-off: y's gradient == the separate dropout backward of LN's dx
    w = torch.randn(144, generator=g).to(gpu)
    b = torch.randn(144, generator=g).to(gpu)
    x = torch.randn(6, 41, 144, generator=g).to(gpu).requires_grad_()
    y.grad = None
    ln = layer_norm(_residual_dropout(x, y, p, True), w, b, 1e-5)
    ln.backward(gout)
    gx, gy = x.grad.clone(), y.grad.clone()
    d2 = gy != 0
    assert torch.equal(torch.where(d2, gx * scale, torch.zeros_like(gx)), gy)
    assert torch.equal(_residual_dropout(x, y, p, False), x + y)


def test_qkv_forward_group_equals_separate(gpu, monkeypatch):
    """The q/k/v projections as one grouped launch (ob_bitlinear_fwd_passes_group) == three
    separate launches, bit for bit (stacked passes, both bitwidths)."""
    from onebit_asr import fused
    from onebit_asr.quant import QuantizedLinear, StackedBits

    torch.manual_seed(7)
    layers = [QuantizedLinear(144, 144).to(gpu) for _ in range(3)]
    for l in layers:
        with torch.no_grad():
            l.bias.uniform_(-0.1, 0.1)
    bits = StackedBits(1, gpu)
    bits.set([1])  # passes at 2, 1, 1 bits
    h = torch.randn(3 * 500, 144, device=gpu)
    outs = {}
    for grp in (True, False):
        monkeypatch.setattr(fused, "_QKV_FWD_GROUP", grp)
        with torch.no_grad():
            outs[grp] = fused.qkv_projections(h, *layers, bits[0])
    for a, b in zip(outs[True], outs[False]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("sp", [1, 0])
def test_qkv_input_gradient_summed_in_one_launch(gpu, monkeypatch, sp):
    """The q / k / v node's input gradient from ONE launch (ob_bitlinear_bwd_dx_passes_sum:
    the three sources' codes side by side, each chunk pre-scaled by its layer's alpha) against
    the three launches it replaces (q's plain dX, then k's and v's accumulated through the
    residual epilogue) and against float64 of the reference's sum of the three layers'
    dY (alpha Q) products: 1e-6 / 1e-5 of max (only the rounding order differs). Stacked
    passes at 2 / 1 / (1 or 2) bits, Conformer-S width, rows not a multiple of the tiles."""
    from onebit_asr import fused
    from onebit_asr.quant import QuantizedLinear, StackedBits
    from oracle.quant_oracle import ref_quantize_weight

    P, m, d = 3, 997, 144
    pass_bits = [2, 1, 1 if sp else 2]
    torch.manual_seed(0)
    layers = [QuantizedLinear(d, d).to(gpu) for _ in range(3)]
    sb = StackedBits(1, gpu)
    sb.set([sp])
    h = torch.randn(P * m, d, device=gpu)
    gouts = [torch.randn(P * m, d, device=gpu) for _ in range(3)]
    res = {}
    for on in (False, True):
        monkeypatch.setattr(fused, "_DX_SUM", on)
        x = h.clone().requires_grad_()
        outs = fused.qkv_projections(x, *layers, sb[0])
        torch.autograd.backward(outs, gouts)
        res[on] = x.grad.detach().clone()
    ref = torch.zeros(P * m, d, dtype=torch.float64)
    with torch.no_grad():
        for lay, go in zip(layers, gouts):
            for p in range(P):
                wq = ref_quantize_weight(lay.weight.detach().cpu(), lay.alpha.detach().cpu(),
                                         pass_bits[p])
                ref[p * m:(p + 1) * m] += go[p * m:(p + 1) * m].cpu().double() @ wq.double()
    scale = ref.abs().max().item()
    assert (res[True].cpu().double() - res[False].cpu().double()).abs().max().item() <= 1e-6 * scale
    assert (res[True].cpu().double() - ref).abs().max().item() <= 1e-5 * scale
