"""GPU parity of the channels-last fused conv module (onebit_asr/conv.py conv_module_fused,
csrc/convmod.hip) against the unfused module code (conformer.py:139-167 as restated in
ConvModule's [B,C,T] path: MIOpen / torch GLU, depthwise, BatchNorm, swish).

Bars (written here): forward max|err| <= 1e-5 * max|ref| (BatchNorm statistics are summed
in fp64 here, in fp32 by MIOpen); input and parameter gradients rel-L2 <= 1e-4 (the
BatchNorm backward's two batch means amplify summation-order differences).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


def _module(gpu, d, k=31, p=0.0):
    from onebit_asr.conformer import ConvModule

    torch.manual_seed(7)
    m = ConvModule(d, kernel_size=k, dropout=p).to(gpu)
    with torch.no_grad():
        m.bn.weight.uniform_(0.5, 1.5)
        m.bn.bias.uniform_(-0.2, 0.2)
    return m


def _run(m, x, passes, fused, monkeypatch):
    monkeypatch.setenv("OB_FUSED", "1" if fused else "0")
    for prm in m.parameters():
        prm.grad = None
    xx = x.clone().requires_grad_(True)
    y = m(xx, passes=passes)
    g = torch.randn_like(y, generator=torch.Generator(device=y.device).manual_seed(5))
    (y * g).sum().backward()
    return y.detach(), xx.grad, {n: q.grad.clone() for n, q in m.named_parameters()}


@pytest.mark.parametrize("d,bt,t,passes", [(144, 6, 249, 3), (64, 2, 182, 1), (144, 2, 40, 1),
                                           (36, 3, 7, 3)])
def test_conv_module_fused_equals_unfused(gpu, d, bt, t, passes, monkeypatch):
    m = _module(gpu, d).eval()  # eval: dropout off; BatchNorm still uses batch statistics
    x = torch.randn(bt, t, d, device=gpu) * 2.0 + 0.3
    y0, gx0, g0 = _run(m, x, passes, False, monkeypatch)
    y1, gx1, g1 = _run(m, x, passes, True, monkeypatch)
    err = float((y1 - y0).abs().max() / y0.abs().max())
    assert err <= 1e-5, err
    assert _rel(gx1, gx0) <= 1e-4
    for n in g0:
        if n == "dw.bias":
            # a per-channel constant before BatchNorm has zero gradient (BN subtracts the
            # batch mean): both paths hold round-off only -- bound it against dw.weight's
            scale = float(g0["dw.weight"].abs().max())
            assert float(g1[n].abs().max()) <= 1e-4 * scale
            assert float(g0[n].abs().max()) <= 1e-4 * scale
            continue
        assert _rel(g1[n], g0[n]) <= 1e-4, (n, _rel(g1[n], g0[n]))


def test_conv_module_dropout_mask(gpu, monkeypatch):
    """Training-mode dropout: out - x is zero exactly where the kernel's mask drops and equals
    the p = 0 output / (1 - p) elsewhere; the backward applies the same mask."""
    from onebit_asr import fused

    p = 0.1
    m = _module(gpu, 144, p=p).train()
    x = torch.randn(2, 50, 144, device=gpu)
    monkeypatch.setenv("OB_FUSED", "1")
    fused._rng(torch.device(gpu))
    y = m(x, passes=1)
    m.dropout.p = 0.0
    y0 = m(x, passes=1)
    d, d0 = y - x, y0 - x
    dropped = d == 0
    frac = dropped.float().mean().item()
    assert abs(frac - p) < 0.01
    kept = ~dropped
    assert torch.allclose(d[kept], d0[kept] / (1 - p), rtol=1e-5, atol=1e-6)


def test_convmod_abi_errors(gpu):
    from onebit_asr import _lib

    lib = _lib.load()
    assert lib.ob_convmod_workspace(1, 2, 10, 144, 30) == 0  # even kernel width
    assert lib.ob_convmod_workspace(2, 3, 10, 144, 31) == 0  # Bt not a multiple of P
    assert lib.ob_convmod_workspace(1, 2, 10, 4096, 31) == 0  # LDS tile cannot fit
    assert lib.ob_convmod_workspace(3, 6, 249, 144, 31) > 0


@pytest.mark.parametrize("d,bt,t,passes", [(144, 6, 249, 3), (64, 2, 182, 1), (48, 3, 70, 3)])
def test_conv_module_tiles_bitwise_equal_whole_row(gpu, d, bt, t, passes):
    """The channel-split tile kernels (dz and the GLU backward folded in) == the whole-row
    kernels: the same operations in the same order, so the forward is bitwise equal and the
    gradients agree to rel-L2 <= 1e-6 (hipcc may contract a different multiply-add pair
    into an fma in the two kernels). OB_CM_TILE=0 forces the whole-row kernels; the switch
    is read once per process, so each side runs in its own process."""
    import os
    import subprocess
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    code = f"""
import sys, torch
sys.path[:0] = [{str(root)!r}, {str(root / 'cmu-11785-idl-1.58bit-asr_amd')!r}]
from onebit_asr.conformer import ConvModule
torch.manual_seed(7)
m = ConvModule({d}, kernel_size=31, dropout=0.0).cuda().eval()
with torch.no_grad():
    m.bn.weight.uniform_(0.5, 1.5); m.bn.bias.uniform_(-0.2, 0.2)
x = (torch.randn({bt}, {t}, {d}, device='cuda', generator=torch.Generator(device='cuda').manual_seed(3)) * 2 + 0.3).requires_grad_()
y = m(x, passes={passes})
g = torch.randn(y.shape, device='cuda', generator=torch.Generator(device='cuda').manual_seed(5))
(y * g).sum().backward()
out = {{'y': y.detach().cpu(), 'gx': x.grad.cpu()}}
out.update({{n: q.grad.cpu() for n, q in m.named_parameters()}})
torch.save(out, sys.argv[1])
"""
    res = []
    for flag in ("1", "0"):
        f = f"/tmp/cm_tile_{os.getpid()}_{flag}.pt"
        env = dict(os.environ, OB_CM_TILE=flag, OB_FUSED="1")
        r = subprocess.run([sys.executable, "-c", code, f], env=env, capture_output=True,
                           text=True, timeout=180)
        assert r.returncode == 0, r.stderr[-2000:]
        res.append(torch.load(f, weights_only=True))
        os.unlink(f)
    assert torch.equal(res[0]["y"], res[1]["y"])
    for k in res[0]:
        if k == "y" or k == "dw.bias":  # dw.bias: a true-zero gradient (rounding residuals)
            continue
        assert _rel(res[0][k], res[1][k]) <= 1e-6, (k, _rel(res[0][k], res[1][k]))


def test_pw2_residual_epilogue_bitwise(gpu, monkeypatch):
    """pw2 + dropout + residual in one dgemm launch (ob_dense_gemm_residual_drop) == pw2, then
    the residual-dropout kernel: output and every gradient bit for bit (training, p = 0.1)."""
    from onebit_asr import conv, fused

    m = _module(gpu, 144, p=0.1).train()
    x = torch.randn(3, 61, 144, device=gpu)
    monkeypatch.setenv("OB_FUSED", "1")
    dev = torch.device(gpu)
    fused._rng(dev)
    snap = fused.rng_snapshot(dev)
    res = []
    for on in (True, False):
        monkeypatch.setattr(conv, "_PW_RESID", on)
        fused.rng_restore(dev, snap)
        res.append(_run(m, x, 3, True, monkeypatch))
    (y1, gx1, g1), (y0, gx0, g0) = res
    assert torch.equal(y1, y0)
    assert torch.equal(gx1, gx0)
    for n in g0:
        assert torch.equal(g1[n], g0[n]), n
