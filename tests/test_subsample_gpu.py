"""Conv2dSubsampling's convolutions in csrc/subsample.hip (conformer.py:183-186) against the
oracle's restatement (oracle/conformer_oracle.py:152-155: F.conv2d -> ReLU twice) run in
float64 on the CPU.

Tolerances (fp32 arithmetic, exact-fp32 MFMA products, fixed-order sums):
  forward Y2           max |err| <= 1e-5 * max |ref|
  dW2, db2, dW0, db0   rel-L2 <= 1e-5 (dW0 / db0 sum ~B T1 F1 terms each)
Shapes: the Conformer-S channel count (144), the cfg0/cfg1 one (64), the minimum frame
count (T = 7 -> T2 = 1), ragged odd/even T and F (the dgrad parity classes differ in size)
and a batch large enough for several row tiles per block."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref(x, w0, b0, w2, b2, g):
    """fp64 oracle forward + the gradients of sum(y2 * g)."""
    F = torch.nn.functional
    p = [t.detach().cpu().double().requires_grad_(True) for t in (w0, b0, w2, b2)]
    z = F.relu(F.conv2d(x.cpu().double()[:, None], p[0], p[1], stride=2))
    y2 = F.relu(F.conv2d(z, p[2], p[3], stride=2))  # [B, C, T2, F2]
    y2 = y2.permute(0, 2, 3, 1)                     # channels last
    (y2 * g.cpu().double()).sum().backward()
    return y2.detach(), [q.grad for q in p]


def _rel(a, b):
    return ((a.double().cpu() - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("B,T,F,C", [
    (2, 7, 80, 144),     # minimum frames: T1 = 3, T2 = 1
    (3, 37, 80, 144),    # odd T
    (2, 40, 81, 144),    # even T, odd F
    (2, 33, 80, 64),     # cfg0 / cfg1 channel count
    (5, 301, 80, 144),   # several row tiles per persistent block
    (4, 64, 80, 96),
])
def test_subsample_matches_fp64(gpu, B, T, F, C):
    from onebit_asr.conv import _SubsampleFn

    torch.manual_seed(B * 1000 + T + C)
    conv0 = torch.nn.Conv2d(1, C, 3, 2)
    conv2 = torch.nn.Conv2d(C, C, 3, 2)
    x = torch.randn(B, T, F)
    t2 = ((T - 3) // 2 + 1 - 3) // 2 + 1
    f2 = ((F - 3) // 2 + 1 - 3) // 2 + 1
    g = torch.randn(B, t2, f2, C)
    y_ref, grads_ref = _ref(x, conv0.weight, conv0.bias, conv2.weight, conv2.bias, g)

    ps = [t.detach().to(gpu).requires_grad_(True)
          for t in (conv0.weight, conv0.bias, conv2.weight, conv2.bias)]
    y = _SubsampleFn.apply(x.to(gpu), *ps)
    assert y.shape == (B, t2, f2, C)
    err = (y.double().cpu() - y_ref).abs().max().item()
    assert err <= 1e-5 * y_ref.abs().max().item(), err
    y.backward(g.to(gpu))
    for name, p, r in zip(("dW0", "db0", "dW2", "db2"), ps, grads_ref):
        assert p.grad.shape == r.shape
        assert _rel(p.grad, r) <= 1e-5, (name, _rel(p.grad, r))


def test_subsample_deterministic(gpu):
    from onebit_asr.conv import _SubsampleFn

    torch.manual_seed(3)
    x = torch.randn(4, 120, 80, device=gpu)
    ps = [torch.randn(s, device=gpu) * 0.1 for s in ((144, 1, 3, 3), (144,), (144, 144, 3, 3),
                                                    (144,))]
    g = torch.randn(4, 29, 19, 144, device=gpu)
    outs = []
    for _ in range(2):
        qs = [p.clone().requires_grad_(True) for p in ps]
        y = _SubsampleFn.apply(x, *qs)
        y.backward(g)
        outs.append([y] + [q.grad for q in qs])
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_module_hip_equals_library_path(gpu, monkeypatch):
    """Conv2dSubsampling.forward through the HIP path == through MIOpen + the NCHW flatten
    (the Linear's column permutation is exact)."""
    from onebit_asr.conformer import Conv2dSubsampling

    torch.manual_seed(7)
    m = Conv2dSubsampling(80, 144).to(gpu)
    x = torch.randn(3, 101, 80, device=gpu)
    outs = {}
    for mode in ("hip", "miopen"):
        monkeypatch.setenv("OB_SUBSAMPLE", mode)
        m.zero_grad()
        y = m(x)
        y.square().sum().backward()
        outs[mode] = [y.detach()] + [p.grad.clone() for p in m.parameters()]
    for a, b in zip(outs["hip"], outs["miopen"]):
        assert ((a - b).norm() / b.norm()).item() <= 2e-5
