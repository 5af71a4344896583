"""Opt-in ternary conv-module pointwise layers (north_star: "conv-module pointwise 1x1s" as
BitLinear call sites). The reference keeps pw1/pw2 full precision
(conformer.py:145,149,225), so the flag defaults off and the default model keeps the
reference's Conv1d keys. With the flag on, pw1/pw2 are QuantizedLinear layers at the block
bitwidth; their math is checked against the full-precision ConvModule whose pointwise
weights are the dequantized alpha*Q (quant.py:68), which is what the layer computes.

Bars (written here): forward max|err| <= 1e-5 * max|ref|, input-gradient rel-L2 <= 1e-5
(the same fp32 products; only summation order and the Conv1d vs GEMM kernels differ)."""
import pytest
import torch


def _rel(a, b):
    return float((a.detach().double() - b.detach().double()).norm()
                 / b.detach().double().norm().clamp_min(1e-30))


def test_default_keeps_reference_keys_cpu():
    from onebit_asr.conformer import ConformerASR
    from onebit_asr.data import CFG1

    m = ConformerASR(80, 100, **CFG1)
    sd = m.state_dict()
    assert sd["encoder.blocks.0.conv.pw1.weight"].shape == (128, 64, 1)
    assert "encoder.blocks.0.conv.pw1.alpha" not in sd


def test_flag_keys_and_precision32_cpu():
    """Flag on: QuantizedLinear keys; at bitwidth 32 the layer is F.linear on the fp weight,
    so the module equals the Conv1d module carrying the same weights."""
    from onebit_asr.conformer import ConvModule

    torch.manual_seed(0)
    q = ConvModule(64, 31, 0.0, quantize_pointwise=True).eval()
    f = ConvModule(64, 31, 0.0).eval()
    sd = q.state_dict()
    assert sd["pw1.weight"].shape == (128, 64) and sd["pw1.alpha"].dim() == 0
    assert sd["pw2.weight"].shape == (64, 64)
    with torch.no_grad():
        fsd = {k: v for k, v in sd.items() if not k.endswith("alpha")}
        fsd["pw1.weight"] = sd["pw1.weight"].unsqueeze(-1)
        fsd["pw2.weight"] = sd["pw2.weight"].unsqueeze(-1)
        f.load_state_dict(fsd)
    x = torch.randn(2, 37, 64)
    y_q = q(x, bitwidth=32)
    y_f = f(x)
    assert (y_q - y_f).abs().max() <= 1e-5 * y_f.abs().max()
    with pytest.raises(ValueError, match="bitwidth"):
        q(x)


@pytest.mark.gpu
@pytest.mark.parametrize("bits", [1, 2])
@pytest.mark.parametrize("fused", [True, False])
def test_ternary_pointwise_matches_dequantized_conv(gpu, bits, fused, monkeypatch):
    from onebit_asr.conformer import ConvModule
    from onebit_asr.quant import quantize_weight

    monkeypatch.setenv("OB_FUSED", "1" if fused else "0")
    torch.manual_seed(1)
    q = ConvModule(144, 31, 0.0, quantize_pointwise=True).to(gpu).eval()
    f = ConvModule(144, 31, 0.0).to(gpu).eval()
    with torch.no_grad():
        for lin in (q.pw1, q.pw2):
            lin.bias.uniform_(-0.1, 0.1)
        sd = q.state_dict()
        fsd = {k: v for k, v in sd.items() if not k.endswith("alpha")}
        for name in ("pw1", "pw2"):
            lin = getattr(q, name)
            w_hat = quantize_weight(lin.weight, lin.alpha.abs() + 1e-8, bits)
            fsd[f"{name}.weight"] = w_hat.unsqueeze(-1)
        f.load_state_dict(fsd)
    x = torch.randn(4, 249, 144, device=gpu)
    xq = x.clone().requires_grad_(True)
    xf = x.clone().requires_grad_(True)
    y_q = q(xq, bitwidth=bits)
    y_f = f(xf)
    assert (y_q - y_f).abs().max() <= 1e-5 * y_f.abs().max()
    g = torch.randn_like(y_f)
    (y_q * g).sum().backward()
    (y_f * g).sum().backward()
    assert _rel(xq.grad, xf.grad) <= 1e-5
    assert q.pw1.alpha.grad is not None and torch.isfinite(q.pw1.alpha.grad)
    assert q.pw2.weight.grad is not None and torch.isfinite(q.pw2.weight.grad).all()


@pytest.mark.gpu
def test_ternary_pointwise_stacked_step(gpu):
    """The three-pass stacked step runs with ternary pointwise layers (PassBits reach them)."""
    from onebit_asr.conformer import ConformerASR
    from onebit_asr.data import CFG1, synthetic_batch
    from onebit_asr.train_step import OneBitStep

    torch.manual_seed(0)
    model = ConformerASR(80, 5004, **CFG1, quantize_conv_pointwise=True).to(gpu)
    step = OneBitStep(model, n_layers=CFG1["enc_layers"])
    batch = {k: v.to(gpu) for k, v in synthetic_batch([400, 300], [20, 12], seed=0).items()}
    loss, parts = step(batch, [1, 0])
    loss.backward()
    torch.cuda.synchronize()
    assert torch.isfinite(loss).item() and torch.isfinite(parts).all().item()
    pw = model.encoder.blocks[0].conv.pw1
    assert pw.alpha.grad is not None and torch.isfinite(pw.alpha.grad).item()
