"""BASELINE configs[3] ("quant off: BitLinear -> bf16 nn.Linear"): ``set_quant_off`` turns
every QuantizedLinear into a plain F.linear in bf16 whatever the bitwidth. It is the
measurement ceiling for the ternary kernels (bench.py --mode quant-off), not a parity path:
the reference has no such mode (its bitwidth 32 is an fp32 F.linear, quant.py:121-122)."""
import pytest
import torch
import torch.nn.functional as F


def _layer(seed=0):
    from onebit_asr.quant import QuantizedLinear

    torch.manual_seed(seed)
    return QuantizedLinear(144, 576)


def test_quant_off_is_bf16_linear_cpu():
    from onebit_asr.quant import set_quant_off

    layer = _layer()
    with torch.no_grad():
        layer.bias.normal_()
    set_quant_off(layer, torch.bfloat16)
    x = torch.randn(5, 7, 144, requires_grad=True)
    for bits in (1, 2, 32):
        y = layer(x, bits)
        ref = F.linear(x.bfloat16(), layer.weight.bfloat16(), layer.bias.bfloat16()).float()
        assert y.dtype == torch.float32 and y.shape == (5, 7, 576)
        assert torch.equal(y, ref)
    layer(x, 2).sum().backward()
    assert layer.weight.grad is not None and layer.bias.grad is not None
    assert layer.alpha.grad is None  # no quantizer in the graph
    assert x.grad is not None


def test_quant_off_restore_and_validation_cpu():
    from onebit_asr.quant import set_quant_off

    layer = set_quant_off(_layer(), torch.bfloat16)
    set_quant_off(layer, None)
    assert layer.quant_off is None
    x = torch.randn(3, 144)
    assert torch.equal(layer(x, 32), F.linear(x, layer.weight, layer.bias))
    with pytest.raises(ValueError, match=r"bitwidth must be one of \{1,2,32\}"):
        layer(x, 4)


@pytest.mark.gpu
def test_quant_off_step_gpu(gpu):
    """The bench's quant-off step (stacked 3-pass body, bf16 library GEMMs) runs, its loss
    is finite, and no BitLinear kernel or alpha gradient is involved."""
    from onebit_asr.conformer import ConformerASR
    from onebit_asr.data import CFG1, synthetic_batch
    from onebit_asr.quant import QuantizedLinear, set_quant_off
    from onebit_asr.train_step import OneBitStep

    torch.manual_seed(0)
    model = set_quant_off(ConformerASR(80, 5004, **CFG1).to(gpu), torch.bfloat16)
    step = OneBitStep(model, n_layers=CFG1["enc_layers"])
    batch = {k: v.to(gpu) for k, v in synthetic_batch([400, 300], [20, 12], seed=0).items()}
    loss, parts = step(batch, [1, 0])
    loss.backward()
    torch.cuda.synchronize()
    assert torch.isfinite(loss).item() and torch.isfinite(parts).all().item()
    qls = [m for m in model.modules() if isinstance(m, QuantizedLinear)]
    assert qls and all(m.alpha.grad is None for m in qls)
    assert all(m.weight.grad is not None and torch.isfinite(m.weight.grad).all() for m in qls)


@pytest.mark.gpu
@pytest.mark.parametrize("N,K", [(576, 144), (144, 576), (144, 144), (100, 36)])
def test_quant_off_bf16w_layer_gpu(gpu, N, K):
    """set_quant_off(m, "bf16w"): the ternary GEMM kernels with B = bf16(W) (alpha_raw 2/3)
    == float64 x . bf16(W)^T + b (activations exact fp32); dX against float64 g . bf16(W);
    dW / db the plain dense gradient (no STE mask, no alpha gradient)."""
    from onebit_asr.quant import QuantizedLinear, set_quant_off

    torch.manual_seed(1)
    layer = QuantizedLinear(K, N).to(gpu)
    with torch.no_grad():
        layer.bias.uniform_(-0.1, 0.1)
    set_quant_off(layer, "bf16w")
    x = torch.randn(2, 300, K, device=gpu, requires_grad=True)
    g = torch.randn(2, 300, N, device=gpu)
    y = layer(x, 2)
    y.backward(g)
    wb = layer.weight.detach().bfloat16().double()
    ref = x.detach().double() @ wb.t() + layer.bias.detach().double()
    assert (y.double() - ref).abs().max().item() <= 1e-5 * ref.abs().max().item()
    dx = g.double() @ wb
    assert (x.grad.double() - dx).abs().max().item() <= 1e-5 * dx.abs().max().item()
    g2, x2 = g.reshape(-1, N).double(), x.detach().reshape(-1, K).double()
    dw = g2.t() @ x2
    rel = ((layer.weight.grad.double() - dw).norm() / dw.norm()).item()
    assert rel <= 1e-5, rel
    db = g2.sum(0)
    assert (layer.bias.grad.double() - db).abs().max().item() <= 1e-5 * db.abs().max().item()
    assert layer.alpha.grad is None


@pytest.mark.gpu
def test_quant_off_bf16w_fused_equals_module_gpu(gpu, monkeypatch):
    """A Conformer block in the bf16w quant-off mode: the fused call sites (FFN, q/k/v,
    out_proj) equal the module path on the same kernels -- outputs and every gradient."""
    from onebit_asr.conformer import ConformerBlock, RelPositionalEncoding
    from onebit_asr.quant import set_quant_off

    out = {}
    for fused in ("1", "0"):
        monkeypatch.setenv("OB_FUSED", fused)
        torch.manual_seed(2)
        blk = ConformerBlock(144, 576, 4, 31, 0.0, 0).to(gpu)
        set_quant_off(blk, "bf16w")
        x = torch.randn(2, 97, 144, device=gpu, requires_grad=True)
        _, pos = RelPositionalEncoding(144).to(gpu)(x)
        y = blk(x, None, 2, pos)
        # (a random upstream gradient: the block ends in a LayerNorm, whose input gradient
        # of sum(y) is zero up to rounding)
        y.backward(torch.randn(y.shape, generator=torch.Generator().manual_seed(3)).to(gpu))
        out[fused] = (y.detach(), x.grad.detach(),
                      {k: p.grad.detach() for k, p in blk.named_parameters() if p.grad is not None})
    y1, gx1, g1 = out["1"]
    y0, gx0, g0 = out["0"]
    assert (y1 - y0).abs().max().item() <= 1e-5 * y0.abs().max().item()
    assert (gx1 - gx0).abs().max().item() <= 1e-5 * gx0.abs().max().item()
    assert g1.keys() == g0.keys()
    scale = max(g.abs().max().item() for g in g0.values())
    for k in g0:
        err = (g1[k] - g0[k]).abs().max().item()
        if "k_proj.bias" in k or "dw.bias" in k:  # exact gradient 0 (softmax shift / BatchNorm)
            assert err <= 1e-6 * scale, (k, err)
            continue
        assert err <= 1e-4 * g0[k].abs().max().item() + 1e-7, (k, err)
