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
