"""int8-activation inference call sites (act_quant="absmax_int8", eval, no autograd):
the fused path -- LayerNorm emitting the per-tensor absmax (ob_layernorm_fwd_amax), lin1 on
the int8 matrix cores with swish and the next absmax in its epilogue, lin2 / out_proj with
the residual (and padded-frame zeroing) in theirs (ob_bitlinear_fwd_i8_epi) -- equals the
unfused module path (separate absmax passes, torch silu / add) bit for bit, and the
absmaxes equal the oracle's max|x|."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_layernorm_amax(gpu):
    from onebit_asr.layernorm import layer_norm, layer_norm_amax

    torch.manual_seed(0)
    for rows, d in [(1, 144), (1000, 144), (3 * 7968, 144), (37, 64)]:
        x = torch.randn(rows, d, device=gpu) * 3
        w, b = torch.randn(d, device=gpu), torch.randn(d, device=gpu)
        y = layer_norm_amax(x, w, b)
        ref = layer_norm(x, w, b)
        assert torch.equal(y, ref)
        assert y._ob_amax.item() == ref.abs().max().item()


@pytest.mark.parametrize("bits", [2, 1])
def test_ffn_i8_fused_equals_unfused(gpu, bits, monkeypatch):
    from onebit_asr.conformer import FeedForwardModule
    from onebit_asr.quant import set_act_quant

    torch.manual_seed(1)
    m = FeedForwardModule(144, 576, 0.1).to(gpu).eval()
    with torch.no_grad():
        for lin in (m.lin1, m.lin2):
            lin.bias.uniform_(-0.1, 0.1)
    set_act_quant(m, "absmax_int8")
    x = torch.randn(4, 249, 144, device=gpu)
    with torch.no_grad():
        monkeypatch.setenv("OB_FUSED", "1")
        y1 = m(x, bits)
        monkeypatch.setenv("OB_FUSED", "0")
        m.ln.emit_amax = False
        y0 = m(x, bits)
    assert torch.equal(y1, y0), (y1 - y0).abs().max().item()


def test_mhsa_i8_out_proj_residual(gpu, monkeypatch):
    """linear_residual_i8 with ragged lengths == out_proj (int8) + padded-row zeroing + x."""
    from onebit_asr.fused import linear_residual_i8
    from onebit_asr.quant import QuantizedLinear

    torch.manual_seed(2)
    lin = QuantizedLinear(144, 144, act_quant="absmax_int8").to(gpu)
    with torch.no_grad():
        lin.bias.uniform_(-0.1, 0.1)
    B, T = 3, 50
    lens = torch.tensor([50, 17, 1], dtype=torch.int32, device=gpu)
    ctx = torch.randn(B, T, 144, device=gpu)
    x = torch.randn(B, T, 144, device=gpu)
    with torch.no_grad():
        y = linear_residual_i8(ctx, x, lin, 2, 1.0, lens, T)
        valid = (torch.arange(T, device=gpu)[None, :] < lens[:, None]).float()
        ref = x + lin(ctx, 2) * valid[..., None]
    assert torch.equal(y, ref)
