"""Packed-ternary checkpoint on the GPU: a model exported with the product's HIP pack and
reloaded into a fresh model gives bit-identical inference logits at bitwidths 2 and 1
(same codes, alpha, bias), its codes equal the oracle's Q(W/a) codes, and the stacked
PassBits forward also runs from the loaded codes (cfg1 size; Conformer-S size ratio)."""
import numpy as np
import pytest
import torch

from oracle.quant_oracle import np_codes

pytestmark = pytest.mark.gpu


def _build(cfg, gpu, seed):
    from onebit_asr.conformer import ConformerASR

    torch.manual_seed(seed)
    return ConformerASR(80, 5004, **cfg).to(gpu).eval()


def test_packed_round_trip_logits_bit_exact(gpu, tmp_path):
    from onebit_asr.checkpoint import _quant_layers, load_packed, save_packed
    from onebit_asr.data import CFG1, synthetic_batch

    src = _build(CFG1, gpu, 0)
    f = tmp_path / "cfg1.safetensors"
    save_packed(src, f)
    dst = load_packed(_build(CFG1, gpu, 1), f, device=gpu)
    batch = synthetic_batch([734, 349], [27, 12], seed=3, device=gpu)
    with torch.no_grad():
        for bits in (2, 1):
            _, m1, l1 = src(batch, precision=bits)
            _, m2, l2 = dst(batch, precision=bits)
            assert torch.equal(m1, m2)
            assert torch.equal(l1, l2), bits
    for name, m in _quant_layers(dst).items():
        s = dict(src.named_modules())[name]
        for b in (2, 1):
            c, ct = m._codes(b)
            wc, wct = np_codes(s.weight.detach().cpu().numpy(), float(s.alpha), b)
            assert np.array_equal(c.cpu().numpy().view(np.uint32), wc), (name, b)
            assert np.array_equal(ct.cpu().numpy().view(np.uint32), wct), (name, b)


def test_conformer_s_packed_size(gpu, tmp_path):
    from onebit_asr.checkpoint import _quant_layers, read_packed, save_packed
    from onebit_asr.data import CONFORMER_S

    model = _build(CONFORMER_S, gpu, 0)
    f = tmp_path / "s.safetensors"
    save_packed(model, f, bits=(2,))
    tensors, meta = read_packed(f)
    qw = sum(m.weight.numel() for m in _quant_layers(model).values())
    codes = sum(v.numel() * 4 for k, v in tensors.items() if ".codes" in k)
    assert codes <= qw * 2 / 8 * 1.13  # 2 bits per weight (+ row padding to 16)
    assert len(_quant_layers(model)) >= 16 * 4


def test_packed_model_refuses_training_on_fused_paths(gpu, tmp_path):
    """the fused FFN / q-k-v / out_proj call sites check the packed layers too, so
    a forward with grad enabled raises instead of training on placeholder weights."""
    from onebit_asr.checkpoint import load_packed, save_packed
    from onebit_asr.data import CFG1, synthetic_batch

    src = _build(CFG1, gpu, 0)
    f = tmp_path / "cfg1.safetensors"
    save_packed(src, f)
    dst = load_packed(_build(CFG1, gpu, 1), f, device=gpu).train()
    batch = synthetic_batch([400, 300], [20, 10], seed=3, device=gpu)
    with pytest.raises(RuntimeError, match="inference-only"):
        dst(batch, precision=2)
    # the packed layers' placeholder weights stay out of the state dict
    sd = dst.state_dict()
    assert "encoder.blocks.0.ff1.lin1.weight" not in sd
    assert "encoder.blocks.0.ff1.lin1.alpha" in sd
