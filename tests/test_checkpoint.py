"""CPU: the packed-ternary checkpoint container (onebit_asr/checkpoint.py) -- codes_t
derived from codes equals the oracle's (oracle/quant_oracle.py np_codes), a file written
with oracle codes loads into a fresh model with every tensor bit-exact, and misuse is
refused (non-packed files, bitwidth 32, grad-enabled forwards, architecture mismatch)."""
import json

import numpy as np
import pytest
import torch

from oracle.quant_oracle import np_codes


@pytest.mark.parametrize("n,k,bits", [(37, 53, 2), (37, 53, 1), (16, 16, 2), (144, 576, 2),
                                      (5, 1, 1)])
def test_transpose_codes_matches_oracle(n, k, bits):
    from onebit_asr.checkpoint import _transpose_codes

    rng = np.random.default_rng(n * k + bits)
    w = rng.standard_normal((n, k)).astype(np.float32) * 0.1
    codes, codes_t = np_codes(w, 0.08, bits)
    got = _transpose_codes(codes.view(np.int32), n, k)
    assert got.dtype == np.int32 and np.array_equal(got.view(np.uint32), codes_t)


def _model(seed):
    from onebit_asr.conformer import ConformerASR

    torch.manual_seed(seed)
    return ConformerASR(80, 37, enc_d_model=16, enc_layers=1, enc_heads=2, enc_d_ff=32,
                        enc_conv_kernel=3, enc_dropout=0.0, dec_layers=1, dec_heads=2,
                        dec_d_ff=32, dec_dropout=0.0)


def _write_oracle_file(model, path, bits=(2, 1)):
    """A packed file made with the oracle's codes (the product writes it from the GPU pack)."""
    from safetensors.torch import save_file

    from onebit_asr.checkpoint import FORMAT, _quant_layers

    layers = _quant_layers(model)
    tensors = {k: v.clone() for k, v in model.state_dict().items()
               if k not in {f"{n}.weight" for n in layers}}
    table = {}
    for name, m in layers.items():
        n, k = m.weight.shape
        for b in bits:
            c, _ = np_codes(m.weight.detach().numpy(), float(m.alpha), b)
            tensors[f"{name}.codes{b}"] = torch.from_numpy(c.view(np.int32).copy())
        table[name] = [n, k, m.bias is not None]
    save_file(tensors, str(path), metadata={"format": FORMAT, "bits": ",".join(map(str, bits)),
                                            "layers": json.dumps(table)})
    return tensors


def test_load_packed_round_trip(tmp_path):
    from onebit_asr.checkpoint import _quant_layers, load_packed

    src = _model(0)
    f = tmp_path / "m.safetensors"
    written = _write_oracle_file(src, f)
    dst = load_packed(_model(1), f)
    s_sd, d_sd = src.state_dict(), dst.state_dict()
    layers = _quant_layers(dst)
    for key, v in s_sd.items():
        if key.endswith(".weight") and key[:-7] in layers:
            continue
        assert torch.equal(d_sd[key], v), key
    for name, m in layers.items():
        n, k = m.weight.shape
        for b in (2, 1):
            c, ct = m._codes(b)
            want_c, want_ct = np_codes(s_sd[f"{name}.weight"].numpy(), float(s_sd[f"{name}.alpha"]), b)
            assert torch.equal(c, written[f"{name}.codes{b}"])
            assert np.array_equal(c.numpy().view(np.uint32), want_c)
            assert np.array_equal(ct.numpy().view(np.uint32), want_ct)
    # size: 2 bits per weight per bitwidth vs 32
    qbytes = sum(m.weight.numel() * 4 for m in layers.values())
    cbytes = sum(written[f"{n}.codes{b}"].numel() * 4 for n in layers for b in (2, 1))
    assert cbytes * 8 <= qbytes * 1.2


def test_packed_misuse_is_refused(tmp_path):
    from safetensors.torch import save_file

    from onebit_asr.checkpoint import load_packed, read_packed

    f = tmp_path / "plain.safetensors"
    save_file({"x": torch.zeros(2)}, str(f))
    with pytest.raises(ValueError):
        read_packed(f)
    g = tmp_path / "m.safetensors"
    _write_oracle_file(_model(0), g, bits=(2,))
    m = load_packed(_model(2), g)
    lin = m.encoder.blocks[0].ff1.lin1
    x = torch.randn(3, 16)
    with pytest.raises(RuntimeError, match="no fp32 weights"):
        with torch.no_grad():
            lin(x, 32)
    with pytest.raises(RuntimeError, match="inference-only"):
        lin(x, 2)
    with pytest.raises(KeyError):
        lin._codes(1)
    # a different architecture does not load
    from onebit_asr.conformer import ConformerASR

    other = ConformerASR(80, 37, enc_d_model=16, enc_layers=2, enc_heads=2, enc_d_ff=32,
                         enc_conv_kernel=3, enc_dropout=0.0, dec_layers=1, dec_heads=2,
                         dec_d_ff=32, dec_dropout=0.0)
    with pytest.raises(ValueError):
        load_packed(other, g)
    # an fp32 state dict replaces the packed codes
    lin.load_state_dict({"weight": torch.zeros(32, 16), "alpha": torch.tensor(0.1),
                         "bias": torch.zeros(32)})
    assert lin._packed is None
