"""CPU: pin the model-level oracle (oracle/conformer_oracle.py) against hand-derived known
answers for the reference's quirks (tests/golden/model_kat.json): rel_shift, the
label-smoothed CE's scalar-mean pad "mask", EOS placed after the padding, the
feat_lens // 4 frame mask clipped to T', and fully masked utterances through MHSA.
The product's CPU-capable pieces of the same quirks (rel_shift, make_att_targets,
att_ce_loss, subsampled_length) are checked against the same answers."""
import json
import math

import pytest
import torch

from oracle.conformer_oracle import OracleConformer, _rel_shift_gather, oracle_losses


@pytest.fixture(scope="module")
def kat(golden_dir):
    return json.loads((golden_dir / "model_kat.json").read_text())


def test_rel_shift_kat(kat):
    from onebit_asr.conformer import rel_shift

    for case in kat["rel_shift"]["cases"]:
        x = torch.tensor(case["x"], dtype=torch.float32)[None, None]
        want = torch.tensor(case["out"], dtype=torch.float32)[None, None]
        assert torch.equal(_rel_shift_gather(x), want)
        assert torch.equal(rel_shift(x), want)
        # batched / multi-head: every [b, h] slice shifts independently
        xb = torch.stack([x[0, 0], 10 * x[0, 0]])[None].repeat(3, 1, 1, 1)
        wb = torch.stack([want[0, 0], 10 * want[0, 0]])[None].repeat(3, 1, 1, 1)
        assert torch.equal(_rel_shift_gather(xb), wb)


def test_ce_scalar_mean_quirk(kat):
    from onebit_asr.losses import att_ce_loss

    k = kat["ce_scalar_mean"]
    logits = torch.tensor(k["logits"], dtype=torch.float64)
    tgt = torch.tensor(k["targets"])
    _, ce, _, _ = oracle_losses()
    got = ce(logits, tgt, k["pad_id"], k["label_smoothing"]).item()
    assert got == pytest.approx(k["loss"], rel=1e-7)  # the fp32 pad mask rounds it
    assert abs(got - k["pad_excluding_loss_would_be"]) > 0.1
    prod = att_ce_loss(logits, tgt, k["pad_id"], label_smoothing=k["label_smoothing"]).item()
    assert prod == pytest.approx(k["loss"], rel=1e-7)


def test_att_targets_eos_after_padding(kat):
    from onebit_asr.losses import make_att_targets

    k = kat["att_targets"]
    tokens = torch.tensor(k["tokens"])
    targets, _, _, _ = oracle_losses()
    for fn in (targets, make_att_targets):
        tin, tout, tpad = fn(tokens, k["bos"], k["eos"], k["pad"])
        assert tin.tolist() == k["tgt_inp"]
        assert tout.tolist() == k["tgt_out"]
        assert tpad.tolist() == k["tgt_pad_mask"]


def _tiny_oracle(seed=0, n_layers=1):
    """A small model in the reference's parameter layout (d=16, 2 heads, conv kernel 3)."""
    from onebit_asr.conformer import ConformerASR

    torch.manual_seed(seed)
    prod = ConformerASR(80, 37, enc_d_model=16, enc_layers=n_layers, enc_heads=2, enc_d_ff=32,
                        enc_conv_kernel=3, enc_dropout=0.0, dec_layers=1, dec_heads=2,
                        dec_d_ff=32, dec_dropout=0.0)
    return OracleConformer(prod.state_dict(), input_dim=80, vocab_size=37, d_model=16,
                           n_layers=n_layers, n_heads=2, d_ff=32, conv_kernel=3, dec_layers=1,
                           dec_heads=2, dec_d_ff=32)


def test_frame_mask_clip(kat):
    from onebit_asr.conformer import subsampled_length

    orc = _tiny_oracle()
    for case in kat["frame_mask"]["cases"]:
        assert subsampled_length(case["T"]) == case["T_sub"]
        lens = torch.tensor(case["feat_lens"])
        feats = torch.randn(len(lens), case["T"], 80)
        with torch.no_grad():
            enc, valid = orc.encode(feats, lens, precision=2)
        assert valid.shape == (len(lens), case["T_sub"])
        assert valid.sum(1).tolist() == case["valid"]
        # valid frames are a prefix
        for b, n in enumerate(case["valid"]):
            assert valid[b, :n].all() and not valid[b, n:].any()


def test_fully_masked_utterance_passes_mhsa_unchanged(kat):
    k = kat["masked_rows"]
    orc = _tiny_oracle(seed=1)
    lens = torch.tensor(k["feat_lens"])
    with torch.no_grad():
        # the encoder's first MHSA call, on the input the oracle gives it
        torch.manual_seed(2)
        x = torch.randn(len(lens), 1, 16)
        valid = torch.arange(1)[None, :] < torch.div(lens, 4, rounding_mode="floor")[:, None]
        mask = valid[:, :, None] & valid[:, None, :]
        pos = torch.zeros(1, 1, 16)
        for bits in (1, 2, 32):
            y = orc._mhsa(x, mask, bits, pos, "encoder.blocks.0.mhsa")
            u = k["masked_utterance"]
            assert torch.isfinite(y).all()
            assert torch.equal(y[u], x[u])
            assert not torch.equal(y[0], x[0])
        enc, valid2 = orc.encode(torch.randn(len(lens), k["T"], 80), lens, precision=2)
        assert torch.isfinite(enc).all() and valid2.sum().item() == 1


def test_kat_values_are_the_hand_formulas(kat):
    k = kat["ce_scalar_mean"]
    assert k["loss"] == pytest.approx(0.9847901, abs=1e-7)
    assert k["pad_excluding_loss_would_be"] == pytest.approx(math.log(2))
