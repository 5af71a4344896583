"""Inference path: batched greedy CTC decode vs the oracle restatement of metrics.py:51-60,
and the graphed forward + decode vs the eager one (logits within 1e-4 * max|logit|; each
decode bit-exact against the oracle on its own logits)."""
import numpy as np
import pytest
import torch

from oracle.decode_oracle import np_ctc_greedy_decode, np_ctc_greedy_decode_batch

pytestmark = pytest.mark.gpu


def _check(out, cnt, ref):
    out, cnt = out.cpu().numpy(), cnt.cpu().numpy()
    for b, toks in enumerate(ref):
        assert cnt[b] == len(toks), (b, cnt[b], len(toks))
        assert out[b, :cnt[b]].tolist() == toks
        assert (out[b, cnt[b]:] == -1).all()


@pytest.mark.parametrize("B,T,V", [(1, 1, 5), (3, 17, 7), (8, 249, 5004), (2, 130, 64)])
def test_greedy_decode_matches_oracle(gpu, B, T, V):
    from onebit_asr.infer import ctc_greedy_decode_batch

    rng = np.random.default_rng(B * T + V)
    # few distinct logit levels -> many ties, repeats and blanks
    logits = rng.integers(0, 4, size=(B, T, V)).astype(np.float32)
    logits[..., 3] += rng.integers(0, 2, size=(B, T)).astype(np.float32) * 2  # blank often wins
    lens = rng.integers(0, T + 1, size=B)
    lens[0] = T
    out, cnt = ctc_greedy_decode_batch(torch.from_numpy(logits).to(gpu), torch.from_numpy(lens).to(gpu))
    _check(out, cnt, np_ctc_greedy_decode_batch(logits, lens))


def test_greedy_decode_reference_signature(gpu):
    from onebit_asr.infer import ctc_greedy_decode

    x = np.full((6, 5), -1.0, np.float32)
    for t, v in enumerate([4, 4, 3, 4, 2, 2]):  # a a _ a b b  ->  a a b
        x[t, v] = 1.0
    assert ctc_greedy_decode(torch.from_numpy(x).to(gpu)) == np_ctc_greedy_decode(x) == [4, 4, 2]


@pytest.mark.parametrize("act_quant", [None, "absmax_int8"])
def test_graphed_inference_matches_eager(gpu, act_quant):
    from onebit_asr.conformer import ConformerASR
    from onebit_asr.data import CFG1, synthetic_batch
    from onebit_asr.infer import GraphedInference, encode_and_decode
    from onebit_asr.quant import set_act_quant

    torch.manual_seed(0)
    model = ConformerASR(80, 5004, **CFG1).to(gpu).eval()
    b1 = synthetic_batch([734, 349], [27, 12], seed=0, device=gpu)
    b2 = synthetic_batch([734, 349], [27, 12], seed=1, device=gpu)
    gi = GraphedInference(model, precision=2, act_quant=act_quant)
    got = [tuple(t.clone() for t in gi.run(b)) for b in (b1, b2, b1)]
    set_act_quant(model, act_quant)
    for b, (out, cnt, logits) in zip((b1, b2, b1), got):
        e_out, e_cnt, e_logits = encode_and_decode(model, b, precision=2)
        # MIOpen may pick other conv solvers under capture: rounding-level differences
        err = (logits - e_logits).abs().max().item()
        assert err <= 1e-4 * e_logits.abs().max().item(), err
        lens = (b["feat_lens"] // 4).clamp(max=logits.size(1)).cpu().numpy()
        _check(out, cnt, np_ctc_greedy_decode_batch(logits.cpu().numpy(), lens))
        _check(e_out, e_cnt, np_ctc_greedy_decode_batch(e_logits.cpu().numpy(), lens))
