"""GPU parity of the whole cfg1 model and three-pass step against the CPU oracle.

cfg1 (SURVEY §8d / BASELINE configs[0]): 2-block d_model=64 Conformer, V=5004, B=2 with
real utterance shapes [734, 349] frames / [27, 12] tokens, dropout 0. Bars:
  CTC logits max|err| <= 1e-3, CTC loss and step loss rel <= 1e-4,
  EVERY parameter gradient rel-L2 <= 1e-3 (alpha, a single cancellation-prone sum:
  <= 2e-3) -- QuantizedLinear layers, pos_bias_u/v, LayerNorms, conv module, subsampling,
  CTC head and decoder; parameters whose true gradient is zero (key biases, the
  depthwise bias before BatchNorm, the key third of the decoder's in_proj_bias) within
  1e-6 absolute.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

CFG1_ORACLE = dict(input_dim=80, vocab_size=5004, d_model=64, n_layers=2, n_heads=4, d_ff=256,
                   conv_kernel=31, dec_layers=2, dec_heads=4, dec_d_ff=1024, dropout=0.0)


@pytest.fixture(scope="module")
def pair(gpu):
    from onebit_asr.conformer import ConformerASR
    from onebit_asr.data import CFG1
    from oracle.conformer_oracle import OracleConformer

    torch.manual_seed(0)
    prod = ConformerASR(80, 5004, **CFG1).to(gpu)
    orc = OracleConformer(prod.state_dict(), **CFG1_ORACLE)
    return prod, orc


@pytest.fixture(scope="module")
def batch():
    from onebit_asr.data import synthetic_batch

    return synthetic_batch([734, 349], [27, 12], seed=0)


def _to(b, dev):
    return {k: v.to(dev) for k, v in b.items()}


@pytest.mark.parametrize("precision,sp_mask", [(2, None), (1, None), (2, [1, 0]), (32, None)])
def test_forward_parity(pair, batch, gpu, precision, sp_mask):
    from onebit_asr.losses import ctc_loss_from_logits

    prod, orc = pair
    with torch.no_grad():
        enc_p, mask_p, lg_p = prod(_to(batch, gpu), precision, sp_mask)
        enc_o, mask_o, lg_o = orc(batch, precision, sp_mask)
    assert torch.equal(mask_p.cpu(), mask_o)
    err = (lg_p.cpu() - lg_o).abs().max().item()
    assert err <= 1e-3, err
    lp = ctc_loss_from_logits(lg_p, mask_p.sum(1).long(), batch["tokens"].to(gpu),
                              batch["token_lens"].to(gpu), 3).item()
    lo = ctc_loss_from_logits(lg_o, mask_o.sum(1).long(), batch["tokens"], batch["token_lens"], 3).item()
    assert abs(lp - lo) <= 1e-4 * abs(lo), (lp, lo)


# parameters whose true gradient is zero (softmax shift invariance for key biases, a bias
# right before BatchNorm): both sides hold rounding noise there
ZERO_GRAD = ("k_proj.bias", "conv.dw.bias", "in_proj_bias")
BAR_QL = 1e-3      # QuantizedLinear weight / bias
BAR_ALPHA = 2e-3   # alpha: one cancellation-prone sum over N*K
BAR_OTHER = 1e-3   # every other parameter (LN, conv module, subsampling, heads, decoder)


def _bar(name):
    if name.endswith(".alpha"):
        return BAR_ALPHA
    if name.startswith("encoder.blocks.") and any(s in name for s in (".lin1.", ".lin2.", "_proj.")):
        return BAR_QL
    return BAR_OTHER


def test_step_loss_and_grads(pair, batch, gpu):
    from onebit_asr.train_step import OneBitStep
    from oracle.conformer_oracle import oracle_step_loss

    prod, orc = pair
    sp_mask = [1, 0]
    step = OneBitStep(prod, n_layers=2)
    prod.zero_grad(set_to_none=True)
    orc.zero_grad(set_to_none=True)
    loss_p, parts_p = step(_to(batch, gpu), sp_mask)
    loss_p.backward()
    loss_o, parts_o = oracle_step_loss(orc, batch, sp_mask)
    loss_o.backward()
    assert abs(loss_p.item() - loss_o.item()) <= 1e-4 * abs(loss_o.item())
    np.testing.assert_allclose(parts_p.cpu().numpy(), parts_o.numpy(), rtol=1e-4, atol=1e-6)
    ref = dict(orc.named_reference_parameters())
    worst = {}
    names = [n for n, _ in prod.named_parameters()]
    assert set(names) == set(ref), set(names) ^ set(ref)
    for name, p in prod.named_parameters():
        g_p = p.grad.detach().cpu().double()
        g_o = ref[name].grad.detach().double()
        d = g_p - g_o
        if any(z in name for z in ZERO_GRAD):
            if name.endswith("in_proj_bias"):  # only the key third is zero in truth
                e = g_o.numel() // 3
                for part in (slice(0, e), slice(2 * e, 3 * e)):
                    rel = d[part].norm().item() / max(g_o[part].norm().item(), 1e-12)
                    assert rel <= BAR_OTHER, (name, rel)
                d, g_o = d[e:2 * e], g_o[e:2 * e]
            # noise of two summation orders around a true zero: absolute, against the
            # gradient scale of the whole model
            assert d.abs().max().item() <= 1e-6, (name, d.abs().max().item())
            continue
        rel = d.norm().item() / max(g_o.norm().item(), 1e-12)
        bar = _bar(name)
        worst[name] = rel
        assert rel <= bar or d.abs().max().item() <= 1e-7, (name, rel, bar)
    assert len(worst) > 100


def test_train_step_runs_and_updates(gpu):
    """One optimizer step through the product step (clip + AdamW + schedule) changes weights
    and keeps everything finite."""
    from onebit_asr.conformer import ConformerASR
    from onebit_asr.data import CFG1, synthetic_batch
    from onebit_asr.train_step import OneBitStep, WarmupCosine, make_optimizer, train_step

    torch.manual_seed(1)
    model = ConformerASR(80, 5004, **CFG1).to(gpu)
    step = OneBitStep(model, n_layers=2)
    opt = make_optimizer(model.parameters())
    sched = WarmupCosine(opt, warmup_steps=10, total_steps=100)
    b = synthetic_batch([400, 300], [20, 10], seed=3, device=gpu)
    w0 = model.encoder.blocks[0].ff1.lin1.weight.detach().clone()
    for _ in range(2):
        loss, parts = train_step(step, opt, sched, b, [0, 1])
    assert torch.isfinite(loss).item() and torch.isfinite(parts).all().item()
    assert not torch.equal(w0, model.encoder.blocks[0].ff1.lin1.weight.detach())
