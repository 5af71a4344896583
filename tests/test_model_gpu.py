"""GPU parity of the whole cfg1 model and three-pass step against the CPU oracle.

cfg1 (SURVEY §8d / BASELINE configs[0]): 2-block d_model=64 Conformer, V=5004, B=2 with
real utterance shapes [734, 349] frames / [27, 12] tokens, dropout 0. Bars:
  CTC logits max|err| <= 1e-3, CTC loss and step loss rel <= 1e-4,
  every QuantizedLinear parameter gradient rel-L2 <= 1e-3 (alpha, a single
  cancellation-prone sum: <= 2e-3).
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
    checked = 0
    for name, p in prod.named_parameters():
        if not name.startswith("encoder.blocks.") or not any(
                s in name for s in (".lin1.", ".lin2.", "_proj.")):
            continue
        g_p = p.grad.detach().cpu().double()
        g_o = ref[name].grad.detach().double()
        denom = g_o.norm().item()
        rel = (g_p - g_o).norm().item() / max(denom, 1e-12)
        # alpha gradients are single cancellation-prone sums (sum of G * term over N*K)
        bar = 2e-3 if name.endswith(".alpha") else 1e-3
        assert rel <= bar or (g_p - g_o).abs().max().item() <= 1e-7, (name, rel)
        checked += 1
    assert checked == 2 * 9 * 3  # weight, alpha, bias of 9 layers x 2 blocks


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
