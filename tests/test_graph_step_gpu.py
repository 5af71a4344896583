"""GraphedTrainStep (the whole 3-pass step + clip + AdamW as one HIP graph) on cfg1.

* graph replay == the same step run eagerly: per-step loss and parts rel <= 1e-5;
  parameters: every element within 2*lr per step, and all but 0.5% of each tensor within
  1e-5 * max|p| + 1e-4 (Adam turns rounding-level differences of near-zero gradients into
  up to lr-sized steps; lr <= 5e-4 here);
* == the reference-order eager ``train_step`` (non-capturable AdamW, Python-list SP mask):
  losses rel <= 1e-4 (capturable AdamW rounds its bias corrections differently);
* a new SP mask and a new batch (same shape) take effect on replay without re-capture.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

MASKS = [[1, 0], [0, 1], [1, 1], [0, 0]]


def _model(gpu):
    from onebit_asr.conformer import ConformerASR
    from onebit_asr.data import CFG1

    torch.manual_seed(0)
    return ConformerASR(80, 5004, **CFG1).to(gpu)


def _batches(gpu):
    from onebit_asr.data import synthetic_batch

    b1 = synthetic_batch([734, 349], [27, 12], seed=0, device=gpu)
    b2 = synthetic_batch([734, 349], [27, 12], seed=1, device=gpu)
    return [b1, b1, b1, b2]  # step 4 swaps the batch contents


def _run_graphed(gpu, use_graph):
    from onebit_asr.graph_step import GraphedTrainStep
    from onebit_asr.train_step import OneBitStep

    model = _model(gpu)
    gs = GraphedTrainStep(OneBitStep(model, n_layers=2), n_layers=2, warmup_iters=2,
                          warmup_steps=4, total_steps=20, use_graph=use_graph)
    losses, parts = [], []
    batches = _batches(gpu)
    # first call primes: warmup_iters (=2) steps with MASKS[0]; then one step per call
    for mask, b in zip(MASKS, batches):
        loss, p = gs.step(b, mask)
        losses.append(loss.item())
        parts.append(p.clone())
    return model, gs, losses, parts


def test_graph_replay_matches_eager(gpu):
    m_g, gs_g, l_g, p_g = _run_graphed(gpu, True)
    assert gs_g.graph_a is not None and gs_g.steps_done == 5
    m_e, gs_e, l_e, p_e = _run_graphed(gpu, False)
    assert gs_e.graph_a is None
    for a, b in zip(l_g, l_e):
        assert abs(a - b) <= 1e-5 * abs(b), (l_g, l_e)
    for a, b in zip(p_g, p_e):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
    # MIOpen may pick other (deterministic) conv solvers under capture: rounding-level
    # gradient differences, which Adam turns into up to lr-sized steps where a gradient
    # element is ~0 (its sign is noise). Bound: every element within 2 * lr_max per step
    # (5 steps, lr <= 5e-4); all but 0.5% of each tensor within 1e-5 * max|p| + 1e-4.
    # Parameters whose true gradient is zero (a bias before BatchNorm, key biases under the
    # softmax's shift invariance) move by lr-sized noise steps everywhere: max bound only.
    zero_grad = ("conv.dw.bias", "k_proj.bias", "in_proj_bias")
    for (k, a), (_, b) in zip(m_g.named_parameters(), m_e.named_parameters()):
        diff = (a - b).abs()
        assert diff.max().item() <= 5 * 2 * 5e-4, (k, diff.max().item())
        if any(z in k for z in zero_grad):
            continue
        loose = (diff > 1e-5 * b.abs().max().item() + 1e-4).float().mean().item()
        assert loose <= 5e-3, (k, loose)


def test_graph_matches_reference_step_order(gpu):
    from onebit_asr.train_step import OneBitStep, WarmupCosine, make_optimizer, train_step

    _, _, l_g, _ = _run_graphed(gpu, True)
    model = _model(gpu)
    step = OneBitStep(model, n_layers=2)
    opt = make_optimizer(model.parameters())
    sched = WarmupCosine(opt, 4, 20)
    batches = _batches(gpu)
    ref = []
    for mask, b in zip([MASKS[0]] + MASKS, batches[:1] + batches):
        loss, _ = train_step(step, opt, sched, b, mask)
        ref.append(loss.item())
    # graphed: prime returns the 2nd warm-up step's loss, then steps 3..5
    ref_cmp = ref[1:]
    for a, b in zip(l_g, ref_cmp):
        assert abs(a - b) <= 1e-4 * abs(b), (l_g, ref_cmp)
    assert l_g[-1] != l_g[-2]  # the swapped batch / mask changed the replayed step
