"""The training step captured as a HIP graph (onebit_asr/graph_step.py) at cfg1.

* replay == eager, per parameter, for the stacked step AND the reference's literal three
  forwards (train.py:82-111): three consecutive replays of one captured forward+backward
  (fixed parameters, dropout 0) reproduce the eager gradients of EVERY parameter within
  rel-L2 1e-5 (MIOpen's atomic weight-gradient convolutions are the only run-to-run
  noise, ~3e-7) and the loss / parts within rel 1e-6. Replays after the first are the ones
  that caught the ROCm graph-memset bug (onebit_asr/linear.py);
* GraphedTrainStep replay == the same class run eagerly over 4 steps, with a new SP mask
  and a new batch taking effect on replay: per-step loss and parts rel <= 1e-5;
  parameters: every element within 2*lr per step, and all but 0.5% of each tensor within
  1e-5 * max|p| + 1e-4 (Adam turns rounding-level differences of near-zero gradients into
  up to lr-sized steps; lr <= 5e-4 here);
* == the reference-order eager ``train_step`` (torch AdamW, Python-list SP mask), step for
  step: losses rel <= 1e-4 (capturable AdamW rounds its bias corrections differently);
* the first ``step()`` performs exactly one update (the warm-up before capture leaves no
  trace): parameters after it match one reference-order step.
"""
import pytest
import torch

from _steputil import StepRunner, build, rel_errors

pytestmark = pytest.mark.gpu

MASKS = [[1, 0], [0, 1], [1, 1], [0, 0]]


def _cfg1():
    from onebit_asr.data import CFG1

    return CFG1


def _batch(gpu, seed=0):
    from onebit_asr.data import synthetic_batch

    return synthetic_batch([734, 349], [27, 12], seed=seed, device=gpu)


@pytest.mark.parametrize("stacked", [True, False], ids=["stacked", "literal"])
def test_replay_reproduces_eager_gradients(gpu, stacked):
    model = build(_cfg1(), gpu)
    run = StepRunner(model, 2, _batch(gpu), [1, 0], stacked)
    l_e, parts_e, g_e = run.eager()
    run.capture()
    for r in range(3):
        l_r, parts_r, g_r = run.replay()
        assert abs(l_r.item() - l_e.item()) <= 1e-6 * abs(l_e.item()), (r, l_r, l_e)
        torch.testing.assert_close(parts_r, parts_e, rtol=1e-6, atol=1e-7)
        errs = rel_errors(g_r, g_e)
        assert len(errs) == sum(1 for g in g_e.values() if g is not None)
        worst = max(errs, key=errs.get)
        assert errs[worst] <= 1e-5, (r, worst, errs[worst])


def _run_graphed(gpu, use_graph):
    from onebit_asr.graph_step import GraphedTrainStep
    from onebit_asr.train_step import OneBitStep

    model = build(_cfg1(), gpu, seed=0)
    gs = GraphedTrainStep(OneBitStep(model, n_layers=2), n_layers=2, warmup_iters=2,
                          warmup_steps=4, total_steps=20, use_graph=use_graph)
    losses, parts = [], []
    batches = [_batch(gpu)] * 3 + [_batch(gpu, seed=1)]  # step 4 swaps the batch contents
    for mask, b in zip(MASKS, batches):
        loss, p = gs.step(b, mask)
        losses.append(loss.item())
        parts.append(p.clone())
    return model, gs, losses, parts


def test_graph_replay_matches_eager(gpu):
    m_g, gs_g, l_g, p_g = _run_graphed(gpu, True)
    assert gs_g.graph_a is not None and gs_g.steps_done == 4 and gs_g.sched.step_num == 4
    m_e, gs_e, l_e, p_e = _run_graphed(gpu, False)
    assert gs_e.graph_a is None
    for a, b in zip(l_g, l_e):
        assert abs(a - b) <= 1e-5 * abs(b), (l_g, l_e)
    for a, b in zip(p_g, p_e):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
    # parameters whose true gradient is zero (a bias before BatchNorm, key biases under the
    # softmax's shift invariance) move by lr-sized noise steps everywhere: max bound only
    zero_grad = ("conv.dw.bias", "k_proj.bias", "in_proj_bias")
    for (k, a), (_, b) in zip(m_g.named_parameters(), m_e.named_parameters()):
        diff = (a - b).abs()
        assert diff.max().item() <= 4 * 2 * 5e-4, (k, diff.max().item())
        if any(z in k for z in zero_grad):
            continue
        loose = (diff > 1e-5 * b.abs().max().item() + 1e-4).float().mean().item()
        assert loose <= 5e-3, (k, loose)


def test_graph_matches_reference_step_order(gpu):
    from onebit_asr.train_step import OneBitStep, WarmupCosine, make_optimizer, train_step

    _, _, l_g, _ = _run_graphed(gpu, True)
    model = build(_cfg1(), gpu, seed=0)
    step = OneBitStep(model, n_layers=2)
    opt = make_optimizer(model.parameters())
    sched = WarmupCosine(opt, 4, 20)
    batches = [_batch(gpu)] * 3 + [_batch(gpu, seed=1)]
    ref = []
    for mask, b in zip(MASKS, batches):
        loss, _ = train_step(step, opt, sched, b, mask)
        ref.append(loss.item())
    for a, b in zip(l_g, ref):  # step k of the graph path == step k of the reference order
        assert abs(a - b) <= 1e-4 * abs(b), (l_g, ref)
    assert l_g[-1] != l_g[-2]  # the swapped batch / mask changed the replayed step


def test_first_step_is_one_update(gpu):
    from onebit_asr.graph_step import GraphedTrainStep
    from onebit_asr.train_step import OneBitStep, WarmupCosine, make_optimizer, train_step

    m_g = build(_cfg1(), gpu, seed=0)
    gs = GraphedTrainStep(OneBitStep(m_g, n_layers=2), n_layers=2, warmup_iters=3,
                          warmup_steps=4, total_steps=20)
    gs.step(_batch(gpu), MASKS[0])
    assert gs.steps_done == 1 and gs.sched.step_num == 1
    m_r = build(_cfg1(), gpu, seed=0)
    opt = make_optimizer(m_r.parameters())
    train_step(OneBitStep(m_r, n_layers=2), opt, WarmupCosine(opt, 4, 20), _batch(gpu), MASKS[0])
    w0 = build(_cfg1(), gpu, seed=0)
    assert gs.opt.step_t.item() == 1.0
    zero_grad = ("conv.dw.bias", "k_proj.bias", "in_proj_bias")
    for (k, a), (_, b), (_, c) in zip(m_g.named_parameters(), m_r.named_parameters(),
                                      w0.named_parameters()):
        # one AdamW step (first step at the full lr, train.py quirk) moves an element by
        # <= lr (1 + wd |p|); the 3 warm-up steps would have moved it up to 3 lr more
        bound = 5e-4 * (1.0 + 1e-2 * c.abs().max().item()) * 1.01 + 1e-6
        assert (a - c).abs().max().item() <= bound, k
        if any(z in k for z in zero_grad):
            continue
        loose = ((a - b).abs() > 1e-5 * b.abs().max().item() + 1e-4).float().mean().item()
        assert loose <= 5e-3, (k, loose)
