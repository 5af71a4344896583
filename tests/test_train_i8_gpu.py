"""The training step with absmax-int8 activations (act_quant="absmax_int8", the opt-in
north-star mode; not the reference's arithmetic, which keeps activations fp32 --
/root/reference/onebit_asr/quant.py:126) at cfg1, stacked passes:

* a captured forward+backward replays the eager int8 gradients of every parameter within
  rel-L2 1e-5 and the loss within rel 1e-6 (the int8 forward, its per-call absmax and the
  STE backward are graph-safe);
* the int8 step stays close to the reference-arithmetic (fp32-activation) step on the same
  model and batch: loss within 3% and the whole gradient vector at cosine >= 0.98 (the
  per-tensor int8 rounding is the only difference);
* GraphedTrainStep (``bench.py --mode train-i8``) replays == the same class run eagerly
  over 3 steps (losses rel <= 1e-5);
* ``bench.py --mode train-i8`` (small batch) prints its line with the int8-GEMM roofline.
Module-level int8 forward / backward parity against the numpy oracle is in
test_bitlinear_i8_gpu.py."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest
import torch

from _steputil import StepRunner, build, rel_errors

pytestmark = pytest.mark.gpu

MASKS = [[1, 0], [0, 1], [1, 1]]


def _cfg1():
    from onebit_asr.data import CFG1

    return CFG1


def _batch(gpu, seed=0):
    from onebit_asr.data import synthetic_batch

    return synthetic_batch([734, 349], [27, 12], seed=seed, device=gpu)


def _int8(model):
    from onebit_asr.quant import set_act_quant

    return set_act_quant(model, "absmax_int8")


def test_int8_step_replays_eager(gpu):
    model = _int8(build(_cfg1(), gpu))
    run = StepRunner(model, 2, _batch(gpu), [1, 0], stacked=True)
    l_e, parts_e, g_e = run.eager()
    run.capture()
    for r in range(2):
        l_r, parts_r, g_r = run.replay()
        assert abs(l_r.item() - l_e.item()) <= 1e-6 * abs(l_e.item()), (r, l_r, l_e)
        torch.testing.assert_close(parts_r, parts_e, rtol=1e-6, atol=1e-7)
        errs = rel_errors(g_r, g_e)
        worst = max(errs, key=errs.get)
        assert errs[worst] <= 1e-5, (r, worst, errs[worst])


def test_int8_step_close_to_fp32_activations(gpu):
    ref = StepRunner(build(_cfg1(), gpu), 2, _batch(gpu), [1, 1], stacked=True)
    l_f, _, g_f = ref.eager()
    got = StepRunner(_int8(build(_cfg1(), gpu)), 2, _batch(gpu), [1, 1], stacked=True)
    l_i, _, g_i = got.eager()
    assert abs(l_i.item() - l_f.item()) <= 3e-2 * abs(l_f.item()), (l_i.item(), l_f.item())
    keys = [k for k in g_f if g_f[k] is not None]
    assert all(g_i[k] is not None and torch.isfinite(g_i[k]).all() for k in keys)
    a = torch.cat([g_i[k].double().reshape(-1) for k in keys])
    b = torch.cat([g_f[k].double().reshape(-1) for k in keys])
    cos = torch.nn.functional.cosine_similarity(a, b, dim=0).item()
    assert cos >= 0.98, cos


def _graphed(gpu, use_graph):
    from onebit_asr.graph_step import GraphedTrainStep
    from onebit_asr.train_step import OneBitStep

    model = _int8(build(_cfg1(), gpu, seed=0))
    gs = GraphedTrainStep(OneBitStep(model, n_layers=2), n_layers=2, warmup_iters=2,
                          warmup_steps=4, total_steps=20, use_graph=use_graph)
    losses = [gs.step(_batch(gpu), m)[0].item() for m in MASKS]
    return gs, losses


def test_int8_graphed_train_step(gpu):
    gs_g, l_g = _graphed(gpu, True)
    assert gs_g.graph_a is not None and gs_g.steps_done == 3
    _, l_e = _graphed(gpu, False)
    assert all(torch.isfinite(torch.tensor(l_g)))
    for a, b in zip(l_g, l_e):
        assert abs(a - b) <= 1e-5 * abs(b), (l_g, l_e)


def test_bench_train_i8_line(gpu):
    root = Path(__file__).resolve().parents[1]
    cmd = [sys.executable, str(root / "bench.py"), "--mode", "train-i8", "--steps", "2",
           "--warmup", "1", "--batch", "4", "--frames", "600", "--tokens", "20"]
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    res = json.loads(lines[0])
    assert res["config"]["workload"] == "conformer-s-1.58bit-train-step-int8-act"
    assert res["value"] > 0 and "cpu_baseline" not in res
    roof = res["roofline"]
    assert roof["kernel"].startswith("tgemm_i8") and 0 < roof["frac"] < 1
    assert {s["layer"] for s in roof["shapes"]} == {"lin1", "lin2", "qkvo", "pos"}
