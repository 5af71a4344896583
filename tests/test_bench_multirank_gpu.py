"""``bench.py --gpus 2`` started as one process spawns its two ranks itself.

The box has one GPU, so the two ranks share it over gloo (``--dist-backend gloo``); the
8-GPU scaling runs use RCCL for the same exchange. Checks: the JSON line reports
n_gpus == 2 and dp2, the whole-job value counts both ranks' frames, and the replicas'
parameters are bitwise identical after the timed steps (graph A + all-reduce + graph B
on each rank). Reference step: onebit_asr/train.py:114-120.
"""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


@pytest.mark.gpu
def test_bench_gpus2_spawns_two_ranks(gpu):
    env = dict(os.environ, OMP_NUM_THREADS="4")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--batch", "4", "--frames", "600", "--tokens", "20", "--no-cpu-baseline",
           "--no-roofline", "--dist-backend", "gloo"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["config"]["parallelism"] == "dp2"
    assert res["replicas_bitwise_equal"] is True
    frames = 2 * 4 * 600 * 2
    assert abs(res["value"] - frames / (res["ms_per_step"] * 2 / 1e3)) <= 0.01 * res["value"]


def test_bench_rejects_world_mismatch():
    """No GPU needed: the check runs before anything touches the device."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "1"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE 1 != --gpus 2" in r.stderr
