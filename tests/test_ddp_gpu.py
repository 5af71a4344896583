"""The multi-rank GraphedTrainStep path on the GPU (untested): 2 ranks on
the box's GPU via torch.distributed.run, gloo exchange (tests/ddp_gpu_worker.py).
  * both graphs captured (graph A: zero flat grads + forward + backward; graph B: clip +
    FusedAdamW with grad_scale 1/world);
  * after the first step the flat buffer holds the SUM of the two shards' single-process
    gradients (rel-L2 <= 1e-5 per parameter; the all-reduce is the only exchange);
  * after two steps the replicas' parameters are bitwise identical."""
import os
import subprocess
import sys
from pathlib import Path

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parents[1]


def test_graphed_two_rank_step_gloo_on_gpu(gpu, tmp_path):
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={port}",
           str(ROOT / "tests" / "ddp_gpu_worker.py"), str(tmp_path)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = [torch.load(tmp_path / f"rank{k}.pt", weights_only=True) for k in range(2)]
    assert res[0]["graphed"] and res[1]["graphed"]
    for k, g in res[0]["summed"].items():
        ref = res[0]["local"][k].double() + res[1]["local"][k].double()
        assert torch.equal(g, res[1]["summed"][k]), k  # the all-reduce result is shared
        n = ref.norm().item()
        err = (g.double() - ref).norm().item()
        assert err <= 1e-5 * n + 1e-12, (k, err, n)
    for k, p in res[0]["params"].items():
        assert torch.equal(p, res[1]["params"][k]), k
