"""The multi-rank step path on its real transport (RCCL never ran): at world size
1 over RCCL (graph_step._MULTI_RANK_PATH_AT_WORLD_1), in a child process
(tests/rccl_capture_worker.py):
  * both exchanges (the default deferred one and the bucketed one, several buckets) are
    captured into the step's single graph (no fallback to the eager exchange);
  * two graphed steps give the parameters of the single-GPU path (the one-rank all-reduce is
    an identity; the multi-rank path finishes its gradients on the spot instead of deferring
    them, which is bit-identical);
  * the same for the reference's literal three-pass body through the deferred exchange."""
import socket
import subprocess
import sys
from pathlib import Path

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parents[1]


def test_bucketed_allreduce_captured_over_rccl(gpu, tmp_path):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    r = subprocess.run([sys.executable, str(ROOT / "tests" / "rccl_capture_worker.py"),
                        str(tmp_path), str(port)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = torch.load(tmp_path / "result.pt", weights_only=True)
    assert res["multi"] and res["multi_deferred"] and not res["plain_multi"]
    assert res["captured"], "the bucketed RCCL all-reduce was not captured into the step graph"
    assert res["captured_deferred"], "the deferred exchange was not captured into the step graph"
    assert res["buckets"] > 2 and res["buckets_deferred"] == 0
    for key in ("p_multi", "p_deferred"):
        for k, p in res["p_plain"].items():
            q = res[key][k]
            err = (q.double() - p.double()).abs().max().item()
            assert err <= 1e-6 * max(p.abs().max().item(), 1e-30), (key, k, err)
    # the literal three-pass body: every parameter is used by three passes, so no gradient
    # site may write its flat slice in place (a pass's write clobbering another's)
    assert res["multi_literal"] and res["captured_literal"]
    for k, p in res["p_literal_plain"].items():
        q = res["p_literal"][k]
        err = (q.double() - p.double()).abs().max().item()
        assert err <= 1e-6 * max(p.abs().max().item(), 1e-30), ("p_literal", k, err)
