"""The overlapped deferred exchange's chunk plan (deferred._chunk_plan, CPU: pure bookkeeping
over the grouped launch's output pointers): chunks of whole gemms in descending flat-buffer
order, buckets that tile the buffer without a gap or an overlap, gemms sharing a parameter
(linear.linear_rows_split's row halves) kept in one chunk, outputs outside the buffer -> no
plan (one launch, the exchange after the backward)."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "cmu-11785-idl-1.58bit-asr_amd"))

from onebit_asr import deferred  # noqa: E402


class _X:
    def __init__(self, flat, chunks):
        self.flat, self.chunks = flat, chunks


def _gemm(base, w_off, n, k, b_off=None, a_off=None, m=100):
    g = deferred.DwgGemm()
    g.dW = base + 4 * w_off
    g.db = base + 4 * b_off if b_off is not None else None
    g.dalpha = base + 4 * a_off if a_off is not None else None
    g.N, g.K, g.M, g.P = n, k, m, 1
    return g


def _check_tiles(plan, n):
    chunks, rest = plan
    hi = n
    for gemms, lo, up in chunks:
        assert up == hi and lo < up
        hi = lo
    assert rest == hi


def test_plan_buckets_tile_the_buffer():
    flat = torch.zeros(10_000)
    b = flat.data_ptr()
    # params laid out: [pre 100] [L0 w 400, a 1, pad 3, b 20] ... five layers, then a tail
    gems, off = [], 100
    for _ in range(5):
        gems.append(_gemm(b, off, 20, 20, b_off=off + 404, a_off=off + 400))
        off += 424 + 4
    saved = deferred._S.dwg
    try:
        deferred._S.dwg = gems
        plan = deferred._chunk_plan(_X(flat, 3))
    finally:
        deferred._S.dwg = saved
    assert plan is not None
    _check_tiles(plan, flat.numel())
    chunks, rest = plan
    assert len(chunks) == 3 and rest <= 100
    launched = [g for gs, _, _ in chunks for g in gs]
    assert sorted(id(g) for g in launched) == sorted(id(g) for g in gems)
    assert [g.dW for g in launched] == sorted((g.dW for g in gems), reverse=True)


def test_plan_keeps_row_split_gemms_together():
    flat = torch.zeros(4_000)
    b = flat.data_ptr()
    # one packed [3e, e] weight at 0 (e = 8: 192 elements) and its bias at 192: two gemms
    # writing its row ranges; another layer after it
    e = 8
    q = _gemm(b, 0, e, e, b_off=192)
    kv = _gemm(b, e * e, 2 * e, e, b_off=192 + e)
    other = _gemm(b, 400, e, e, b_off=464)
    saved = deferred._S.dwg
    try:
        deferred._S.dwg = [q, kv, other]
        plan = deferred._chunk_plan(_X(flat, 3))
    finally:
        deferred._S.dwg = saved
    _check_tiles(plan, flat.numel())
    chunks, _ = plan
    where = {id(g): i for i, (gs, _, _) in enumerate(chunks) for g in gs}
    assert where[id(q)] == where[id(kv)]
    assert 1 <= len(chunks) <= 2


def test_plan_refuses_outputs_outside_the_buffer():
    flat = torch.zeros(1_000)
    b = flat.data_ptr()
    saved = deferred._S.dwg
    try:
        deferred._S.dwg = [_gemm(b, 0, 4, 4), _gemm(b, 990, 4, 4)]  # 16 elements past 990
        assert deferred._chunk_plan(_X(flat, 2)) is None
        assert "outside" in deferred.PLAN_NOTE
    finally:
        deferred._S.dwg = saved
