#!/usr/bin/env python3
"""Weight gradient of the V = 5004 linears (CTC head at [23904, 144], decoder output layer at
[3936, 144]): library fp32 g^T x (hipBLASLt) vs ob_dense_dw (bf16x6 register tiles, exact
fp32 products, fixed-order chunk sums). usage: python tools/ctc_dw_bench.py"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "cmu-11785-idl-1.58bit-asr_amd")]

import torch  # noqa: E402

from onebit_asr import _lib  # noqa: E402

dev = torch.device("cuda:0")
lib = _lib.load()


def t(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


for m in (23904, 3936):
    k, n = 144, 5004
    x = torch.randn(m, k, device=dev)
    g = torch.randn(m, n, device=dev)
    gw = torch.empty(n, k, device=dev)
    gb = torch.empty(n, device=dev)
    wsb = lib.ob_dense_dw_workspace(m, n, k)
    ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream().cuda_stream

    def ours():
        _lib.check(lib.ob_dense_dw(g.data_ptr(), x.data_ptr(), m, n, k, gw.data_ptr(), gb.data_ptr(),
                                   ws.data_ptr(), wsb, s), "ob_dense_dw")

    lib_us = t(lambda: g.t() @ x)
    ours_us = t(ours) if wsb else float("nan")
    ref = (g.double().t() @ x.double())
    rel = ((gw.double() - ref).norm() / ref.norm()).item() if wsb else float("nan")
    print(f"M={m}: library g^T x {lib_us:.1f} us, ob_dense_dw {ours_us:.1f} us (ws {wsb >> 20} MB, "
          f"rel-L2 vs float64 {rel:.2e})", flush=True)
