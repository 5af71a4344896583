#!/usr/bin/env python3
"""LayerNorm kernel timing at the Conformer-S shape (rows = 3 passes x 32 x 249, d = 144):
forward, backward with dgamma/dbeta, backward with dres + dy2 (dropout 0.1), graph-replayed
launches timed with HIP events on the launch stream (an older library: ONEBIT_HIP_LIB).
Usage: python tools/ln_bench.py [--reps 100]"""
import argparse
import ctypes
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "cmu-11785-idl-1.58bit-asr_amd"), str(ROOT / "tools")]

import torch  # noqa: E402

from kbench import timed  # noqa: E402
from onebit_asr import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=100)
    ap.add_argument("--rows", type=int, default=3 * 32 * 249)
    ap.add_argument("--d", type=int, default=144)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    lib = _lib.load()
    R, d = args.rows, args.d
    torch.manual_seed(0)
    x = torch.randn(R, d, device=dev)
    g = torch.randn(d, device=dev)
    b = torch.randn(d, device=dev)
    y = torch.empty_like(x)
    mean = torch.empty(R, device=dev)
    rstd = torch.empty(R, device=dev)
    dy = torch.randn_like(x)
    dres = torch.randn_like(x)
    dx = torch.empty_like(x)
    dy2 = torch.empty_like(x)
    dg = torch.empty(d, device=dev)
    db = torch.empty(d, device=dev)
    wsb = lib.ob_layernorm_bwd_workspace(R, d)
    ws = torch.empty(max(wsb, 4), dtype=torch.uint8, device=dev)
    rng = torch.tensor([1234, 0], dtype=torch.int64, device=dev)
    lens = torch.full((R // 249,), 249, dtype=torch.int32, device=dev)
    P = _lib.ptr

    def fwd(s=None):
        _lib.check(lib.ob_layernorm_fwd(x.data_ptr(), g.data_ptr(), b.data_ptr(), R, d, 1e-5,
                                        y.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                                        s or torch.cuda.current_stream().cuda_stream), "fwd")

    def bwd(s=None):
        _lib.check(lib.ob_layernorm_bwd(dy.data_ptr(), x.data_ptr(), g.data_ptr(), mean.data_ptr(),
                                        rstd.data_ptr(), R, d, dx.data_ptr(), dg.data_ptr(),
                                        db.data_ptr(), ws.data_ptr(), wsb,
                                        s or torch.cuda.current_stream().cuda_stream), "bwd")

    def bwd_ex(s=None):
        _lib.check(lib.ob_layernorm_bwd_ex(dy.data_ptr(), x.data_ptr(), g.data_ptr(),
                                           mean.data_ptr(), rstd.data_ptr(), R, d, dres.data_ptr(),
                                           dx.data_ptr(), dg.data_ptr(), db.data_ptr(),
                                           ws.data_ptr(), wsb, dy2.data_ptr(), 0.5, 0.1,
                                           rng.data_ptr(), 0, lens.data_ptr(), 249,
                                           s or torch.cuda.current_stream().cuda_stream), "bwd_ex")

    fwd()
    torch.cuda.synchronize()
    out = {"env": {k: v for k, v in os.environ.items() if k.startswith(("OB_LN", "ONEBIT"))}}
    for name, fn in (("fwd", fwd), ("bwd", bwd), ("bwd_ex", bwd_ex)):
        out[name + "_us"] = round(timed(fn, args.reps, True), 2)
    # checksums: bit-identical across settings is the expectation
    bwd_ex()
    fwd()
    torch.cuda.synchronize()
    out["sum"] = [float(t.double().sum()) for t in (y, mean, rstd, dx, dy2, dg, db)]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
