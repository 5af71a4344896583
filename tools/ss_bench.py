#!/usr/bin/env python3
"""Conv2dSubsampling C ABI at the Conformer-S training shape (B=32, T=1000, F=80, C=144):
pack + fwd + bwd, back-to-back, for rocprofv3 --stats (per-kernel times) or its own
wall-clock per call. Usage: python tools/ss_bench.py [--reps 10] [--C 144]"""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "cmu-11785-idl-1.58bit-asr_amd")]

import torch  # noqa: E402

from onebit_asr import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--B", type=int, default=32)
    ap.add_argument("--T", type=int, default=1000)
    ap.add_argument("--F", type=int, default=80)
    ap.add_argument("--C", type=int, default=144)
    a = ap.parse_args()
    lib = _lib.load()
    dev = torch.device("cuda:0")
    B, T, F, C = a.B, a.T, a.F, a.C
    t1, f1 = (T - 3) // 2 + 1, (F - 3) // 2 + 1
    t2, f2 = (t1 - 3) // 2 + 1, (f1 - 3) // 2 + 1
    x = torch.randn(B, T, F, device=dev)
    w0 = torch.randn(C, 1, 3, 3, device=dev) * 0.3
    b0 = torch.randn(C, device=dev) * 0.1
    w2 = torch.randn(C, C, 3, 3, device=dev) * 0.03
    b2 = torch.randn(C, device=dev) * 0.1
    img = torch.empty(lib.ob_subsample_image_bytes(C), dtype=torch.uint8, device=dev)
    y1 = torch.empty(B, t1, f1, C, device=dev)
    y2 = torch.empty(B, t2, f2, C, device=dev)
    g = torch.randn(B, t2, f2, C, device=dev)
    wsb = lib.ob_subsample_bwd_workspace(B, T, F, C)
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    dw0, db0 = torch.empty_like(w0), torch.empty_like(b0)
    dw2, db2 = torch.empty_like(w2), torch.empty_like(b2)
    st = torch.cuda.current_stream().cuda_stream

    def once():
        _lib.check(lib.ob_subsample_pack(w2.data_ptr(), C, img.data_ptr(), st), "pack")
        _lib.check(lib.ob_subsample_fwd(x.data_ptr(), B, T, F, C, w0.data_ptr(), b0.data_ptr(),
                                        img.data_ptr(), b2.data_ptr(), y1.data_ptr(),
                                        y2.data_ptr(), st), "fwd")
        _lib.check(lib.ob_subsample_bwd(x.data_ptr(), w0.data_ptr(), b0.data_ptr(), y1.data_ptr(),
                                        y2.data_ptr(), g.data_ptr(),
                                        B, T, F, C, img.data_ptr(), dw0.data_ptr(),
                                        db0.data_ptr(), dw2.data_ptr(), db2.data_ptr(),
                                        ws.data_ptr(), wsb, st), "bwd")

    for _ in range(2):
        once()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        once()
    e1.record()
    e1.synchronize()
    print(f"subsample pack+fwd+bwd B={B} T={T} F={F} C={C}: "
          f"{e0.elapsed_time(e1) * 1e3 / a.reps:.1f} us/call")


if __name__ == "__main__":
    main()
