#!/usr/bin/env python3
"""Time the fused rel-pos attention kernels at the Conformer-S training shape (3 stacked
passes x B=32 -> Bt = 96, T = 249, H = 4, d = 36, dropout 0.1). Usage:
python tools/attn_bench.py [--reps 20] [--op fwd|bwd] [--bt 96] [--p 0.1]"""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "cmu-11785-idl-1.58bit-asr_amd")]

import torch  # noqa: E402

from onebit_asr import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--op", default=None)
    ap.add_argument("--bt", type=int, default=96)
    ap.add_argument("--passes", type=int, default=3)
    ap.add_argument("--t", type=int, default=249)
    ap.add_argument("--p", type=float, default=0.1)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    lib = _lib.load()
    Bt, P, T, H, d = a.bt, a.passes, a.t, 4, 36
    C = H * d
    g = torch.Generator(device=dev).manual_seed(0)
    q, k, v, do = (torch.randn(Bt, T, C, device=dev, generator=g) for _ in range(4))
    pos = torch.randn(P, T, C, device=dev, generator=g)
    u, vb = torch.randn(H, d, device=dev) * 0.01, torch.randn(H, d, device=dev) * 0.01
    lens = torch.full((Bt,), T, dtype=torch.int32, device=dev)
    rng = torch.tensor([1234, 1], dtype=torch.int64, device=dev)
    saved = torch.empty(lib.ob_relattn_saved_elems(Bt, T, H, d), device=dev)
    ctx = torch.empty_like(q)
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    dpos, du, dvb = torch.empty_like(pos), torch.empty_like(u), torch.empty_like(vb)
    wsb = lib.ob_relattn_bwd_workspace(Bt, T, H, d)
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)

    def fwd(s):
        return lib.ob_relattn_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), pos.data_ptr(),
                                  u.data_ptr(), vb.data_ptr(), lens.data_ptr(), Bt, P, T, H, d, a.p,
                                  rng.data_ptr(), 0, saved.data_ptr(), None, ctx.data_ptr(), s)

    def bwd(s):
        return lib.ob_relattn_bwd(do.data_ptr(), ctx.data_ptr(), q.data_ptr(), k.data_ptr(), v.data_ptr(),
                                  pos.data_ptr(), u.data_ptr(), vb.data_ptr(), lens.data_ptr(), Bt,
                                  P, T, H, d, a.p, rng.data_ptr(), 0, saved.data_ptr(), saved.numel(),
                                  dq.data_ptr(),
                                  dk.data_ptr(), dv.data_ptr(), dpos.data_ptr(), du.data_ptr(),
                                  dvb.data_ptr(), ws.data_ptr(), wsb, s)

    s = torch.cuda.current_stream().cuda_stream
    for name, fn in (("fwd", fwd), ("bwd", bwd)):
        if a.op and a.op != name:
            if name == "fwd":
                _lib.check(fwd(s), "fwd")  # bwd needs the saved state
            continue
        for _ in range(2):
            _lib.check(fn(s), name)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            fn(s)
        e1.record()
        e1.synchronize()
        print(f"attn {name}: {e0.elapsed_time(e1) * 1e3 / a.reps:.1f} us per call", flush=True)


if __name__ == "__main__":
    main()
