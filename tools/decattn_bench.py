#!/usr/bin/env python3
"""The decoder attention core (ob_decattn_fwd / _bwd) alone at the training shapes: B = 96
(3 stacked passes x 32), H = 4, dh = 36, self-attention Lq = Lk = 41 and cross-attention
Lk = 250, dropout 0.1; graph-replayed launches timed with HIP events (kbench.timed).
Usage: python tools/decattn_bench.py [--reps 50]"""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "cmu-11785-idl-1.58bit-asr_amd"), str(ROOT / "tools")]

import torch  # noqa: E402

from kbench import timed  # noqa: E402
from onebit_asr import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    lib = _lib.load()
    B, H, dh, Lq = 96, 4, 36, 41
    e = H * dh
    rng = torch.tensor([1, 2], dtype=torch.int64, device=dev)
    for name, Lk, self_mode in (("self", 41, True), ("cross", 250, False)):
        xq = torch.randn(B, Lq, 3 * e if self_mode else e, device=dev)
        xkv = None if self_mode else torch.randn(B, Lk, 2 * e, device=dev)
        src = xq if self_mode else xkv
        sq = xq.shape[-1]
        skv = src.shape[-1]
        ko, vo = (e, 2 * e) if self_mode else (0, e)
        km = torch.zeros(B, Lk, dtype=torch.bool, device=dev)
        probs = torch.empty(B, H, Lq, Lk, device=dev)
        ctx = torch.empty(B, Lq, e, device=dev)
        dctx = torch.randn(B, Lq, e, device=dev)
        gq = torch.empty_like(xq)
        gs = torch.empty_like(src)

        def fwd(s=None):
            lib.ob_decattn_fwd(xq.data_ptr(), sq, src.data_ptr() + 4 * ko, skv,
                               src.data_ptr() + 4 * vo, skv, km.data_ptr(), int(self_mode), B, H,
                               Lq, Lk, dh, 0.1, rng.data_ptr(), 0, probs.data_ptr(), ctx.data_ptr(),
                               s or torch.cuda.current_stream().cuda_stream)

        def bwd(s=None):
            lib.ob_decattn_bwd(dctx.data_ptr(), ctx.data_ptr(), xq.data_ptr(), sq, src.data_ptr() + 4 * ko, skv,
                               src.data_ptr() + 4 * vo, skv, B, H, Lq, Lk, dh, 0.1,
                               probs.data_ptr(), gq.data_ptr(), sq, gs.data_ptr() + 4 * ko, skv,
                               gs.data_ptr() + 4 * vo, skv,
                               s or torch.cuda.current_stream().cuda_stream)

        fwd()
        torch.cuda.synchronize()
        print(f"{name:5s} Lk={Lk:3d}: fwd {timed(fwd, args.reps, True):7.2f} us  "
              f"bwd {timed(bwd, args.reps, True):7.2f} us")


if __name__ == "__main__":
    main()
