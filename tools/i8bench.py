#!/usr/bin/env python3
"""The int8-operand BitLinear GEMM (ob_bitlinear_fwd_i8q) alone at the inference shapes
(B = 256 x 249 frames), per mode; HIP events around a graph of back-to-back launches.
usage: python tools/i8bench.py [--reps 20] [--only lin1_q8]"""
import argparse
import math
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "cmu-11785-idl-1.58bit-asr_amd")]

import torch  # noqa: E402

from onebit_asr import _lib  # noqa: E402
from onebit_asr.quant import pack_codes  # noqa: E402

M = 256 * 249
CASES = {  # name: (K, N, mode)
    "lin1_q8": (144, 576, 3), "lin1_plain": (144, 576, 0), "lin2_res": (576, 144, 2),
    "qkv_plain": (144, 144, 0),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default=None)
    a = ap.parse_args()
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    for name, (K, N, mode) in CASES.items():
        if a.only and name != a.only:
            continue
        g = torch.Generator(device=dev).manual_seed(K + N)
        xq = torch.randint(-127, 128, (M, K), device=dev, generator=g, dtype=torch.int32).to(torch.int8)
        W = (torch.rand(N, K, device=dev, generator=g) * 2 - 1) * (2 / math.sqrt(K))
        alpha = W.abs().mean()
        b = torch.zeros(N, device=dev)
        codes, _ = pack_codes(W, alpha, 2)
        R = torch.randn(M, N, device=dev, generator=g)
        Y = torch.empty(M, N, device=dev)
        amax = torch.full((1,), 4.0, device=dev)
        amax_out = torch.empty(1, device=dev)

        def fn(s):
            return lib.ob_bitlinear_fwd_i8q(xq.data_ptr(), 1, M, K, codes.data_ptr(), None, None,
                                            alpha.data_ptr(), 1, amax.data_ptr(), b.data_ptr(), N,
                                            mode, R.data_ptr(), 0.5, None, 0, amax_out.data_ptr(),
                                            Y.data_ptr(), s)

        side = torch.cuda.Stream(dev)
        with torch.cuda.stream(side):
            for _ in range(3):
                _lib.check(fn(side.cuda_stream), name)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, stream=side):
                for _ in range(a.reps):
                    fn(torch.cuda.current_stream(dev).cuda_stream)
            graph.replay()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(side)
            graph.replay()
            e1.record(side)
        e1.synchronize()
        print(f"{name:12s} K={K} N={N} mode={mode}: {e0.elapsed_time(e1) * 1e3 / a.reps:8.2f} us/call")


if __name__ == "__main__":
    main()
