#!/usr/bin/env python3
"""Per-kernel timing of the BitLinear C ABI at the Conformer-S shapes (HIP events on the
launch stream, back-to-back launches). Usage: python tools/kbench.py [--reps 50]"""
import argparse
import math
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "cmu-11785-idl-1.58bit-asr_amd")]

import torch  # noqa: E402

from onebit_asr import _lib  # noqa: E402
from onebit_asr.quant import pack_codes  # noqa: E402

SHAPES = [("lin1", 7968, 144, 576), ("lin2", 7968, 576, 144), ("qkvo", 7968, 144, 144),
          ("pos", 249, 144, 144)]


def timed(fn, reps, graph):
    """us per launch. graph=True replays `reps` captured launches (no host launch cost in
    the measured span, as in a captured training step)."""
    st = torch.cuda.current_stream()
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    if graph:
        g = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream()
        with torch.cuda.stream(side):
            with torch.cuda.graph(g, stream=side):
                cs = torch.cuda.current_stream().cuda_stream
                for _ in range(reps):
                    fn(cs)
        g.replay()
        torch.cuda.synchronize()
        run = g.replay
        n = reps
    else:
        run = lambda: [fn() for _ in range(reps)]  # noqa: E731
        n = reps
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record(st)
    run()
    e1.record(st)
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--no-graph", dest="graph", action="store_false")
    ap.add_argument("--shape", default=None, help="only this layer (lin1|lin2|qkvo|pos)")
    ap.add_argument("--op", default=None, help="only this op (pack|fwd|dx|dw)")
    ap.add_argument("--fused", action="store_true", help="also time the fused-epilogue entries")
    ap.add_argument("--passes", type=int, default=3,
                    help="stacked passes per launch (the training step runs 3; 0 = single-pass entries)")
    ap.add_argument("--i8", action="store_true",
                    help="also time the opt-in int8-activation forward (absmax + i8 MFMA GEMM)")
    ap.add_argument("--rows", type=int, default=0,
                    help="rows per pass for the M=7968 shapes (e.g. 63744 = configs[4] bs=256)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    lib = _lib.load()
    st = torch.cuda.current_stream(dev)
    s = st.cuda_stream
    print(f"{'layer':6s} {'M':>5s} {'K':>4s} {'N':>4s} | {'pack':>7s} {'fwd':>7s} {'dx':>7s} {'dw':>7s} us | fwd GB/s  dw GB/s")
    for name, M, K, N in SHAPES:
        if args.shape and name != args.shape:
            continue
        if args.rows and M == 7968:
            M = args.rows
        P = max(args.passes, 1)
        X = torch.randn(P * M, K, device=dev)
        dY = torch.randn(P * M, N, device=dev)
        W = (torch.rand(N, K, device=dev) * 2 - 1) * (2 / math.sqrt(K))
        alpha = W.abs().mean()
        b = torch.zeros(N, device=dev)
        codes, codes_t = pack_codes(W, alpha, 2)
        c1, c1t = pack_codes(W, alpha, 1)
        pbits = torch.tensor([2, 1, 1, 2][:P], dtype=torch.int32, device=dev)
        Y = torch.empty(P * M, N, device=dev)
        dX = torch.empty(P * M, K, device=dev)
        dW = torch.empty(N, K, device=dev)
        da = torch.empty((), device=dev)
        db = torch.empty(N, device=dev)
        wsb = lib.ob_bitlinear_bwd_dw_passes_workspace(P, M, N, K)
        ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
        fns = {
            "pack": lambda cs=s: lib.ob_quant_pack(W.data_ptr(), alpha.data_ptr(), 1, 2, N, K,
                                              codes.data_ptr(), codes_t.data_ptr(), cs),
            "fwd": lambda cs=s: lib.ob_bitlinear_fwd(X.data_ptr(), M, K, codes.data_ptr(), alpha.data_ptr(), 1,
                                                b.data_ptr(), N, Y.data_ptr(), cs),
            "dx": lambda cs=s: lib.ob_bitlinear_bwd_dx(dY.data_ptr(), M, N, codes_t.data_ptr(),
                                                  alpha.data_ptr(), 1, K, dX.data_ptr(), cs),
            "dw": lambda cs=s: lib.ob_bitlinear_bwd_dw(dY.data_ptr(), X.data_ptr(), M, N, K, W.data_ptr(),
                                                  alpha.data_ptr(), 1, 2, dW.data_ptr(), da.data_ptr(),
                                                  db.data_ptr(), ws.data_ptr(), wsb, cs),
        }
        if args.passes > 0:
            fns.update({
                "fwd": lambda cs=s: lib.ob_bitlinear_fwd_passes(
                    X.data_ptr(), P, M, K, codes.data_ptr(), c1.data_ptr(), pbits.data_ptr(),
                    alpha.data_ptr(), 1, b.data_ptr(), N, Y.data_ptr(), cs),
                "dx": lambda cs=s: lib.ob_bitlinear_bwd_dx_passes(
                    dY.data_ptr(), P, M, N, codes_t.data_ptr(), c1t.data_ptr(), pbits.data_ptr(),
                    alpha.data_ptr(), 1, K, dX.data_ptr(), cs),
                "dw": lambda cs=s: lib.ob_bitlinear_bwd_dw_passes(
                    dY.data_ptr(), X.data_ptr(), P, M, N, K, W.data_ptr(), alpha.data_ptr(), 1,
                    pbits.data_ptr(), dW.data_ptr(), da.data_ptr(), db.data_ptr(), ws.data_ptr(),
                    wsb, cs),
            })
        if args.passes > 0 and args.fused:
            Yp = torch.empty(P * M, N, device=dev)
            R = torch.randn(P * M, N, device=dev)
            pre = torch.randn(P * M, K, device=dev)
            rng = torch.tensor([1234, 5], dtype=torch.int64, device=dev)
            pd = 0.1
            # the step's residual epilogue zeroes rows past each utterance's length:
            # 249-row utterances (M = 32 x 249 at Conformer-S), ragged lengths
            Tq = 249 if M % 249 == 0 else M
            lens = torch.randint(Tq // 2, Tq + 1, (P * M // Tq,), dtype=torch.int32, device=dev)
            fns.update({
                "fswish": lambda cs=s: lib.ob_bitlinear_fwd_swish_drop(
                    X.data_ptr(), P, M, K, codes.data_ptr(), c1.data_ptr(), pbits.data_ptr(),
                    alpha.data_ptr(), 1, b.data_ptr(), N, pd, rng.data_ptr(), 0, Yp.data_ptr(),
                    Y.data_ptr(), cs),
                "fres": lambda cs=s: lib.ob_bitlinear_fwd_residual(
                    X.data_ptr(), P, M, K, codes.data_ptr(), c1.data_ptr(), pbits.data_ptr(),
                    alpha.data_ptr(), 1, b.data_ptr(), N, R.data_ptr(), 0.5, pd, rng.data_ptr(), 0,
                    None, 0, Y.data_ptr(), cs),
                "fresl": lambda cs=s: lib.ob_bitlinear_fwd_residual(
                    X.data_ptr(), P, M, K, codes.data_ptr(), c1.data_ptr(), pbits.data_ptr(),
                    alpha.data_ptr(), 1, b.data_ptr(), N, R.data_ptr(), 0.5, pd, rng.data_ptr(), 0,
                    lens.data_ptr(), Tq, Y.data_ptr(), cs),
                "dxswish": lambda cs=s: lib.ob_bitlinear_bwd_dx_swish_drop(
                    dY.data_ptr(), P, M, N, codes_t.data_ptr(), c1t.data_ptr(), pbits.data_ptr(),
                    alpha.data_ptr(), 1, K, pre.data_ptr(), pd, rng.data_ptr(), 0, dX.data_ptr(),
                    cs),
                "dropbwd": lambda cs=s: lib.ob_drop_scale_bwd(
                    dY.data_ptr(), P * M, N, 0.5, pd, rng.data_ptr(), 0, None, 0, R.data_ptr(), cs),
            })
        if args.i8:  # north_star's int8 path vs the fp32-exact bf16x3 forward, same shape
            amax = torch.empty(P, device=dev)
            wsa = lib.ob_act_absmax_workspace(P)
            wa = torch.empty(max(wsa, 1), dtype=torch.uint8, device=dev)
            fns.update({
                "absmax": lambda cs=s: lib.ob_act_absmax(X.data_ptr(), P, M * K, amax.data_ptr(),
                                                         wa.data_ptr(), wsa, cs),
                "fwd_i8": lambda cs=s: lib.ob_bitlinear_fwd_i8(
                    X.data_ptr(), P, M, K, codes.data_ptr(), c1.data_ptr(), pbits.data_ptr(),
                    alpha.data_ptr(), 1, amax.data_ptr(), b.data_ptr(), N, Y.data_ptr(), cs),
            })
        res = {}
        for k, fn in fns.items():
            res[k] = timed(fn, args.reps, args.graph) if (not args.op or k == args.op) else float("nan")
        gb_f = 4 * P * (M * K + M * N) / res["fwd"] / 1e3
        gb_w = 4 * P * (M * K + M * N) / res["dw"] / 1e3
        print(f"{name:6s} {M:5d} {K:4d} {N:4d} | {res['pack']:7.2f} {res['fwd']:7.2f} {res['dx']:7.2f} {res['dw']:7.2f} us | {gb_f:8.0f} {gb_w:8.0f}")
        if "fwd_i8" in res:
            gb_i8 = 4 * P * (M * K + M * N) / res["fwd_i8"] / 1e3
            tops = 2 * P * M * K * N / res["fwd_i8"] / 1e6
            print(f"{'':6s} int8: absmax {res['absmax']:7.2f}  fwd_i8 {res['fwd_i8']:7.2f} us "
                  f"({gb_i8:.0f} GB/s fp32-in/out, {tops:.1f} TOP/s)  vs bf16x3 fwd {res['fwd']:7.2f} us")
        if "fswish" in res:
            print(f"{'':6s} fused: fwd+swish {res['fswish']:7.2f}  fwd+residual {res['fres']:7.2f} "
                  f"(with lengths {res['fresl']:7.2f})  "
                  f"dx+swish-bwd {res['dxswish']:7.2f}  drop-scale-bwd {res['dropbwd']:7.2f} us")


if __name__ == "__main__":
    main()
