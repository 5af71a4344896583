#!/usr/bin/env python3
"""Benchmark: mel-frames/s of the Conformer-S 1.58-bit training step (BASELINE.json metric).

One "step" = the reference's full training step body (onebit_asr/train.py:82-120): the
2-bit teacher, 1-bit student and stochastic-precision passes with decoder and
CTC/CE/KL losses, backward, clip 5.0, AdamW, warmup-cosine -- on one synthetic padded
batch of B=32 utterances x 1000 frames x 80 mels per GPU (configs[1]; configs[2] for N>1
with one process per GPU, DDP gradient all-reduce over RCCL).

value = mel frames processed by ALL ranks / max-over-ranks wall time of the K timed steps.

Also reported:
  roofline     -- the dominant BitLinear kernel: algorithmic bytes/FLOPs per launch (step mix)
                  / its average launch duration, timed with HIP events on its stream;
  cpu_baseline -- the CPU oracle (oracle/conformer_oracle.py, a restatement of the
                  reference) on the host cores, bounded sample, rank 0 at N=1 only.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       torchrun --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import ctypes
import json
import math
import os
import platform
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
PKG = ROOT / "cmu-11785-idl-1.58bit-asr_amd"
for _p in (str(ROOT), str(PKG)):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

# gfx950 peaks (MI355X_MICROARCH.md, chip-level parameters)
PEAK_HBM_GBS = 8000.0
PEAK_FP32_MFMA_TFLOPS = 157.3

N_MELS, VOCAB = 80, 5004


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--frames", type=int, default=1000)
    ap.add_argument("--tokens", type=int, default=40)
    ap.add_argument("--eager", action="store_true",
                    help="run the step eagerly (DDP for N>1) instead of the captured HIP graph")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--traffic-json", default=str(ROOT / "profiles" / "pmc_traffic.json"))
    ap.add_argument("--roofline-only", action="store_true", help="skip the step timing")
    ap.add_argument("--branch-streams", action="store_true",
                    help="A/B: the decoder branch on a side stream beside the CTC branch "
                         "(OneBitStep branch_streams=True; measured slower, off by default)")
    ap.add_argument("--progress", action="store_true", help="progress lines on stderr")
    ap.add_argument("--mode", default="train",
                    choices=["train", "train-i8", "quant-off", "quant-off-lib", "infer",
                             "infer-fp32act"],
                    help="train: configs[1]/[2] (default); train-i8: the same step with "
                         "absmax-int8 activations on every BitLinear (opt-in north-star mode, "
                         "not the reference's arithmetic); quant-off: configs[3] (BitLinear -> "
                         "bf16 weights on the same fused kernels, set_quant_off 'bf16w'); "
                         "quant-off-lib: the same with bf16 library GEMMs (hipBLASLt); "
                         "infer / infer-fp32act: configs[4] (B=256, 2-bit, int8 / fp32 "
                         "activations, greedy CTC decode)")
    ap.add_argument("--conv-pw-ternary", action="store_true",
                    help="opt-in ternary conv-module pw1/pw2 (north_star; not reference math)")
    ap.add_argument("--conv-find", action="store_true",
                    help="torch.backends.cudnn.benchmark (MIOpen Find) for the subsampling convs")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="N>1 exchange: nccl (= RCCL, one GPU per rank) or gloo (ranks may "
                         "share a GPU: the -m gpu test of the multi-rank bench on a 1-GPU box)")
    args = ap.parse_args()
    if args.conv_find:
        torch.backends.cudnn.benchmark = True
    if args.mode.startswith("infer") and args.batch == 32:
        args.batch = 256  # configs[4]
    return args


# ------------------------------------------------------------------------- roofline
def ql_shapes(batch: int, frames: int, d: int = 144, d_ff: int = 576, layers: int = 16):
    """(name, M per pass, K, N, launches per step) of every BitLinear call in one step. The
    step runs the three passes stacked (OneBitStep stacked=True): one launch per kernel
    covers P = 3 passes, i.e. 3*M rows."""
    from onebit_asr.conformer import subsampled_length

    t = subsampled_length(frames)
    m = batch * t
    per_block = [("lin1", m, d, d_ff, 2), ("lin2", m, d_ff, d, 2), ("qkvo", m, d, d, 4),
                 ("pos", t, d, d, 1)]
    return [(n, M, K, N, c * layers) for (n, M, K, N, c) in per_block]


PASSES = 3
PASS_BITS = [2, 1, 1]  # teacher, student, an SP pass at 1 bit


def dwg_bitlinear_shapes(batch, frames):
    """(N, K, M per pass, P, bitlinear) of the BitLinear weight gradients of one step: the
    grouped launch's composition when no step has run (--roofline-only)."""
    out = []
    for _name, M, K, N, count in ql_shapes(batch, frames):
        for _ in range(count):
            out.append((N, K, M, PASSES, True, len(out)))
    return out


def roofline_dwg(dev, shapes, from_step, reps=5, log=lambda m: None, graph_replay=True):
    """The grouped weight-gradient launch (ob_dw_grouped: every deferred dW of a backward in
    ONE stream-K launch) with the composition the step's backward issued (deferred.LAST_DWG:
    the BitLinear dWs with their STE mask / dalpha, plus the full-precision dWs of the same
    launch), on fresh buffers (every gemm its own dY; X shared exactly where the step shares it,
    q / k / v of one LayerNorm output). Timed with HIP events around graph-replayed
    launches on the launch stream. Returns (us per launch, algorithmic bytes, FLOPs, MFMA
    cycles summed over SIMDs, detail)."""
    from onebit_asr import _lib, deferred

    lib = _lib.load()
    g = torch.Generator(device=dev).manual_seed(11)
    pmax = max(sh[3] for sh in shapes)
    bits_t = torch.tensor((PASS_BITS * pmax)[:pmax], dtype=torch.int32, device=dev)
    keep, descs = [], []
    by = fl = cyc = 0.0
    n_bl = 0
    t16 = lambda a: -(-a // 16)  # noqa: E731
    t32 = lambda a: -(-a // 32)  # noqa: E731
    xs = {}
    for i, (N, K, M, P, bl, xid) in enumerate(shapes):
        rows = P * M
        if xid == i:  # q / k / v of one LN output share X, as in the step
            xs[i] = torch.randn(rows, K, device=dev, generator=g)
        X = xs[xid]
        dY = torch.randn(rows, N, device=dev, generator=g)
        dW, db = torch.empty(N, K, device=dev), torch.empty(N, device=dev)
        W = alpha = da = None
        if bl:
            W = (torch.rand(N, K, device=dev, generator=g) * 2 - 1) * (2 / math.sqrt(K))
            alpha, da = W.abs().mean(), torch.empty((), device=dev)
            n_bl += 1
        keep += [X, dY, dW, db, W, alpha, da]
        descs.append(deferred.DwgGemm(dY.data_ptr(), X.data_ptr(), _lib.ptr(W), _lib.ptr(alpha),
                                      bits_t.data_ptr() if bl else None, dW.data_ptr(),
                                      db.data_ptr(), _lib.ptr(da), N, K, M, P, 1, 2))
        # dY, X read; dW (and db) written; a BitLinear also reads W (STE mask, dalpha)
        by += 4 * (rows * (N + K) + N * K * (2 if bl else 1) + N)
        fl += 2.0 * rows * N * K
        cyc += 16 * 6 * t16(N) * t16(K) * t32(rows)  # bf16x6: 6 16x16x32 MFMAs per block
    G = len(descs)
    arr = (deferred.DwgGemm * G)(*descs)
    ad = ctypes.addressof(arr)
    wsb = lib.ob_dw_grouped_workspace(ad, G)
    nt = lib.ob_dw_grouped_tickets(ad, G)
    if not wsb:
        raise RuntimeError("roofline: grouped dW composition not supported")
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    tk = torch.zeros(nt, dtype=torch.int32, device=dev)
    side = torch.cuda.Stream(dev)

    def fn(s):
        return lib.ob_dw_grouped(ad, G, ws.data_ptr(), wsb, tk.data_ptr(), nt, s)

    log(f"roofline dw_grouped: {G} gemms ({n_bl} BitLinear)")
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        for _ in range(2):
            _lib.check(fn(side.cuda_stream), "roofline warm-up")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if graph_replay:
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, stream=side):
                for _ in range(reps):
                    fn(torch.cuda.current_stream(dev).cuda_stream)
            graph.replay()
            e0.record(side)
            graph.replay()
            e1.record(side)
        else:  # eager launches (PMC passes: tools/dwg_bench.py)
            e0.record(side)
            for _ in range(reps):
                _lib.check(fn(side.cuda_stream), "roofline dw_grouped")
            e1.record(side)
    e1.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    detail = {"gemms": G, "bitlinear_gemms": n_bl, "us_per_launch": round(us, 1),
              "composition": ("the step's backward (deferred.LAST_DWG)" if from_step else
                              "the step's BitLinear dWs only (no step ran)")}
    del keep
    return us, by, fl, cyc, detail


def roofline(batch, frames, dev, reps=20, log=lambda m: None, dwg_shapes=None):
    """Time each BitLinear kernel family at the step's stacked shapes with HIP events on the
    launch stream (kernels captured in a HIP graph and replayed, so the events bracket
    device time, not Python launch gaps). The forward / dX ternary GEMMs are one family of
    launches (272 a step); the weight gradients are ONE grouped launch a step (ob_dw_grouped,
    timed at the composition the step issued). The line's roofline is the dominant KERNEL --
    the one with the most time per step: the grouped dW launch whenever it takes more than the
    whole ternary family would in one kernel's share, i.e. more than any single ternary launch
    kind (roofline_fused) -- against its roof; both families are listed. Algorithmic bytes /
    FLOPs per launch are counted for the P passes one launch covers."""
    from onebit_asr import _lib
    from onebit_asr.quant import pack_codes

    lib = _lib.load()
    P = PASSES
    fam = {"ternary_gemm": [0.0, 0.0, 0.0, 0, 0.0], "dw_grouped": [0.0, 0.0, 0.0, 0, 0.0]}
    # fam value: [total_time_us_per_step, total_bytes_per_step, total_flops_per_step, launches,
    #             MFMA pipe cycles per step summed over SIMDs]
    detail = []
    side = torch.cuda.Stream(dev)
    bits_t = torch.tensor(PASS_BITS, dtype=torch.int32, device=dev)
    for name, M, K, N, count in ql_shapes(batch, frames):
        g = torch.Generator(device=dev).manual_seed(M + K + N)
        X = torch.randn(P * M, K, device=dev, generator=g)
        dY = torch.randn(P * M, N, device=dev, generator=g)
        W = (torch.rand(N, K, device=dev, generator=g) * 2 - 1) * (2 / math.sqrt(K))
        alpha = W.abs().mean()
        b = torch.zeros(N, device=dev)
        c2, c2t = pack_codes(W, alpha, 2)
        c1, c1t = pack_codes(W, alpha, 1)
        Y = torch.empty(P * M, N, device=dev)
        dX = torch.empty(P * M, K, device=dev)

        def fwd(s):
            return lib.ob_bitlinear_fwd_passes(X.data_ptr(), P, M, K, c2.data_ptr(), c1.data_ptr(),
                                               bits_t.data_ptr(), alpha.data_ptr(), 1, b.data_ptr(),
                                               N, Y.data_ptr(), s)

        def bdx(s):
            return lib.ob_bitlinear_bwd_dx_passes(dY.data_ptr(), P, M, N, c2t.data_ptr(),
                                                  c1t.data_ptr(), bits_t.data_ptr(),
                                                  alpha.data_ptr(), 1, K, dX.data_ptr(), s)

        def timed(fn):
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                for _ in range(3):
                    _lib.check(fn(side.cuda_stream), "roofline warm-up")
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph, stream=side):
                    for _ in range(reps):
                        fn(torch.cuda.current_stream(dev).cuda_stream)
                graph.replay()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(side)
                graph.replay()
                e1.record(side)
            e1.synchronize()
            return e0.elapsed_time(e1) * 1e3 / reps  # us per launch

        log(f"roofline {name}: fwd")
        t_f = timed(fwd)
        log(f"roofline {name}: dx")
        t_dx = timed(bdx)
        cw = 4 * N * ((K + 15) // 16)
        rows = P * M
        by_f = 4 * (rows * K + rows * N + N) + 2 * cw      # X, Y, bias, codes (2 bitwidths)
        by_dx = 4 * (rows * N + rows * K) + 2 * cw          # dY, dX, codes_t
        fl = 2.0 * rows * K * N
        n_dx = 0 if name == "pos" else count  # pos_emb needs no input gradient
        # MFMA instructions the kernels issue: v_mfma_f32_16x16x32_bf16 (16 cycles per SIMD,
        # MI355X_MICROARCH.md cycle constants), 3 per 16x16x32 block in the bf16x3 ternary
        # GEMM (fwd: K padded to 32; dX: N padded), 6 in the bf16x6 dW
        t16 = lambda a: -(-a // 16)  # noqa: E731
        t32 = lambda a: -(-a // 32)  # noqa: E731
        cyc_f = 16 * 3 * t16(rows) * t16(N) * t32(K)
        cyc_dx = 16 * 3 * t16(rows) * t16(K) * t32(N)
        f = fam["ternary_gemm"]
        f[0] += count * t_f + n_dx * t_dx
        f[1] += count * by_f + n_dx * by_dx
        f[2] += (count + n_dx) * fl
        f[3] += count + n_dx
        f[4] += count * cyc_f + n_dx * cyc_dx
        detail.append({"layer": name, "M_per_pass": M, "passes": P, "K": K, "N": N,
                       "launches_per_step": count, "fwd_us": round(t_f, 2),
                       "dx_us": round(t_dx, 2)})
    shapes = dwg_shapes or dwg_bitlinear_shapes(batch, frames)
    t_g, by_g, fl_g, cyc_g, det_g = roofline_dwg(dev, shapes, bool(dwg_shapes), log=log)
    fam["dw_grouped"] = [t_g, by_g, fl_g, 1, cyc_g]
    # the dominant kernel: one grouped dW launch vs the ternary family's launches (the
    # largest single ternary launch kind is well below the family total)
    dom = "dw_grouped" if t_g >= fam["ternary_gemm"][0] / 6 else "ternary_gemm"
    t_us, by, fl, n, cyc = fam[dom]
    avg_t = t_us / n
    gbs = (by / n) / (avg_t * 1e-6) / 1e9
    tfs = (fl / n) / (avg_t * 1e-6) / 1e12
    # The ternary GEMM streams fp32 activations against 2-bit weights: HBM-bound by
    # construction (its exact-fp32 bf16x3 MFMA work is far below the bf16 roof). The dW GEMM
    # is a dense fp32 x fp32 product (exact via bf16x6): priced against the fp32 dense
    # MFMA peak of its dtype unless its bytes take longer at the HBM peak.
    bound_mfma = dom != "ternary_gemm" and (
        (fl / PEAK_FP32_MFMA_TFLOPS / 1e12) > (by / PEAK_HBM_GBS / 1e9))
    if bound_mfma:
        roof = {"bound": "mfma", "achieved": round(tfs, 2), "peak": PEAK_FP32_MFMA_TFLOPS,
                "unit": "TFLOP/s", "frac": round(tfs / PEAK_FP32_MFMA_TFLOPS, 4)}
    else:
        roof = {"bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": round(gbs / PEAK_HBM_GBS, 4)}
    # MFMA-busy (north_star: "MFMA-busy against gfx950 peak"): the MFMA pipe cycles the
    # family's instructions take, over the 1024 SIMDs x 2.4 GHz x its measured time
    mfma_busy = cyc / 1024 / (t_us * 1e-6 * 2.4e9)
    # both families against both roofs (the dominant one is the line's roofline)
    fams = {}
    for k, (ft, fb, ff, fn_, _c) in fam.items():
        if fn_:
            fams[k] = {"ms_per_step": round(ft / 1e3, 3), "launches_per_step": fn_,
                       "frac_hbm": round((fb / ft * 1e6) / 1e9 / PEAK_HBM_GBS, 4)}
            if k != "ternary_gemm":  # (2-bit weights: no fp32 x fp32 product to price)
                fams[k]["frac_fp32_mfma"] = round((ff / ft * 1e6) / 1e12 / PEAK_FP32_MFMA_TFLOPS, 4)
    roof["families"] = fams
    roof.update({"kernel": dom, "avg_launch_us": round(avg_t, 3),
                 "mfma_busy": round(mfma_busy, 4),
                 "mfma_busy_basis": "issued v_mfma_f32_16x16x32_bf16 cycles (16/SIMD each: 3 per "
                                    "block bf16x3, 6 bf16x6) / (1024 SIMDs x 2.4 GHz x time); "
                                    "PMC SQ_VALU_MFMA_BUSY_CYCLES in profiles/r3/pmc_step_*.md",
                 "bytes_per_launch": int(by / n), "flops_per_launch": int(fl / n),
                 "achieved_GBs": round(gbs, 1), "achieved_TFLOPs": round(tfs, 2),
                 "ql_kernel_ms_per_step": {k: round(v[0] / 1e3, 3) for k, v in fam.items()},
                 "dw_grouped": det_g, "shapes": detail})
    return roof


def roofline_fused(batch, frames, dev, reps=20, log=lambda m: None):
    """The ternary GEMM launches as the step issues them (stacked P = 3 passes, dropout 0.1):
    fused swish / residual / swish-backward epilogues, the k/v dX accumulations and the plain
    q / out launches, each timed like roofline() and priced at its algorithmic bytes (every
    operand read once, every output written once, fp32)."""
    from onebit_asr import _lib
    from onebit_asr.conformer import subsampled_length
    from onebit_asr.quant import pack_codes

    lib = _lib.load()
    P = PASSES
    m = batch * subsampled_length(frames)
    rows = P * m
    d, f = 144, 576
    bits_t = torch.tensor(PASS_BITS, dtype=torch.int32, device=dev)
    rng = torch.tensor([1234, 1], dtype=torch.int64, device=dev)
    side = torch.cuda.Stream(dev)
    g = torch.Generator(device=dev).manual_seed(7)

    def codes(N, K):
        W = (torch.rand(N, K, device=dev, generator=g) * 2 - 1) * (2 / math.sqrt(K))
        a = W.abs().mean()
        c2, c2t = pack_codes(W, a, 2)
        c1, c1t = pack_codes(W, a, 1)
        return c2, c1, c2t, c1t, a

    T = lambda *shape: torch.randn(*shape, device=dev, generator=g)  # noqa: E731
    x144, x576, y144, y576 = T(rows, d), T(rows, f), T(rows, d), T(rows, f)
    pre, o576, o144, gh = T(rows, f), T(rows, f), T(rows, d), T(rows, d)
    b144, b576 = torch.zeros(d, device=dev), torch.zeros(f, device=dev)
    c1 = codes(f, d)  # lin1 [576, 144]
    c2 = codes(d, f)  # lin2 [144, 576]
    cq = codes(d, d)
    bp = bits_t.data_ptr()
    qkv_out = [T(rows, d) for _ in range(3)]
    qkv = [_lib.ptr_array(v) for v in ([cq[0].data_ptr()] * 3, [cq[1].data_ptr()] * 3,
                                        [cq[4].data_ptr()] * 3, [b144.data_ptr()] * 3,
                                        [y.data_ptr() for y in qkv_out])]
    variants = [  # (name, launches per step, algorithmic bytes, fn(stream))
        ("lin1 fwd + swish + dropout (stores pre and act)", 32, 4 * rows * (d + 2 * f),
         lambda s: lib.ob_bitlinear_fwd_swish_drop(
             x144.data_ptr(), P, m, d, c1[0].data_ptr(), c1[1].data_ptr(), bp, c1[4].data_ptr(), 1,
             b576.data_ptr(), f, 0.1, rng.data_ptr(), 0, pre.data_ptr(), o576.data_ptr(), s)),
        ("lin2 fwd + dropout + 0.5 residual", 32, 4 * rows * (f + 2 * d),
         lambda s: lib.ob_bitlinear_fwd_residual(
             x576.data_ptr(), P, m, f, c2[0].data_ptr(), c2[1].data_ptr(), bp, c2[4].data_ptr(), 1,
             b144.data_ptr(), d, y144.data_ptr(), 0.5, 0.1, rng.data_ptr(), 0, None, 0,
             o144.data_ptr(), s)),
        ("lin2 dX + dropout / swish backward", 32, 4 * rows * (d + 2 * f),
         lambda s: lib.ob_bitlinear_bwd_dx_swish_drop(
             y144.data_ptr(), P, m, d, c2[2].data_ptr(), c2[3].data_ptr(), bp, c2[4].data_ptr(), 1,
             f, pre.data_ptr(), 0.1, rng.data_ptr(), 0, o576.data_ptr(), s)),
        ("lin1 dX", 32, 4 * rows * (f + d),
         lambda s: lib.ob_bitlinear_bwd_dx_passes(
             y576.data_ptr(), P, m, f, c1[2].data_ptr(), c1[3].data_ptr(), bp, c1[4].data_ptr(), 1,
             d, o144.data_ptr(), s)),
        ("q / k / v fwd (one grouped launch)", 16, 4 * rows * 4 * d,
         lambda s: lib.ob_bitlinear_fwd_passes_group(
             3, x144.data_ptr(), P, m, d, ctypes.addressof(qkv[0]), ctypes.addressof(qkv[1]), bp,
             ctypes.addressof(qkv[2]), 1, ctypes.addressof(qkv[3]), d, ctypes.addressof(qkv[4]),
             s)),
        ("k / v dX accumulated into q's (residual epilogue)", 32, 4 * rows * 3 * d,
         lambda s: lib.ob_bitlinear_fwd_residual(
             y144.data_ptr(), P, m, d, cq[2].data_ptr(), cq[3].data_ptr(), bp, cq[4].data_ptr(), 1,
             None, d, gh.data_ptr(), 1.0, 0.0, None, 0, None, 0, gh.data_ptr(), s)),
        ("q / out_proj dX", 32, 4 * rows * 2 * d,
         lambda s: lib.ob_bitlinear_bwd_dx_passes(
             y144.data_ptr(), P, m, d, cq[2].data_ptr(), cq[3].data_ptr(), bp, cq[4].data_ptr(), 1,
             d, o144.data_ptr(), s)),
        ("out_proj fwd + dropout + residual", 16, 4 * rows * 3 * d,
         lambda s: lib.ob_bitlinear_fwd_residual(
             x144.data_ptr(), P, m, d, cq[0].data_ptr(), cq[1].data_ptr(), bp, cq[4].data_ptr(), 1,
             b144.data_ptr(), d, y144.data_ptr(), 1.0, 0.1, rng.data_ptr(), 0, None, 0,
             o144.data_ptr(), s)),
    ]
    out = []
    tot_t = tot_b = 0.0
    for name, count, by, fn in variants:
        log(f"roofline in-step: {name}")
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(3):
                _lib.check(fn(side.cuda_stream), name)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, stream=side):
                for _ in range(reps):
                    fn(torch.cuda.current_stream(dev).cuda_stream)
            graph.replay()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(side)
            graph.replay()
            e1.record(side)
        e1.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / reps
        tot_t += count * us
        tot_b += count * by
        out.append({"launch": name, "per_step": count, "us": round(us, 2), "alg_bytes": int(by),
                    "GBs": round(by / (us * 1e-6) / 1e9, 1)})
    gbs = tot_b / (tot_t * 1e-6) / 1e9
    return {"ms_per_step": round(tot_t / 1e3, 3), "achieved_GBs": round(gbs, 1),
            "frac_of_hbm": round(gbs / PEAK_HBM_GBS, 4), "launches": out}


def traffic_from(path, kernel):
    """PMC HBM bytes per launch from profiles/pmc_traffic.json, only when it was measured
    on the kernel sources of this tree (its csrc_sha256 == the current source digest);
    otherwise None (the counters belong to another kernel revision)."""
    from onebit_asr._lib import source_digest

    try:
        data = json.loads(Path(path).read_text())
    except Exception:
        return None
    if data.get("csrc_sha256") != source_digest():
        return None
    return data.get(kernel, {}).get("hbm_bytes_per_launch")


# ------------------------------------------------------------------------- cpu baseline
def _cgroup_cpus():
    """The job's cgroup CPU quota in CPUs (cgroup v2 cpu.max / v1 cfs quota), or None."""
    try:
        q, per = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except Exception:
        pass
    try:
        q = int(Path("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read_text())
        per = int(Path("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read_text())
        return None if q <= 0 else round(q / per, 2)
    except Exception:
        return None


def cpu_baseline(seconds: float, bsz: int = 4, progress=lambda msg: None):
    """The oracle step (CPU restatement) on a bounded sample of the same workload on the
    host's cores: torch intra-op threads swept 8, 16, 32, ... up to the affinity count
    (the host's best, not a fixed count) and the fastest used; the sweep, the
    affinity / os.cpu_count() / cgroup-quota core counts are stated in the sample."""
    from onebit_asr.conformer import ConformerASR
    from onebit_asr.data import CONFORMER_S, synthetic_batch
    from onebit_asr.train_step import sample_sp_mask
    from oracle.conformer_oracle import OracleConformer, oracle_step_loss

    n_cpu = os.cpu_count() or 1
    try:
        n_aff = len(os.sched_getaffinity(0))
    except AttributeError:
        n_aff = n_cpu
    torch.manual_seed(1234)
    prod = ConformerASR(N_MELS, VOCAB, **CONFORMER_S)
    orc = OracleConformer(prod.state_dict(), input_dim=N_MELS, vocab_size=VOCAB, d_model=144,
                          n_layers=16, n_heads=4, d_ff=576, conv_kernel=31, dec_layers=2,
                          dec_heads=4, dec_d_ff=1024, dropout=0.1)
    orc.train()
    opt = torch.optim.AdamW(orc.parameters(), lr=5e-4, betas=(0.9, 0.98), weight_decay=1e-2)
    b = synthetic_batch([1000] * bsz, [40] * bsz, seed=99)
    g = torch.Generator().manual_seed(4321)

    def one():
        loss, _ = oracle_step_loss(orc, b, sample_sp_mask(16, generator=g))
        opt.zero_grad()
        loss.backward()
        torch.nn.utils.clip_grad_norm_(orc.parameters(), 5.0)
        opt.step()

    # The GPU box gives a one-GPU job a 16-CPU share (cgroup quota) although affinity and
    # os.cpu_count() show the whole machine: more intra-op threads than the share
    # oversubscribes it. Thread counts are swept upwards (8, 16, 32, 64, 128, ... up to the
    # affinity count) and the sweep stops at the first count slower than 1.25x the best so
    # far (every count past it only oversubscribes more); the fastest is used. The first
    # count also warms the model up (the thread pool's start at a new count is milliseconds).
    quota = _cgroup_cpus()
    cands = sorted({c for c in (8, 16, 32, 64, 128, 256) if c <= n_aff} | {min(8, n_aff)})
    trial = {}
    for th in cands:
        torch.set_num_threads(th)
        if not trial:
            one()  # warm-up
        t0 = time.perf_counter()
        one()
        trial[th] = time.perf_counter() - t0
        progress(f"cpu baseline: {th} threads, one step {trial[th]:.1f} s")
        if trial[th] > 1.25 * min(trial.values()):
            break
    threads = min(trial, key=trial.get)
    torch.set_num_threads(threads)
    times = []
    t_end = time.perf_counter() + seconds
    while time.perf_counter() < t_end and len(times) < 20:
        t0 = time.perf_counter()
        one()
        times.append(time.perf_counter() - t0)
        progress(f"cpu baseline: step {len(times)} {times[-1]:.1f} s")
    t = sorted(times)[len(times) // 2]
    cpu = platform.processor() or platform.machine()
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                cpu = line.split(":", 1)[1].strip()
                break
    except Exception:
        pass
    tried = ", ".join(f"{k} threads {bsz * 1000 / v:.0f}" for k, v in sorted(trial.items()))
    out = {"value": round(bsz * 1000 / t, 1), "unit": "mel-frames/s", "cores": threads,
           "kind": "port",
           "sample": f"oracle (CPU fp32 restatement) full 3-pass step + AdamW on Conformer-S, "
                     f"B={bsz} x 1000 frames, median of {len(times)} steps after warm-up; "
                     f"{threads} torch threads on {cpu} (affinity {n_aff} cores, "
                     f"os.cpu_count() {n_cpu}, cgroup CPU quota {quota}; thread sweep, "
                     f"one-step mel-frames/s: {tried})"}
    out["cfg1"] = cpu_cfg1(progress)
    out["ql_microbench"] = cpu_ql_microbench(progress)
    return out


def cpu_cfg1(progress=lambda msg: None, steps: int = 10):
    """SURVEY 8(d)'s parity config on the host: the oracle step (3 passes + losses + backward
    + clip + AdamW) of the 2-block d_model 64 Conformer at B = 2, feat_lens [734, 349], 10
    steps after one warm-up, at the thread count cpu_baseline chose."""
    from onebit_asr.conformer import ConformerASR
    from onebit_asr.data import CFG1, synthetic_batch
    from onebit_asr.train_step import sample_sp_mask
    from oracle.conformer_oracle import OracleConformer, oracle_step_loss

    torch.manual_seed(0)
    prod = ConformerASR(N_MELS, VOCAB, **CFG1)
    orc = OracleConformer(prod.state_dict(), input_dim=N_MELS, vocab_size=VOCAB, d_model=64,
                          n_layers=2, n_heads=4, d_ff=256, conv_kernel=31, dec_layers=2,
                          dec_heads=4, dec_d_ff=1024, dropout=0.0)
    opt = torch.optim.AdamW(orc.parameters(), lr=5e-4, betas=(0.9, 0.98), weight_decay=1e-2)
    b = synthetic_batch([734, 349], [27, 12], seed=0)
    g = torch.Generator().manual_seed(1)

    def one():
        loss, _ = oracle_step_loss(orc, b, sample_sp_mask(2, generator=g))
        opt.zero_grad()
        loss.backward()
        torch.nn.utils.clip_grad_norm_(orc.parameters(), 5.0)
        opt.step()

    one()
    t0 = time.perf_counter()
    for _ in range(steps):
        one()
    dt = (time.perf_counter() - t0) / steps
    progress(f"cpu baseline: cfg1 step {dt * 1e3:.0f} ms")
    return {"value": round((734 + 349) / dt, 1), "unit": "mel-frames/s",
            "ms_per_step": round(dt * 1e3, 2), "threads": torch.get_num_threads(),
            "sample": f"oracle step, 2 blocks d_model 64, B = 2 (734 + 349 frames), {steps} steps"}


def cpu_ql_microbench(progress=lambda msg: None, reps: int = 3):
    """QuantizedLinear alone on the host (the oracle's torch restatement of quant.py:38-127:
    quantize + F.linear forward, autograd backward for dX, dW, dalpha, db) at each
    Conformer-S shape with the 3 stacked passes' rows (M = 3 x 32 x 249), 2-bit; median of
    ``reps`` after one warm-up, at the thread count cpu_baseline chose."""
    from oracle.quant_oracle import ref_layer_init, ref_quantized_linear

    gen = torch.Generator().manual_seed(5)
    rows = 3 * 32 * 249
    res = []
    for name, k, n in (("lin1", 144, 576), ("lin2", 576, 144), ("qkvo", 144, 144)):
        w, a, bias = ref_layer_init(k, n, gen)
        w.requires_grad_()
        a.requires_grad_()
        bias.requires_grad_()
        x = torch.randn(rows, k, generator=gen, requires_grad=True)
        gy = torch.randn(rows, n, generator=gen)
        ts = []
        for i in range(reps + 1):
            t0 = time.perf_counter()
            y = ref_quantized_linear(x, w, a, bias, 2)
            y.backward(gy)
            if i:
                ts.append(time.perf_counter() - t0)
            x.grad = w.grad = a.grad = bias.grad = None
        t = sorted(ts)[len(ts) // 2]
        flop = 6.0 * rows * k * n
        res.append({"layer": name, "M": rows, "K": k, "N": n, "fwd_bwd_ms": round(t * 1e3, 2),
                    "GFLOPs": round(flop / t / 1e9, 1)})
        progress(f"cpu baseline: QL {name} fwd+bwd {t * 1e3:.0f} ms")
    return res


# ------------------------------------------------------------------------- inference
PEAK_I8_MFMA_TOPS = 5000.0  # 2x the dense bf16 rate (MI355X_MICROARCH.md, Matrix cores)


def roofline_i8(batch, frames, dev, act_quant, reps=20):
    """The inference step's BitLinear kernels at their B=256 shapes (one pass, 2-bit), as the
    step launches them. int8 path: ff.lin1 on the int8 LN image writing the int8 swish image
    at its own absmax (two launches: absmax, quantise + store), ff.lin2 reading that int8
    image with the 0.5-scaled residual, q/k/v on the int8 LN image, out_proj on the fp32
    attention context (absmax pass + in-register quantisation, residual), pos_proj; fp32
    path: the bf16x3 GEMM. Algorithmic bytes: each operand read once, each output written
    once (int8 = 1 byte, fp32 = 4). HIP events around a graph of `reps` launches on the
    launch stream."""
    from onebit_asr import _lib
    from onebit_asr.conformer import subsampled_length
    from onebit_asr.quant import pack_codes

    lib = _lib.load()
    t = subsampled_length(frames)
    m = batch * t
    # (name, M, K, N, launches per step, kind)
    if act_quant:
        shapes = [("lin1", m, 144, 576, 32, "swish_q8"), ("lin2", m, 576, 144, 32, "resid_q8"),
                  ("qkv", m, 144, 144, 48, "plain_q8"), ("out", m, 144, 144, 16, "resid_f32"),
                  ("pos", t, 144, 144, 16, "plain_f32")]
    else:
        shapes = [("lin1", m, 144, 576, 32, "plain"), ("lin2", m, 576, 144, 32, "plain"),
                  ("qkvo", m, 144, 144, 64, "plain"), ("pos", t, 144, 144, 16, "plain")]
    side = torch.cuda.Stream(dev)
    tot_t = tot_b = tot_f = 0.0
    n_launch = 0
    detail = []
    for name, M, K, N, count, kind in shapes:
        g = torch.Generator(device=dev).manual_seed(M + K + N)
        X = torch.randn(M, K, device=dev, generator=g)
        Xq = torch.randint(-127, 128, (M, K), device=dev, generator=g, dtype=torch.int32).to(torch.int8)
        R = torch.randn(M, N, device=dev, generator=g)
        W = (torch.rand(N, K, device=dev, generator=g) * 2 - 1) * (2 / math.sqrt(K))
        alpha = W.abs().mean()
        b = torch.zeros(N, device=dev)
        c2, _ = pack_codes(W, alpha, 2)
        Y = torch.empty(M, N, device=dev)
        amax = torch.full((1,), 4.0, device=dev)
        amax_out = torch.empty(1, device=dev)
        wsb = lib.ob_act_absmax_workspace(1)
        ws = torch.empty(wsb, dtype=torch.uint8, device=dev)

        def gemm(s):
            if kind == "plain":
                return lib.ob_bitlinear_fwd(X.data_ptr(), M, K, c2.data_ptr(), alpha.data_ptr(), 1,
                                            b.data_ptr(), N, Y.data_ptr(), s)
            if kind.endswith("q8"):
                mode = {"swish_q8": 3, "resid_q8": 2, "plain_q8": 0}[kind]
                return lib.ob_bitlinear_fwd_i8q(Xq.data_ptr(), 1, M, K, c2.data_ptr(), None, None,
                                                alpha.data_ptr(), 1, amax.data_ptr(), b.data_ptr(),
                                                N, mode, R.data_ptr(), 0.5, None, 0,
                                                amax_out.data_ptr(), Y.data_ptr(), s)
            st = lib.ob_act_absmax(X.data_ptr(), 1, M * K, amax.data_ptr(), ws.data_ptr(), wsb, s)
            if st:
                return st
            if kind == "resid_f32":
                return lib.ob_bitlinear_fwd_i8_epi(X.data_ptr(), 1, M, K, c2.data_ptr(), None, None,
                                                   alpha.data_ptr(), 1, amax.data_ptr(),
                                                   b.data_ptr(), N, 2, R.data_ptr(), 1.0, None, 0,
                                                   None, Y.data_ptr(), s)
            return lib.ob_bitlinear_fwd_i8(X.data_ptr(), 1, M, K, c2.data_ptr(), None, None,
                                           alpha.data_ptr(), 1, amax.data_ptr(), b.data_ptr(), N,
                                           Y.data_ptr(), s)

        def timed(fn):
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                for _ in range(3):
                    _lib.check(fn(side.cuda_stream), "roofline warm-up")
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph, stream=side):
                    for _ in range(reps):
                        fn(torch.cuda.current_stream(dev).cuda_stream)
                graph.replay()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(side)
                graph.replay()
                e1.record(side)
            e1.synchronize()
            return e0.elapsed_time(e1) * 1e3 / reps

        tg = timed(gemm)
        a_bytes = (1 if kind.endswith("q8") else 4) * M * K
        out_bytes = {"swish_q8": 1, "resid_q8": 8, "resid_f32": 8}.get(kind, 4) * M * N
        by = a_bytes + out_bytes + 4 * N + 4 * N * ((K + 15) // 16)
        fl = 2.0 * M * K * N
        tot_t += count * tg
        tot_b += count * by
        tot_f += count * fl
        n_launch += count
        detail.append({"layer": name, "kind": kind, "M": M, "K": K, "N": N,
                       "launches_per_step": count, "us": round(tg, 2),
                       "alg_bytes": int(by), "GBs": round(by / (tg * 1e-6) / 1e9, 1),
                       "TOPs": round(fl / (tg * 1e-6) / 1e12, 2)})
    avg = tot_t / n_launch
    gbs = (tot_b / n_launch) / (avg * 1e-6) / 1e9
    tops = (tot_f / n_launch) / (avg * 1e-6) / 1e12
    peak_c = PEAK_I8_MFMA_TOPS if act_quant else 2500.0
    return {"bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": round(gbs / PEAK_HBM_GBS, 4),
            "kernel": "tgemm_i8 (i8 MFMA, int8 operands in HBM)" if act_quant else "tgemm_bf16x3",
            "avg_launch_us": round(avg, 3), "bytes_per_launch": int(tot_b / n_launch),
            "flops_per_launch": int(tot_f / n_launch), "achieved_TOPs": round(tops, 2),
            "mfma_peak_TOPs": peak_c, "mfma_frac": round(tops / peak_c, 4),
            "ql_kernel_ms_per_step": round(tot_t / 1e3, 3), "shapes": detail, "traffic": None}


def roofline_i8_train(batch, frames, dev, reps=20, log=lambda m: None):
    """``--mode train-i8``: the training step's int8 forward GEMMs (ob_bitlinear_fwd_i8 on
    the stacked 3-pass rows, fp32 X quantised in registers at its per-pass absmax, i8 MFMA)
    at their Conformer-S shapes, and the per-call absmax launch that precedes each one (in
    training no LN / swish producer emits the scale). dX and dW stay on the fp32 kernels
    (STE; quant.py _BitLinearI8Fn). Algorithmic bytes of the GEMM: fp32 X read once, fp32 Y
    written once, the codes; FLOPs 2MKN. HIP events around `reps` graph-replayed launches."""
    from onebit_asr import _lib
    from onebit_asr.quant import pack_codes

    lib = _lib.load()
    side = torch.cuda.Stream(dev)
    pbits = torch.tensor(PASS_BITS, dtype=torch.int32, device=dev)
    tot = {"gemm_t": 0.0, "absmax_t": 0.0, "b": 0.0, "f": 0.0, "n": 0}
    detail = []
    for name, M, K, N, count in ql_shapes(batch, frames):  # qkvo: four module calls a block
        rows = PASSES * M
        g = torch.Generator(device=dev).manual_seed(M + K + N)
        X = torch.randn(rows, K, device=dev, generator=g)
        W = (torch.rand(N, K, device=dev, generator=g) * 2 - 1) * (2 / math.sqrt(K))
        alpha = W.abs().mean()
        b = torch.zeros(N, device=dev)
        c2, _ = pack_codes(W, alpha, 2)
        c1, _ = pack_codes(W, alpha, 1)
        Y = torch.empty(rows, N, device=dev)
        amax = torch.empty(PASSES, device=dev)
        wsb = lib.ob_act_absmax_workspace(PASSES)
        ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dev)
        _lib.check(lib.ob_act_absmax(X.data_ptr(), PASSES, M * K, amax.data_ptr(), ws.data_ptr(),
                                     wsb, torch.cuda.current_stream(dev).cuda_stream), "absmax")

        def absmax(s):
            return lib.ob_act_absmax(X.data_ptr(), PASSES, M * K, amax.data_ptr(), ws.data_ptr(),
                                     wsb, s)

        def gemm(s):
            return lib.ob_bitlinear_fwd_i8(X.data_ptr(), PASSES, M, K, c2.data_ptr(), c1.data_ptr(),
                                           pbits.data_ptr(), alpha.data_ptr(), 1, amax.data_ptr(),
                                           b.data_ptr(), N, Y.data_ptr(), s)

        def timed(fn):
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                for _ in range(3):
                    _lib.check(fn(side.cuda_stream), "roofline warm-up")
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph, stream=side):
                    for _ in range(reps):
                        fn(torch.cuda.current_stream(dev).cuda_stream)
                graph.replay()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(side)
                graph.replay()
                e1.record(side)
            e1.synchronize()
            return e0.elapsed_time(e1) * 1e3 / reps

        tg, ta = timed(gemm), timed(absmax)
        by = 4 * rows * K + 4 * rows * N + 4 * N + 2 * 4 * N * ((K + 15) // 16)
        fl = 2.0 * rows * K * N
        tot["gemm_t"] += count * tg
        tot["absmax_t"] += count * ta
        tot["b"] += count * by
        tot["f"] += count * fl
        tot["n"] += count
        detail.append({"layer": name, "rows": rows, "K": K, "N": N, "launches_per_step": count,
                       "gemm_us": round(tg, 2), "absmax_us": round(ta, 2), "alg_bytes": int(by),
                       "GBs": round(by / (tg * 1e-6) / 1e9, 1),
                       "TOPs": round(fl / (tg * 1e-6) / 1e12, 2)})
        log(f"roofline train-i8 {name}: gemm {tg:.2f} us, absmax {ta:.2f} us")
    n = tot["n"]
    avg = tot["gemm_t"] / n
    gbs = (tot["b"] / n) / (avg * 1e-6) / 1e9
    tops = (tot["f"] / n) / (avg * 1e-6) / 1e12
    return {"bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": round(gbs / PEAK_HBM_GBS, 4),
            "kernel": "tgemm_i8 (ob_bitlinear_fwd_i8: fp32 X quantised in registers, i8 MFMA)",
            "avg_launch_us": round(avg, 3), "bytes_per_launch": int(tot["b"] / n),
            "flops_per_launch": int(tot["f"] / n), "achieved_TOPs": round(tops, 2),
            "mfma_peak_TOPs": PEAK_I8_MFMA_TOPS, "mfma_frac": round(tops / PEAK_I8_MFMA_TOPS, 4),
            "i8_gemm_ms_per_step": round(tot["gemm_t"] / 1e3, 3),
            "absmax_ms_per_step": round(tot["absmax_t"] / 1e3, 3), "shapes": detail,
            "traffic": None}


def run_infer(args):
    from onebit_asr.conformer import ConformerASR
    from onebit_asr.data import CONFORMER_S, synthetic_batch
    from onebit_asr.infer import GraphedInference

    dev = torch.device("cuda", 0)
    act = "absmax_int8" if args.mode == "infer" else None
    torch.manual_seed(1234)
    model = ConformerASR(N_MELS, VOCAB, **CONFORMER_S).to(dev)
    batch = synthetic_batch([args.frames] * args.batch, [args.tokens] * args.batch, seed=1234,
                            device=dev)
    gi = GraphedInference(model, precision=2, act_quant=act, use_graph=not args.eager)
    log(args, "inference: capture")
    out = gi.run(batch)
    torch.cuda.synchronize()
    for _ in range(args.warmup):
        out = gi.run(batch)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = gi.run(batch)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    frames = args.batch * args.frames * args.steps
    res = {
        "metric": "mel-frames/sec (Conformer-S 1.58-bit inference + greedy CTC decode)",
        "value": round(frames / elapsed, 1), "unit": "mel-frames/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None,
        "dtype": "int8 x ternary (i8 MFMA), fp32 elsewhere" if act else "fp32",
        "data": "synthetic (N(0,1) 80-mel x 1000-frame padded batches, random-init weights)",
        "config": {"workload": "conformer-s-1.58bit-inference-greedy-ctc",
                   "execution": "eager" if args.eager else "hip-graph", "global_batch": args.batch,
                   "frames": args.frames, "precision": 2, "act_quant": act,
                   "d_model": 144, "blocks": 16, "vocab": VOCAB},
        "mean_tokens_per_utt": round(out[1].float().mean().item(), 2),
    }
    if not args.no_roofline:
        res["roofline"] = roofline_i8(args.batch, args.frames, dev, act)
    print(json.dumps(res), flush=True)


# ------------------------------------------------------------------------- main
def log(args, msg):
    if args.progress:
        print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def spawn_ranks(args) -> int:
    """``bench.py --gpus N`` started as ONE process (no WORLD_SIZE in the environment): start
    the N ranks as fresh child processes under torch.distributed.run -- before this process
    has touched the GPU (nothing above initialises HIP; no exec) -- and print rank 0's JSON
    line. Fails loudly when the line does not report N ranks."""
    import socket
    import subprocess

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1", f"--master-port={port}",
           str(Path(__file__).resolve())] + sys.argv[1:]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, text=True)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    for ln in r.stdout.splitlines():
        if not ln.startswith("{"):
            print(ln, file=sys.stderr)
    if r.returncode != 0:
        print(f"bench: {args.gpus}-rank run failed (exit {r.returncode})", file=sys.stderr)
        return r.returncode or 1
    if len(lines) != 1:
        print(f"bench: expected one JSON line from rank 0, got {len(lines)}", file=sys.stderr)
        return 1
    if json.loads(lines[0]).get("n_gpus") != args.gpus:
        print(f"bench: the line reports n_gpus != --gpus {args.gpus}", file=sys.stderr)
        return 1
    print(lines[0], flush=True)
    return 0


def replicas_equal(model, dev) -> bool:
    """After the timed steps: are the N replicas' parameters bitwise identical? (elementwise
    max == min over ranks of every parameter)."""
    flat = torch.cat([p.detach().reshape(-1) for p in model.parameters()]).to(dev)
    hi, lo = flat.clone(), flat.clone()
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    dist.all_reduce(lo, op=dist.ReduceOp.MIN)
    return bool(torch.equal(hi, lo))


def exchange_desc(args, gs):
    """The gradient exchange the timed steps ran (graph path: the bucket plan and whether the
    collectives were captured into the step graph)."""
    via = "RCCL" if args.dist_backend == "nccl" else "gloo"
    if gs is None:
        return f"DDP (eager) over {via}"
    where = "captured in the step graph" if gs.comm_in_graph else "between two graph replays"
    if gs.exchange == "deferred":
        return (f"deferred gradient finishes, then one fp32 all-reduce of the packed 47 MB "
                f"gradients per step over {via}, {where}")
    if gs.buckets is None:
        return f"one flat fp32 gradient all-reduce per step over {via}, {where}"
    return (f"{len(gs.buckets.buckets)} bucketed fp32 all-reduces per step (~{gs.bucket_bytes >> 20} MB, "
            f"reverse parameter order, started from the backward) over {via}, {where}")


def main():
    args = parse()
    if args.mode.startswith("infer"):
        return run_infer(args)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench: WORLD_SIZE {world} != --gpus {args.gpus}")
    distributed = world > 1
    n_dev = torch.cuda.device_count()
    if args.dist_backend == "nccl" and local >= n_dev:
        raise SystemExit(f"bench: rank {rank} needs GPU {local} but only {n_dev} are visible "
                         "(RCCL takes one GPU per rank; --dist-backend gloo shares one)")
    dev = torch.device("cuda", local % max(n_dev, 1))
    if distributed:
        torch.cuda.set_device(dev)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    from onebit_asr.conformer import ConformerASR
    from onebit_asr.data import CONFORMER_S, synthetic_batch
    from onebit_asr.train_step import OneBitStep, WarmupCosine, make_optimizer, sample_sp_mask, train_step

    torch.manual_seed(1234)  # identical init on every rank (DDP / the graph path broadcast)
    model = ConformerASR(N_MELS, VOCAB, **CONFORMER_S,
                         quantize_conv_pointwise=args.conv_pw_ternary).to(dev)
    quant_off = args.mode.startswith("quant-off")
    train_i8 = args.mode == "train-i8"
    if train_i8:  # every BitLinear on absmax-int8 activations (quant.py _BitLinearI8Fn)
        from onebit_asr.quant import set_act_quant

        set_act_quant(model, "absmax_int8")
    if quant_off:  # configs[3]: every BitLinear -> bf16 weights, same step body
        from onebit_asr.quant import set_quant_off

        # quant-off: the ternary path's fused kernels with B = bf16(W) (only the weight format
        # differs); quant-off-lib: bf16 F.linear on hipBLASLt
        set_quant_off(model, "bf16w" if args.mode == "quant-off" else torch.bfloat16)
    n_layers = CONFORMER_S["enc_layers"]
    step_mod = OneBitStep(model, n_layers=n_layers, branch_streams=args.branch_streams)
    batch = synthetic_batch([args.frames] * args.batch, [args.tokens] * args.batch,
                            seed=1234 + rank, device=dev)
    sp_gen = torch.Generator().manual_seed(4321)  # same SP masks on every rank
    if distributed:
        with torch.no_grad():  # replicas start identical (DDP does the same); in place on
            for p in model.parameters():  # the parameter itself, so its version is bumped
                dist.broadcast(p, 0)

    if args.eager:
        if distributed:
            from torch.nn.parallel import DistributedDataParallel as DDP

            step_mod = DDP(step_mod, device_ids=[dev.index], broadcast_buffers=False,
                           gradient_as_bucket_view=True)
        opt = make_optimizer(model.parameters())
        sched = WarmupCosine(opt, warmup_steps=4000, total_steps=100000)

        def step():
            return train_step(step_mod, opt, sched, batch, sample_sp_mask(n_layers, generator=sp_gen))
    else:
        from onebit_asr.graph_step import GraphedTrainStep

        gs = GraphedTrainStep(step_mod, n_layers, warmup_steps=4000, total_steps=100000,
                              process_group=dist.group.WORLD if distributed else None,
                              warmup_iters=2)

        def step():
            return gs.step(batch, sample_sp_mask(n_layers, generator=sp_gen))

    if args.roofline_only:
        roof = roofline(args.batch, args.frames, dev, log=lambda m: log(args, m))
        roof["in_step_fused"] = roofline_fused(args.batch, args.frames, dev,
                                               log=lambda m: log(args, m))
        print(json.dumps({"roofline": roof}), flush=True)
        return
    log(args, "model built; first step (graph mode: warm-up steps + capture)")
    for i in range(max(args.warmup, 1)):  # graph mode: the first call captures
        loss, _ = step()
        torch.cuda.synchronize()
        log(args, f"warm-up step {i} done, loss {loss.item():.4f}")
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss, _ = step()
    torch.cuda.synchronize()
    log(args, "timed steps done")
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if distributed:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    loss_val = float(loss.item())
    same = replicas_equal(model, dev) if distributed else None

    frames_total = world * args.batch * args.frames * args.steps
    value = frames_total / elapsed
    out = {
        "metric": ("mel-frames/sec (Conformer-S quant-off train step, BitLinear -> bf16 nn.Linear)"
                   if quant_off else
                   "mel-frames/sec (Conformer-S 1.58-bit train step, absmax-int8 activations: "
                   "opt-in, not the reference's arithmetic)" if train_i8 else
                   "mel-frames/sec (Conformer-S 1.58-bit train step)"),
        "quant_off": (None if not quant_off else
                      "bf16 weights on the fused ternary-GEMM kernels (exact fp32 activations)"
                      if args.mode == "quant-off" else "bf16 F.linear on hipBLASLt"),
        "value": round(value, 1),
        "unit": "mel-frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": ("bf16 weights x fp32 activations (fused kernels), fp32 elsewhere"
                  if args.mode == "quant-off" else
                  "bf16 linears (hipBLASLt), fp32 elsewhere" if quant_off else
                  "int8 x ternary forward GEMMs (i8 MFMA); fp32 dX / dW and elsewhere"
                  if train_i8 else "fp32"),
        "data": "synthetic (N(0,1) 80-mel x 1000-frame padded batches, random-init weights)",
        "config": {"workload": ("conformer-s-quant-off-bf16-train-step" if quant_off
                                else "conformer-s-1.58bit-train-step-int8-act" if train_i8
                                else "conformer-s-1.58bit-train-step"), "global_batch": args.batch * world,
                   "execution": "eager" if args.eager else "hip-graph",
                   "per_gpu_batch": args.batch, "frames": args.frames, "tokens": args.tokens,
                   "d_model": 144, "blocks": 16, "d_ff": 576, "heads": 4, "vocab": VOCAB,
                   "parallelism": f"dp{world}",
                   "exchange": exchange_desc(args, gs if not args.eager else None)
                               if distributed else None,
                   "passes": "teacher 2-bit + student 1-bit + SP",
                   "subsampling": "computed once, shared by the 3 stacked passes (exact: no "
                                  "dropout, full-precision weights; the reference runs it 3x)",
                   "conv_pointwise": "ternary (opt-in)" if args.conv_pw_ternary else "fp32 (reference)"},
        "final_loss": round(loss_val, 4),
    }
    if distributed:
        out["replicas_bitwise_equal"] = same
    if quant_off:  # no ternary kernel runs: the line is the ceiling the 1.58-bit step is read against
        out["roofline"] = None
    elif train_i8:  # the int8 forward GEMMs; the fp32 oracle step is no baseline for this mode
        out["roofline"] = (None if args.no_roofline or rank != 0 or world != 1 else
                           roofline_i8_train(args.batch, args.frames, dev,
                                             log=lambda m: log(args, m)))
    elif rank == 0 and world == 1 and not args.no_roofline:
        from onebit_asr import deferred

        roof = roofline(args.batch, args.frames, dev, log=lambda m: log(args, m),
                        dwg_shapes=list(deferred.LAST_DWG) or None)
        roof["traffic"] = traffic_from(args.traffic_json, roof["kernel"])
        # the same family as the step launches it (fused epilogues, dX accumulations)
        roof["in_step_fused"] = roofline_fused(args.batch, args.frames, dev,
                                               log=lambda m: log(args, m))
        out["roofline"] = roof
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not quant_off and not train_i8:
        # (progress always on stderr: the CPU leg runs minutes without other output)
        out["cpu_baseline"] = cpu_baseline(
            args.cpu_seconds,
            progress=lambda m: print(f"[bench {time.strftime('%H:%M:%S')}] {m}", file=sys.stderr,
                                     flush=True))
    if rank == 0:
        print(json.dumps(out), flush=True)
    if distributed:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
