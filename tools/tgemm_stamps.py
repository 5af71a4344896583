#!/usr/bin/env python3
"""Where a ternary-GEMM wave spends its cycles, from a diagnostic build (-DOB_TGEMM_STAMPS:
per wave the prologue / main-loop / epilogue cycles, the row tiles done and s_memrealtime at
start and end, into buffers of their own). Shapes: the Conformer-S stacked-pass launches.
Build:  make -C cmu-11785-idl-1.58bit-asr_amd/csrc OUT=$PWD/exp/libtgstamp.so BUILD=$PWD/exp/tgstamp \
        HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -DOB_TGEMM_STAMPS"
Run:    ONEBIT_HIP_LIB=exp/libtgstamp.so python tools/tgemm_stamps.py"""
import ctypes
import math
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "cmu-11785-idl-1.58bit-asr_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from onebit_asr import _lib  # noqa: E402
from onebit_asr.quant import pack_codes  # noqa: E402


def report(lib, name, run):
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    st = np.zeros(32768, dtype=np.uint64)
    rt = np.zeros(16384, dtype=np.uint64)
    fn = lib.ob_tgemm_stamps
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    assert fn(st.ctypes.data, rt.ctypes.data) == 0
    st = st.reshape(-1, 4).astype(np.float64)
    rt = rt.reshape(-1, 2).astype(np.float64)
    live = (rt[:, 1] > 0) & (st[:, 3] > 0)
    st, rt = st[live], rt[live]
    dur = (rt[:, 1] - rt[:, 0]) / 100.0  # us
    span = (rt[:, 1].max() - rt[:, 0].min()) / 100.0
    cyc = st[:, :3].sum(axis=1)
    clk = np.median(cyc / np.maximum(dur, 1e-9)) / 1e3
    tiles = st[:, 3]
    print(f"{name}: {len(st)} waves, span {span:.1f} us, wave duration median {np.median(dur):.1f} us, "
          f"waves in flight on average {dur.sum() / span:.0f} ({dur.sum() / span / 1024:.2f} per SIMD), "
          f"clock ~{clk:.2f} GHz")
    print(f"   per wave (median cycles): prologue {np.median(st[:, 0]):.0f}, main loops "
          f"{np.median(st[:, 1]):.0f}, epilogues {np.median(st[:, 2]):.0f}, row tiles "
          f"{np.median(tiles):.0f}; per row tile: loop {np.median(st[:, 1] / tiles):.0f}, "
          f"epilogue {np.median(st[:, 2] / tiles):.0f}")


def main():
    lib = _lib.load()
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    P, M = 3, 7968
    for name, K, N in (("lin1 (K 144, N 576)", 144, 576), ("lin2 (K 576, N 144)", 576, 144)):
        X = torch.randn(P * M, K, device=dev)
        dY = torch.randn(P * M, N, device=dev)
        W = (torch.rand(N, K, device=dev) * 2 - 1) * (2 / math.sqrt(K))
        alpha = W.abs().mean()
        b = torch.zeros(N, device=dev)
        codes, codes_t = pack_codes(W, alpha, 2)
        c1, c1t = pack_codes(W, alpha, 1)
        pbits = torch.tensor([2, 1, 1], dtype=torch.int32, device=dev)
        Y = torch.empty(P * M, N, device=dev)
        dX = torch.empty(P * M, K, device=dev)
        report(lib, name + " fwd", lambda: lib.ob_bitlinear_fwd_passes(
            X.data_ptr(), P, M, K, codes.data_ptr(), c1.data_ptr(), pbits.data_ptr(),
            alpha.data_ptr(), 1, b.data_ptr(), N, Y.data_ptr(), s))
        report(lib, name + " dX", lambda: lib.ob_bitlinear_bwd_dx_passes(
            dY.data_ptr(), P, M, N, codes_t.data_ptr(), c1t.data_ptr(), pbits.data_ptr(),
            alpha.data_ptr(), 1, K, dX.data_ptr(), s))
        if N == 576:  # the FFN's fused launches: lin1 fwd + swish + dropout, lin2 dX + swish bwd
            rng = torch.tensor([1234, 5], dtype=torch.int64, device=dev)
            Y2 = torch.empty_like(Y)
            report(lib, name + " fwd + swish + dropout", lambda: lib.ob_bitlinear_fwd_swish_drop(
                X.data_ptr(), P, M, K, codes.data_ptr(), c1.data_ptr(), pbits.data_ptr(),
                alpha.data_ptr(), 1, b.data_ptr(), N, 0.1, rng.data_ptr(), 0, Y2.data_ptr(),
                Y.data_ptr(), s))
            dY2 = torch.randn(P * M, K, device=dev)
            pre = torch.randn(P * M, N, device=dev)
            dX2 = torch.empty(P * M, N, device=dev)
            report(lib, "lin2 dX + dropout / swish bwd (K 144, N 576)",
                   lambda: lib.ob_bitlinear_bwd_dx_swish_drop(
                       dY2.data_ptr(), P, M, K, codes.data_ptr(), c1.data_ptr(), pbits.data_ptr(),
                       alpha.data_ptr(), 1, N, pre.data_ptr(), 0.1, rng.data_ptr(), 0,
                       dX2.data_ptr(), s))


if __name__ == "__main__":
    main()
