#!/usr/bin/env python3
"""Where a dW-GEMM wave (dw_lds_kernel) spends its cycles, from a diagnostic build
(-DOB_DW_STAMPS): prologue, MFMA phases, split / LDS-store phases, load issue, barrier
waits, partial + alpha epilogue, db epilogue; block concurrency from s_memrealtime.
Build:  make -C cmu-11785-idl-1.58bit-asr_amd/csrc OUT=$PWD/exp/libdwstamp.so BUILD=$PWD/exp/dwstamp \\
        HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -DOB_DW_STAMPS"
Run:    ONEBIT_HIP_LIB=exp/libdwstamp.so python tools/dw_stamps.py"""
import ctypes
import math
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "cmu-11785-idl-1.58bit-asr_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from onebit_asr import _lib  # noqa: E402

PH = ["prologue", "mfma", "split+store", "load issue", "barrier", "partials+alpha", "db", "-"]


def main():
    lib = _lib.load()
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    P, M = 3, 7968
    for name, K, N in (("lin1 (N 576, K 144)", 144, 576), ("lin2 (N 144, K 576)", 576, 144)):
        X = torch.randn(P * M, K, device=dev)
        dY = torch.randn(P * M, N, device=dev)
        W = (torch.rand(N, K, device=dev) * 2 - 1) * (2 / math.sqrt(K))
        alpha = W.abs().mean()
        pbits = torch.tensor([2, 1, 1], dtype=torch.int32, device=dev)
        dW = torch.empty(N, K, device=dev)
        da = torch.empty((), device=dev)
        db = torch.empty(N, device=dev)
        wsb = lib.ob_bitlinear_bwd_dw_passes_workspace(P, M, N, K)
        ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
        for _ in range(3):
            _lib.check(lib.ob_bitlinear_bwd_dw_passes(
                dY.data_ptr(), X.data_ptr(), P, M, N, K, W.data_ptr(), alpha.data_ptr(), 1,
                pbits.data_ptr(), dW.data_ptr(), da.data_ptr(), db.data_ptr(), ws.data_ptr(), wsb,
                s), "dw")
        torch.cuda.synchronize()
        st = np.zeros(8 * 4096, dtype=np.uint64)
        rt = np.zeros(2 * 4096, dtype=np.uint64)
        fn = lib.ob_dw_stamps
        fn.restype = ctypes.c_int
        fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        assert fn(st.ctypes.data, rt.ctypes.data) == 0
        st = st.reshape(-1, 8).astype(np.float64)
        rt = rt.reshape(-1, 2).astype(np.float64)
        live = rt[:, 1] > 0
        st, rt = st[live], rt[live]
        dur = (rt[:, 1] - rt[:, 0]) / 100.0
        span = (rt[:, 1].max() - rt[:, 0].min()) / 100.0
        clk = np.median(st.sum(axis=1) / np.maximum(dur, 1e-9)) / 1e3
        print(f"{name} dW partial: {len(st)} waves, span {span:.1f} us, wave duration median "
              f"{np.median(dur):.1f} us, waves in flight on average {dur.sum() / span:.0f}, "
              f"clock ~{clk:.2f} GHz")
        med = np.median(st, axis=0)
        print("   per wave (median cycles): " + "  ".join(f"{n} {m:.0f}" for n, m in zip(PH, med)))


if __name__ == "__main__":
    main()
