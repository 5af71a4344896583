#!/usr/bin/env python3
"""north_star's inner-product A/B at the Conformer-S BitLinear shapes (3 stacked passes of
B = 32 x 249 rows = 23904): the bf16x3 MFMA ternary GEMM (ob_bitlinear_fwd) against the VALU
sign-accumulate form (ob_bitlinear_fwd_signacc, csrc/tgemm_va.hip), HIP events on graph-replayed
launches; algorithmic bytes 4*M*(K+N) + the 2-bit codes. Run under tools/pmc_cmd.sh for the
VALU / MFMA-busy counters. usage: python tools/signacc_ab.py [--reps 50]"""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "cmu-11785-idl-1.58bit-asr_amd"), str(ROOT / "tools")]

import torch  # noqa: E402

from kbench import timed  # noqa: E402
from onebit_asr import _lib  # noqa: E402
from onebit_asr.quant import pack_codes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    lib = _lib.load()
    M = 3 * 32 * 249
    g = torch.Generator(device=dev).manual_seed(0)
    for name, K, N in (("lin1", 144, 576), ("qkvo", 144, 144), ("lin2", 576, 144)):
        W = (torch.rand(N, K, device=dev, generator=g) * 2 - 1) * (2 / K ** 0.5)
        alpha = W.abs().mean().reshape(())
        codes, _ = pack_codes(W, alpha, 2)
        X = torch.randn(M, K, device=dev, generator=g)
        b = torch.randn(N, device=dev, generator=g) * 0.1
        Y0 = torch.empty(M, N, device=dev)
        Y1 = torch.empty(M, N, device=dev)

        def mfma(s=None):
            _lib.check(lib.ob_bitlinear_fwd(X.data_ptr(), M, K, codes.data_ptr(), alpha.data_ptr(),
                                            1, b.data_ptr(), N, Y0.data_ptr(),
                                            s if s is not None else _lib.stream_of(X)), "fwd")

        def sacc(s=None):
            _lib.check(lib.ob_bitlinear_fwd_signacc(X.data_ptr(), M, K, codes.data_ptr(),
                                                    alpha.data_ptr(), 1, b.data_ptr(), N,
                                                    Y1.data_ptr(),
                                                    s if s is not None else _lib.stream_of(X)),
                       "signacc")

        t0 = timed(mfma, a.reps, True)
        t1 = timed(sacc, a.reps, True)
        torch.cuda.synchronize()
        err = (Y0 - Y1).abs().max().item() / Y0.abs().max().item()
        byt = 4 * M * (K + N) + codes.numel() * 4
        fl = 2 * M * K * N
        print(f"{name} M={M} K={K} N={N}: bf16x3-MFMA {t0:7.1f} us ({byt / t0 / 1e3:6.0f} GB/s, "
              f"{fl / t0 / 1e6:5.1f} TFLOP/s)  VALU sign-accumulate {t1:7.1f} us "
              f"({byt / t1 / 1e3:6.0f} GB/s, {fl / t1 / 1e6:5.1f} TFLOP/s)  max|dY|/max|Y| {err:.1e}",
              flush=True)


if __name__ == "__main__":
    main()
