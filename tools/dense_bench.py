"""Time the pointwise-conv GEMMs (csrc/dgemm.hip, ob_dense_*) against the rocBLAS fp32 calls
they replace, at the Conformer-S train-step shapes (3 stacked passes x 32 x 249 rows).

  python tools/dense_bench.py [--iters 50]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cmu-11785-idl-1.58bit-asr_amd"))
from onebit_asr import _lib  # noqa: E402


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--m", type=int, default=23904)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    lib = _lib.load()
    st = _lib.stream_of(torch.empty(1, device=dev))
    m = a.m
    torch.backends.cuda.preferred_blas_library("cublas")
    shapes = [(m, 144, 288, 0), (m, 144, 144, 0), (m, 288, 144, 1), (m, 144, 144, 1),
              (m, 144, 5004, 0), (3936, 144, 144, 0), (3936, 144, 432, 0), (3936, 144, 144, 1),
              (3936, 144, 1024, 0), (3936, 1024, 144, 0), (m, 5004, 144, 1), (3936, 5004, 144, 1),
              # subsampling's output linear (K = 144 x 19): training B = 32, inference B = 256
              (7968, 2736, 144, 0), (63744, 2736, 144, 0)]
    for m, k, n, trans in shapes:
        if n % 4:
            continue
        x = torch.randn(m, k, device=dev)
        w = torch.randn((k, n) if trans else (n, k), device=dev)
        b = None if trans else torch.randn(n, device=dev)
        y = torch.empty(m, n, device=dev)
        hip = timeit(lambda: lib.ob_dense_gemm(x.data_ptr(), m, k, w.data_ptr(), trans,
                                               _lib.ptr(b), n, y.data_ptr(), st), a.iters)
        if trans:
            blas = timeit(lambda: x @ w, a.iters)
        else:
            blas = timeit(lambda: torch.addmm(b, x, w.t()), a.iters)
        byt = 4 * m * (k + n)
        fl = 2 * m * n * k
        print(f"gemm M={m} K={k} N={n} trans={trans}: hip {hip:7.1f} us ({byt / hip / 1e3:6.0f} GB/s, "
              f"{6 * fl / hip / 1e6:6.0f} bf16-TFLOP/s)  rocBLAS {blas:7.1f} us", flush=True)
    m = a.m
    for n, k in [(288, 144), (144, 144)]:
        dy = torch.randn(m, n, device=dev)
        x = torch.randn(m, k, device=dev)
        dw = torch.empty(n, k, device=dev)
        db = torch.empty(n, device=dev)
        wsb = lib.ob_dense_dw_workspace(m, n, k)
        ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
        hip = timeit(lambda: lib.ob_dense_dw(dy.data_ptr(), x.data_ptr(), m, n, k, dw.data_ptr(),
                                             db.data_ptr(), ws.data_ptr(), wsb, st), a.iters)
        blas = timeit(lambda: (dy.t() @ x, dy.sum(0)), a.iters)
        byt = 4 * m * (k + n)
        print(f"dW N={n} K={k}: hip {hip:7.1f} us ({byt / hip / 1e3:6.0f} GB/s)  "
              f"rocBLAS+sum {blas:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
