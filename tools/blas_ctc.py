#!/usr/bin/env python3
"""Library-GEMM variants for the backward of the V = 5004 linears (CTC head at [23904, 144],
decoder output layer at [3936, 144]): dX = g W and dW = g^T x under hipBLASLt and rocBLAS,
and dW computed transposed ((x^T g)^T). usage: python tools/blas_ctc.py"""
import torch

dev = torch.device("cuda:0")


def t(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


for m in (23904, 3936):
    k, n = 144, 5004
    x = torch.randn(m, k, device=dev)
    w = torch.randn(n, k, device=dev)
    g = torch.randn(m, n, device=dev)
    wt = w.t().contiguous()
    for lib in ("cublaslt", "cublas"):
        torch.backends.cuda.preferred_blas_library(lib)
        r = {
            "dX g@w": t(lambda: g @ w),
            "dX (w^T g^T)^T": t(lambda: (wt @ g.t()).t()),
            "dW g^T@x": t(lambda: g.t() @ x),
            "dW (x^T g)^T": t(lambda: (x.t() @ g).t()),
        }
        print(m, lib, {a: round(b, 1) for a, b in r.items()}, flush=True)
