#!/usr/bin/env python3
"""Times the conv module's pw GEMMs (F.linear fwd + bwd) under hipBLASLt and rocBLAS."""
import torch
import torch.nn.functional as F

dev = torch.device("cuda:0")
shapes = [(23904, 144, 288), (23904, 144, 144), (23904, 144, 5004), (3 * 32 * 41, 144, 1024)]


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


for lib in ["cublaslt", "cublas"]:
    torch.backends.cuda.preferred_blas_library(lib)
    for m, k, n in shapes:
        x = torch.randn(m, k, device=dev, requires_grad=True)
        w = torch.randn(n, k, device=dev, requires_grad=True)
        b = torch.randn(n, device=dev, requires_grad=True)
        g = torch.randn(m, n, device=dev)
        fwd = t(lambda: F.linear(x, w, b))
        y = F.linear(x, w, b)
        bwd = t(lambda: torch.autograd.grad(y, (x, w, b), g, retain_graph=True))
        print(f"{lib:9s} M={m:6d} K={k:4d} N={n:5d}  fwd {fwd:8.1f} us  bwd {bwd:8.1f} us", flush=True)
