#!/usr/bin/env python3
"""Minimal check of stock fp32 torch Linear layers under HIP-graph replay: eager grads vs
three replays of a captured forward+backward. Variants: --blas {default,cublas,cublaslt},
--act {none,relu}. Prints the worst relative error of every parameter per replay."""
import argparse
import sys

import torch
import torch.nn.functional as F


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blas", default="default")
    ap.add_argument("--act", default="relu")
    ap.add_argument("--rows", type=int, default=96 * 41)
    ap.add_argument("--k", type=int, default=144)
    ap.add_argument("--n", type=int, default=1024)
    a = ap.parse_args()
    if a.blas != "default":
        torch.backends.cuda.preferred_blas_library(a.blas)
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    lin1 = torch.nn.Linear(a.k, a.n).to(dev)
    lin2 = torch.nn.Linear(a.n, a.k).to(dev)
    x = torch.randn(a.rows // 41, 41, a.k, device=dev, requires_grad=True)
    g = torch.randn(a.rows // 41, 41, a.k, device=dev)
    params = {"lin1.w": lin1.weight, "lin1.b": lin1.bias, "lin2.w": lin2.weight,
              "lin2.b": lin2.bias, "x": x}

    def fwd_bwd():
        for p in params.values():
            p.grad = None
        h = lin1(x)
        if a.act == "relu":
            h = F.relu(h)
        y = lin2(h)
        y.backward(g)

    def snap():
        return {k: p.grad.detach().clone() for k, p in params.items()}

    fwd_bwd()
    ref = snap()
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        fwd_bwd()
        fwd_bwd()
    torch.cuda.current_stream(dev).wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        fwd_bwd()
    worst = 0.0
    for r in range(3):
        graph.replay()
        torch.cuda.synchronize()
        cur = snap()
        errs = {k: ((cur[k] - ref[k]).norm() / ref[k].norm().clamp_min(1e-30)).item() for k in ref}
        worst = max(worst, max(errs.values()))
        print(f"blas={a.blas} act={a.act} replay#{r + 1}: " +
              " ".join(f"{k}={v:.1e}" for k, v in errs.items()), flush=True)
    print(f"RESULT blas={a.blas} act={a.act} worst={worst:.2e} {'OK' if worst < 1e-5 else 'CORRUPT'}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
