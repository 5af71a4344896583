#!/usr/bin/env python3
"""Does torch's reduction kernel stay correct across HIP-graph replays when other
allocations inside the graph reuse its temporaries? A captured body computes sums /
means of large tensors, then fills freshly allocated small buffers with junk; replays
1..3 are compared with eager."""
import sys

import torch


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(3936, 1024, device=dev, generator=g)
    y = torch.randn(96, 249, 5004, device=dev, generator=g)

    def body(junk: bool):
        outs = [x.sum(0), y.sum((0, 1)), y.mean(), x.square().mean(), x.sum(1)]
        if junk:
            for n in (64, 256, 1024, 4096, 16384):
                torch.full((n,), 12345.0, device=dev).add_(1.0)
        return outs

    ref = [t.clone() for t in body(False)]
    for junk in (False, True):
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            body(junk)
        torch.cuda.current_stream(dev).wait_stream(s)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            outs = body(junk)
        for r in range(3):
            graph.replay()
            torch.cuda.synchronize()
            errs = [((o - e).abs().max() / e.abs().max()).item() for o, e in zip(outs, ref)]
            print(f"junk={junk} replay#{r + 1}: " + " ".join(f"{v:.1e}" for v in errs), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
