#!/usr/bin/env python3
"""Does a hipMemsetAsync captured into a HIP graph re-run on every replay? Capture
[memset(buf, 0); buf += 1] and check buf == 1 after each replay, for several sizes;
the same with torch's zero_() in place of the raw memset."""
import ctypes
import sys

import torch


def main():
    dev = torch.device("cuda", 0)
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipMemsetAsync.restype = ctypes.c_int
    hip.hipMemsetAsync.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
    for how in ("hipMemsetAsync", "zero_", "fill_0"):
        for n in (1, 4, 64, 1000, 1 << 20):
            buf = torch.full((n,), 5.0, device=dev)
            torch.cuda.synchronize()
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                if how == "hipMemsetAsync":
                    st = hip.hipMemsetAsync(buf.data_ptr(), 0, 4 * n,
                                            torch.cuda.current_stream(dev).cuda_stream)
                    assert st == 0, st
                elif how == "zero_":
                    buf.zero_()
                else:
                    buf.fill_(0.0)
                buf.add_(1.0)
            vals = []
            for _ in range(3):
                graph.replay()
                torch.cuda.synchronize()
                vals.append((buf.min().item(), buf.max().item()))
            ok = all(v == (1.0, 1.0) for v in vals)
            print(f"{how:15s} n={n:8d}: {vals} {'OK' if ok else 'BROKEN'}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
