#!/usr/bin/env python3
"""The N > 1 step's per-rank cost on one GPU: bench.py's Conformer-S step through the
multi-rank path at world size 1 over RCCL (graph_step._MULTI_RANK_PATH_AT_WORLD_1) with
each exchange (deferred: pack / one all-reduce / unpack after deferred finishes; bucketed:
gradient views, finishes on the spot, bucket all-reduces from the hooks), both captured
into the step graph, against the single-GPU path, same process.
Round 6: the deferred exchange also with its grouped dW split into 3 launches whose buckets are
all-reduced under the next launch (overlap_chunks 3, the default) against one launch
(overlap_chunks 1). usage: python tools/multi_path_bench.py [steps] [only]
(only = "chunked": just the overlapped configuration, e.g. under rocprofv3)"""
import os
import socket
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "cmu-11785-idl-1.58bit-asr_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    only = sys.argv[2] if len(sys.argv) > 2 else ""
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=dev)
    from onebit_asr import graph_step
    from onebit_asr.conformer import ConformerASR
    from onebit_asr.data import CONFORMER_S, synthetic_batch
    from onebit_asr.train_step import OneBitStep, sample_sp_mask

    n_layers = CONFORMER_S["enc_layers"]
    batch = synthetic_batch([1000] * 32, [40] * 32, seed=1234, device=dev)
    cfgs = ((False, "deferred", 1), (True, "deferred", 1), (True, "deferred", 3),
            (True, "bucketed", 1))
    if only == "chunked":
        cfgs = ((True, "deferred", 3),)
    for multi, exchange, chunks in cfgs:
        graph_step._MULTI_RANK_PATH_AT_WORLD_1 = multi
        torch.manual_seed(1234)
        model = ConformerASR(80, 5004, **CONFORMER_S).to(dev)
        gs = graph_step.GraphedTrainStep(OneBitStep(model, n_layers=n_layers), n_layers,
                                         warmup_steps=4000, total_steps=100000,
                                         process_group=dist.group.WORLD, warmup_iters=2,
                                         exchange=exchange, overlap_chunks=chunks)
        gen = torch.Generator().manual_seed(4321)
        for _ in range(3):
            gs.step(batch, sample_sp_mask(n_layers, generator=gen))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            gs.step(batch, sample_sp_mask(n_layers, generator=gen))
        torch.cuda.synchronize()
        ms = 1e3 * (time.perf_counter() - t0) / steps
        nb = len(gs.buckets.buckets) if gs.buckets is not None else 0
        cp = [p for p, v in zip(gs.params, gs.flat_views)
              if p.grad is not None and p.grad.data_ptr() != v.data_ptr()] if multi else []
        ov = f" in {chunks} overlapped chunks" if (multi and gs.xchg is not None) else ""
        print(f"{('multi-rank path, ' + exchange + ov) if multi else 'single-GPU path'}: {ms:.3f} ms/step "
              f"(buckets {nb}, all-reduce in the graph: {gs.comm_in_graph}; gradients copied "
              f"around the exchange: {len(cp)} of {len(gs.params)}, "
              f"{sum(p.numel() for p in cp) * 4 / 2**20:.1f} MiB)", flush=True)
        if gs.xchg is not None:
            from onebit_asr import deferred
            print(f"  overlapped exchange ran: {gs.xchg.started}; plan note: {deferred.PLAN_NOTE!r}",
                  flush=True)
        del gs, model
        torch.cuda.empty_cache()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
