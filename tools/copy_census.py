"""Where the step's torch copies and fills come from: one eager run of the GraphedTrainStep
body (use_graph=False, same code path as the captured step) under torch.profiler with
Python stacks; every copy / fill / zero / cat / clone op is attributed to its innermost
frame inside this repository and the counts per call site are printed.

usage (GPU box, repo root): python tools/copy_census.py [--batch 32] [--frames 1000]
"""
import argparse
import collections
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "cmu-11785-idl-1.58bit-asr_amd"))
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

OPS = ("aten::copy_", "aten::fill_", "aten::zero_", "aten::cat", "aten::clone",
       "aten::contiguous", "aten::zeros", "aten::zeros_like", "aten::index_put_",
       "aten::_foreach_copy_", "aten::_foreach_zero_", "aten::repeat", "aten::to",
       "aten::_to_copy", "aten::masked_fill_", "aten::where", "aten::mul", "aten::add",
       "aten::add_", "aten::sub", "aten::div", "aten::sum", "aten::mean")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--frames", type=int, default=1000)
    ap.add_argument("--tokens", type=int, default=40)
    a = ap.parse_args()
    from onebit_asr.conformer import ConformerASR
    from onebit_asr.data import CONFORMER_S, synthetic_batch
    from onebit_asr.graph_step import GraphedTrainStep
    from onebit_asr.train_step import OneBitStep, sample_sp_mask

    dev = torch.device("cuda", 0)
    torch.manual_seed(1234)
    model = ConformerASR(80, 5004, **CONFORMER_S).to(dev)
    n_layers = CONFORMER_S["enc_layers"]
    step_mod = OneBitStep(model, n_layers=n_layers)
    batch = synthetic_batch([a.frames] * a.batch, [a.tokens] * a.batch, seed=1234, device=dev)
    gen = torch.Generator().manual_seed(4321)
    gs = GraphedTrainStep(step_mod, n_layers, use_graph=False)
    for _ in range(2):
        gs.step(batch, sample_sp_mask(n_layers, generator=gen))
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True,
                 record_shapes=True, acc_events=True) as prof:
        gs.step(batch, sample_sp_mask(n_layers, generator=gen))
        torch.cuda.synchronize()
    sites = collections.Counter()
    per_op = collections.Counter()
    root = str(ROOT)
    for ev in prof.events():
        if ev.name not in OPS:
            continue
        # only top-level ops (not the copy_ inside a cat / to)
        if ev.cpu_parent is not None and ev.cpu_parent.name in OPS:
            continue
        frames = [f for f in (ev.stack or []) if "onebit_asr" in f or "bench" in f]
        site = frames[0].split("cmu-11785-idl-1.58bit-asr_amd/")[-1] if frames else ""
        par, chain = ev.cpu_parent, []
        while par is not None:
            if not par.name.startswith("aten::"):
                chain.append(par.name)
            par = par.cpu_parent
        owner = chain[0] if chain else "(top level)"
        dev_k = [k.name[:40] for k in ev.kernels] if hasattr(ev, "kernels") else []
        shapes = str(ev.input_shapes[:2]) if ev.input_shapes else ""
        sites[(ev.name, site or owner[:70], shapes[:60], ",".join(sorted(set(dev_k)))[:50])] += 1
        per_op[ev.name] += 1
    print("per op:", dict(per_op.most_common()))
    for (name, site, shapes, ks), n in sites.most_common(120):
        print(f"{n:5d}  {name:16s} {site:70s} {shapes:60s} {ks}")
    kern = collections.Counter()
    for ev in prof.events():
        if ev.device_type == torch.autograd.DeviceType.CUDA:
            kern[ev.name[:60]] += 1
    print("device kernels (copies / fills):",
          {k: v for k, v in kern.items() if "copy" in k.lower() or "fill" in k.lower()})


if __name__ == "__main__":
    main()
