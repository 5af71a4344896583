#!/usr/bin/env python3
"""Graph vs eager loss trace of the training step (debug aid).
usage: python tools/debug_graph.py [--cfg s|cfg1] [--steps N] [--dropout-off]"""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "cmu-11785-idl-1.58bit-asr_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", default="s")
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--mode", default="graph", choices=["graph", "eager-gs", "eager"])
    ap.add_argument("--torch-opt", action="store_true", help="GraphedTrainStep with torch AdamW")
    ap.add_argument("--literal", action="store_true", help="three literal passes (not stacked)")
    a = ap.parse_args()
    from onebit_asr.conformer import ConformerASR
    from onebit_asr.data import CFG1, CONFORMER_S, synthetic_batch
    from onebit_asr.graph_step import GraphedTrainStep
    from onebit_asr.train_step import OneBitStep, PART_NAMES, WarmupCosine, make_optimizer, sample_sp_mask, train_step

    dev = torch.device("cuda", 0)
    cfg = CONFORMER_S if a.cfg == "s" else CFG1
    torch.manual_seed(1234)
    model = ConformerASR(80, 5004, **cfg).to(dev)
    n = cfg["enc_layers"]
    step = OneBitStep(model, n_layers=n, stacked=False if a.literal else None)
    batch = synthetic_batch([1000] * a.batch, [40] * a.batch, seed=1234, device=dev)
    print(f"mode {a.mode} batch {a.batch} steps {a.steps}", flush=True)
    gen = torch.Generator().manual_seed(4321)
    if a.mode == "eager":
        opt = make_optimizer(model.parameters())
        sched = WarmupCosine(opt, 4000, 100000)
        fn = lambda m: train_step(step, opt, sched, batch, m)  # noqa: E731
    else:
        gs = GraphedTrainStep(step, n, warmup_iters=2, use_graph=(a.mode == "graph"),
                              fused_optimizer=not a.torch_opt)
        fn = lambda m: gs.step(batch, m)  # noqa: E731
    for i in range(a.steps):
        loss, parts = fn(sample_sp_mask(n, generator=gen))
        torch.cuda.synchronize()
        pv = parts.tolist()
        print(f"step {i} loss {loss.item():.5f} " + " ".join(f"{k}={v:.4f}" for k, v in zip(PART_NAMES, pv)),
              flush=True)
        bad = [k for k, p in model.named_parameters() if not torch.isfinite(p).all()]
        badg = [k for k, p in model.named_parameters()
                if p.grad is not None and not torch.isfinite(p.grad).all()]
        if badg:
            print("non-finite grads:", badg[:10], flush=True)
        if bad:
            print("non-finite params:", bad[:10], flush=True)
            if a.mode != "eager" and getattr(gs, "fused", False):
                opt = gs.opt
                names = {id(p): k for k, p in model.named_parameters()}
                tab = opt.table.cpu().tolist()
                for j, i in enumerate(opt._members):
                    p = opt.params[i]
                    if names[id(p)] in bad[:3]:
                        print(names[id(p)], "table", tab[j], "grad_ptr", p.grad.data_ptr(),
                              "param_ptr", p.data_ptr(), "numel", p.numel(),
                              "m finite", bool(torch.isfinite(opt.exp_avg[i]).all()),
                              "v finite", bool(torch.isfinite(opt.exp_avg_sq[i]).all()),
                              "grad", p.grad.flatten()[:4].tolist(), flush=True)
            break


if __name__ == "__main__":
    main()
