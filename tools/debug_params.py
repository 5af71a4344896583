#!/usr/bin/env python3
"""Graph vs eager GraphedTrainStep on cfg1 (as tests/test_graph_step_gpu.py): per step, the
largest parameter / gradient differences (debug aid)."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "cmu-11785-idl-1.58bit-asr_amd")]

import torch  # noqa: E402


def run(use_graph, dev):
    from onebit_asr.conformer import ConformerASR
    from onebit_asr.data import CFG1, synthetic_batch
    from onebit_asr.graph_step import GraphedTrainStep
    from onebit_asr.train_step import OneBitStep

    torch.manual_seed(0)
    model = ConformerASR(80, 5004, **CFG1).to(dev)
    gs = GraphedTrainStep(OneBitStep(model, n_layers=2), n_layers=2, warmup_iters=2,
                          warmup_steps=4, total_steps=20, use_graph=use_graph)
    b1 = synthetic_batch([734, 349], [27, 12], seed=0, device=dev)
    b2 = synthetic_batch([734, 349], [27, 12], seed=1, device=dev)
    snaps = []
    for mask, b in zip([[1, 0], [0, 1], [1, 1], [0, 0]], [b1, b1, b1, b2]):
        loss, _ = gs.step(b, mask)
        torch.cuda.synchronize()
        snaps.append(({k: p.detach().clone() for k, p in model.named_parameters()},
                      {k: (p.grad.detach().clone() if p.grad is not None else None)
                       for k, p in model.named_parameters()}, loss.item()))
    return snaps


def warm_other_work(dev):
    """GPU work before the comparison (as in a pytest session): LN fwd/bwd at several shapes."""
    from onebit_asr.layernorm import layer_norm

    for rows, d in [(1, 1), (7, 64), (23904, 144), (333, 144), (50, 256), (3, 500), (1000, 17)]:
        x = torch.randn(rows, d, device=dev, requires_grad=True)
        w = torch.randn(d, device=dev, requires_grad=True)
        b = torch.randn(d, device=dev, requires_grad=True)
        layer_norm(x, w, b, 1e-5).backward(torch.randn(rows, d, device=dev))
    torch.cuda.synchronize()


def main():
    dev = torch.device("cuda", 0)
    if "--warm" in sys.argv:
        warm_other_work(dev)
    g = run(True, dev)
    e = run(False, dev)
    for s, ((pg, gg, lg), (pe, ge, le)) in enumerate(zip(g, e)):
        print(f"step {s}: loss graph {lg:.6f} eager {le:.6f}")
        diffs = sorted(((pg[k] - pe[k]).abs().max().item(), k) for k in pg)[-5:]
        for d, k in diffs:
            print(f"   param {k:50s} max|diff| {d:.3e}")
        for k in ("encoder.blocks.0.conv.dw.bias",):
            a, b = gg.get(k), ge.get(k)
            print(f"   {k}: p_g {pg[k][:4].tolist()} p_e {pe[k][:4].tolist()}")
            if a is not None and b is not None:
                print(f"      grad_g {a[:4].tolist()} grad_e {b[:4].tolist()} max {a.abs().max().item():.3e} {b.abs().max().item():.3e}")


if __name__ == "__main__":
    main()
