#!/usr/bin/env python3
"""Eager vs HIP-graph replay of one forward+backward (no optimizer): the whole training
step or one part of it (decoder, CTC, encoder), to localise capture problems.

The parameters never change, so every replay must reproduce the eager gradients up to
the kernels' run-to-run determinism (reported first as eager vs eager).

usage: python tools/graph_parity.py [--cfg s|cfg1] [--batch B] [--literal]
                                    [--part step|decoder|ctc|encoder] [--sdpa default|math]
"""
import argparse
import math
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "cmu-11785-idl-1.58bit-asr_amd")]

import torch  # noqa: E402


def snap(named):
    return {k: (t.detach().clone() if t is not None else None) for k, t in named.items()}


def compare(tag, a, b, top=6):
    rows, bad = [], 0
    for k in a:
        x, y = a[k], b[k]
        if x is None or y is None:
            if (x is None) != (y is None):
                rows.append((math.inf, k, "missing on one side"))
                bad += 1
            continue
        nan = (~torch.isfinite(x)).sum().item()
        d = (x - y).double()
        r = d.norm().item() / max(y.double().norm().item(), 1e-30)
        if nan:
            r = math.inf
        if r > 0:
            bad += 1
        rows.append((r, k, f"max|d| {d.abs().max().item():.3e} |ref|max {y.abs().max().item():.3e} nonfinite {nan}"))
    rows.sort(key=lambda t: t[0], reverse=True)
    print(f"== {tag}: {bad}/{len(rows)} differ; worst rel-L2 {rows[0][0]:.3e}", flush=True)
    for r, k, s in rows[:top]:
        if r > 0:
            print(f"   {r:.3e}  {k:55s} {s}", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", default="s")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--literal", action="store_true")
    ap.add_argument("--part", default="step")
    ap.add_argument("--sdpa", default="default")
    ap.add_argument("--blas", default="default")
    a = ap.parse_args()
    if a.blas != "default":
        torch.backends.cuda.preferred_blas_library(a.blas)
    if a.sdpa == "math":
        torch.backends.cuda.enable_flash_sdp(False)
        torch.backends.cuda.enable_mem_efficient_sdp(False)
        torch.backends.cuda.enable_math_sdp(True)
    from onebit_asr.conformer import ConformerASR
    from onebit_asr.ctc import ctc_loss_mean_groups
    from onebit_asr.data import CFG1, CONFORMER_S, synthetic_batch
    from onebit_asr.losses import make_att_targets
    from onebit_asr.quant import QuantizedLinear
    from onebit_asr.train_step import OneBitStep

    dev = torch.device("cuda", 0)
    cfg = dict(CONFORMER_S if a.cfg == "s" else CFG1)
    cfg.update(enc_dropout=0.0, dec_dropout=0.0)
    torch.manual_seed(1234)
    model = ConformerASR(80, 5004, **cfg).to(dev)
    n = cfg["enc_layers"]
    d = cfg["enc_d_model"]
    step = OneBitStep(model, n_layers=n, stacked=False if a.literal else True)
    if a.cfg == "s":
        batch = synthetic_batch([1000] * a.batch, [40] * a.batch, seed=1234, device=dev)
    else:
        batch = synthetic_batch([734, 349], [27, 12], seed=0, device=dev)
    bsz = batch["feats"].size(0)
    mask = [i % 2 for i in range(n)]
    bits = step.make_bits(dev)
    bits.set(mask)
    P = 3
    t_sub = 249 if a.cfg == "s" else 182
    g = torch.Generator(device=dev).manual_seed(7)
    leaf = {}
    if a.part == "decoder":
        leaf["memory"] = torch.randn(P * bsz, t_sub, d, device=dev, generator=g).requires_grad_()
        t_inp, _, t_pad = make_att_targets(batch["tokens"], 1, 2, 0)
        t_inp, t_pad = t_inp.repeat(P, 1), t_pad.repeat(P, 1)
        emask = torch.ones(P * bsz, t_sub, dtype=torch.bool, device=dev)
    elif a.part == "ctc":
        leaf["logits"] = torch.randn(P * bsz, t_sub, 5004, device=dev, generator=g).requires_grad_()
    print(f"cfg {a.cfg} batch {bsz} part {a.part} literal {a.literal} sdpa {a.sdpa}", flush=True)

    def fwd_bwd():
        for p in model.parameters():
            p.grad = None
        for t in leaf.values():
            t.grad = None
        if a.part == "step":
            loss, _ = step(batch, bits)
        elif a.part == "decoder":
            lg = model.decode_logits(leaf["memory"], emask, t_inp, t_pad)
            loss = lg.square().mean()
        elif a.part == "ctc":
            lp = torch.log_softmax(leaf["logits"], dim=-1)
            il = torch.full((P * bsz,), t_sub, dtype=torch.int64, device=dev)
            loss = ctc_loss_mean_groups(lp, batch["tokens"].repeat(P, 1), il,
                                        batch["token_lens"].repeat(P), 3, P).sum()
        elif a.part == "encoder":
            enc, _, ctc = model(batch, precision=2, sp_mask=bits)
            loss = enc.square().mean() + ctc.square().mean()
        else:
            raise SystemExit(f"unknown part {a.part}")
        loss.backward()
        return loss.detach()

    def grads():
        out = {k: p.grad for k, p in model.named_parameters()}
        out.update({"leaf." + k: t.grad for k, t in leaf.items()})
        return snap(out)

    l1 = fwd_bwd()
    e1 = grads()
    l2 = fwd_bwd()
    e2 = grads()
    torch.cuda.synchronize()
    print(f"eager loss {l1.item():.6f} / {l2.item():.6f}", flush=True)
    compare("eager vs eager", e2, e1)
    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        for _ in range(2):
            fwd_bwd()
    torch.cuda.current_stream(dev).wait_stream(side)
    torch.cuda.synchronize()
    for m in model.modules():
        if isinstance(m, QuantizedLinear):
            m._codes_cache = {}
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        lg = fwd_bwd()
    prev = None
    for r in range(3):
        graph.replay()
        torch.cuda.synchronize()
        cur = grads()
        print(f"replay#{r + 1} loss {lg.item():.6f}", flush=True)
        compare(f"replay#{r + 1} vs eager", cur, e1)
        prev = cur
    fwd_bwd()
    compare("eager-after-graph vs eager", grads(), e1)
    del prev


if __name__ == "__main__":
    main()
