#!/usr/bin/env python3
"""Bisect HIP-graph replay corruption in the decoder head: a stock 2-layer
nn.TransformerDecoder (batch_first, relu, dropout 0) + final LN + Linear(vocab), with
each of the package's own pieces switched in or out (--ob-ln, --ob-emb), the loss as
torch's mean or as a sum. Prints per-replay worst gradient error vs eager."""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "cmu-11785-idl-1.58bit-asr_amd")]

import torch  # noqa: E402
import torch.nn as nn  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ob-ln", action="store_true")
    ap.add_argument("--ob-emb", action="store_true")
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--no-mask", action="store_true")
    ap.add_argument("--vocab", type=int, default=5004)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    d, B, U, T = 144, 96, 41, 249
    emb = nn.Embedding(a.vocab, d, padding_idx=0).to(dev)
    layer = nn.TransformerDecoderLayer(d, 4, 1024, 0.0, batch_first=True)
    dec = nn.TransformerDecoder(layer, a.layers).to(dev)
    ln = nn.LayerNorm(d).to(dev)
    out = nn.Linear(d, a.vocab).to(dev)
    g = torch.Generator(device=dev).manual_seed(1)
    mem = torch.randn(B, T, d, device=dev, generator=g).requires_grad_()
    tok = torch.randint(4, a.vocab, (B, U), device=dev, generator=g)
    pad = torch.zeros(B, U, dtype=torch.bool, device=dev)
    pad[:, U - 3:] = True
    mmask = torch.zeros(B, T, dtype=torch.bool, device=dev)
    from onebit_asr.embedding import embedding
    from onebit_asr.layernorm import layer_norm

    mods = {"emb": emb, "dec": dec, "ln": ln, "out": out}
    params = {f"{m}.{k}": p for m, mod in mods.items() for k, p in mod.named_parameters()}
    params["mem"] = mem

    def fwd_bwd():
        for p in params.values():
            p.grad = None
        x = embedding(tok, emb.weight, 0) if a.ob_emb else emb(tok)
        fut = torch.ones(U, U, device=dev).triu(1).bool()
        causal = torch.zeros(U, U, device=dev).masked_fill(fut, float("-inf"))
        if a.no_mask:
            y = dec(x, mem, tgt_mask=causal, tgt_is_causal=True)
        else:
            y = dec(x, mem, tgt_mask=causal, memory_key_padding_mask=mmask,
                    tgt_key_padding_mask=pad, tgt_is_causal=True)
        y = layer_norm(y, ln.weight, ln.bias, ln.eps) if a.ob_ln else ln(y)
        loss = out(y).square().mean()
        loss.backward()
        return loss.detach()

    def snap():
        return {k: p.grad.detach().clone() for k, p in params.items() if p.grad is not None}

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
        errs = sorted((((cur[k] - ref[k]).norm() / ref[k].norm().clamp_min(1e-30)).item(), k) for k in ref)
        worst = max(worst, errs[-1][0])
        print(f"  replay#{r + 1}: worst {errs[-1][0]:.2e} {errs[-1][1]}  next {errs[-2][0]:.2e} {errs[-2][1]}",
              flush=True)
    print(f"RESULT {' '.join(sys.argv[1:]) or 'stock'}: worst={worst:.2e} "
          f"{'OK' if worst < 1e-5 else 'CORRUPT'}", flush=True)


if __name__ == "__main__":
    main()
