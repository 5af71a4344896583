#!/usr/bin/env python3
"""The grouped weight-gradient launch (ob_dw_grouped) alone, at the composition one Conformer-S
training step's backward issues: one eager stacked step (B = 32 x 1000 frames) records the
composition (deferred.LAST_DWG), then bench.roofline_dwg launches it on fresh buffers.
Prints us per launch and the algorithmic bytes / FLOPs. Eager launches with --no-graph (the
PMC passes of tools/traffic.sh count per dispatch).

usage: python tools/dwg_bench.py [--reps N] [--no-graph] [--bitlinear-only]"""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "cmu-11785-idl-1.58bit-asr_amd")]

import torch  # noqa: E402

import bench  # noqa: E402


def step_composition(dev):
    from onebit_asr import deferred
    from onebit_asr.conformer import ConformerASR
    from onebit_asr.data import CONFORMER_S, synthetic_batch
    from onebit_asr.train_step import OneBitStep, sample_sp_mask

    torch.manual_seed(0)
    model = ConformerASR(bench.N_MELS, bench.VOCAB, **CONFORMER_S).to(dev)
    step = OneBitStep(model, n_layers=CONFORMER_S["enc_layers"])
    batch = synthetic_batch([1000] * 32, [40] * 32, seed=1, device=dev)
    mask = sample_sp_mask(CONFORMER_S["enc_layers"], generator=torch.Generator().manual_seed(2))
    bits = step.make_bits(dev)
    bits.set(mask)
    with deferred.scope():
        loss, _ = step(batch, bits)
        loss.backward()
    torch.cuda.synchronize()
    shapes = list(deferred.LAST_DWG)
    del model, step, batch, loss
    torch.cuda.empty_cache()
    return shapes


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--bitlinear-only", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    shapes = (bench.dwg_bitlinear_shapes(32, 1000) if a.bitlinear_only else step_composition(dev))
    us, by, fl, cyc, det = bench.roofline_dwg(dev, shapes, not a.bitlinear_only, reps=a.reps,
                                              graph_replay=not a.no_graph)
    print(f"dw_grouped: {det['gemms']} gemms ({det['bitlinear_gemms']} BitLinear), {us:.1f} us "
          f"per launch, {by / 1e6:.1f} MB, {fl / 1e9:.1f} GFLOP -> {fl / us / 1e6:.1f} TFLOP/s, "
          f"{by / us / 1e3:.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
