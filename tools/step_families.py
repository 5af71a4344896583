#!/usr/bin/env python3
"""Kernel time of the LAST training step in a rocprofv3 kernel trace (the window between the
last two AdamW launch groups, as step_window.py), summed by kernel family.
usage: step_families.py run_kernel_trace.csv"""
import collections
import csv
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).parent))
from trace_step import short  # noqa: E402

# first matching prefix wins (order matters: dgemm_kc before dgemm, dw_grouped before dw_)
FAMILIES = [
    ("relattn", "attention (rel-pos MHSA core)"),
    ("tgemm", "ternary GEMM (+ fused epilogues)"),
    ("dw_grouped", "grouped weight gradients"),
    ("dwg_", "grouped weight gradients"),
    ("dgemm_kc", "dense GEMM, K-chunked (CTC head dX)"),
    ("dgemm", "dense GEMM (pointwise convs, decoder)"),
    ("ss_", "Conv2dSubsampling"),
    ("cm_", "conv module core"),
    ("ln_", "LayerNorm"),
    ("dw_", "other weight gradients (V = 5004 head, decoder)"),
    ("ctc", "CTC"),
    ("Cijk", "hipBLASLt"),
    ("decattn", "decoder attention"),
    ("adamw", "optimizer"),
    ("quant", "weight codes"),
    ("att_kl", "CE / KL losses"),
    ("seqloss", "CE / KL losses"),
    ("loss_", "CE / KL losses"),
    ("Fill", "torch fills"),
    ("copyBuffer", "copies"),
]


def family(name):
    for pre, fam in FAMILIES:
        if pre in name:
            return fam
    return "other (torch glue, small launches)"


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    names = [short(r["Kernel_Name"]) for r in rows]
    idx = [i for i, n in enumerate(names) if "adamw" in n.lower()]
    starts = [idx[0]] + [idx[i] for i in range(1, len(idx)) if idx[i] - idx[i - 1] > 50]
    a, b = starts[-2] + 1, starts[-1]
    while b + 1 < len(names) and "adamw" in names[b + 1].lower():
        b += 1
    agg = collections.defaultdict(lambda: [0.0, 0])
    tot = 0.0
    for i in range(a, b + 1):
        d = (int(rows[i]["End_Timestamp"]) - int(rows[i]["Start_Timestamp"])) / 1e3
        f = family(names[i])
        agg[f][0] += d
        agg[f][1] += 1
        tot += d
    print(f"step window: {b - a + 1} kernels, kernel time {tot / 1e3:.2f} ms")
    for f, (t, c) in sorted(agg.items(), key=lambda kv: -kv[1][0]):
        print(f"{t / 1e3:8.3f} ms {c:5d} launches  {100 * t / tot:5.1f} %  {f}")


if __name__ == "__main__":
    main()
