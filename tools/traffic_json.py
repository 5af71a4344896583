#!/usr/bin/env python3
"""HBM bytes per launch of the BitLinear kernel families from tools/traffic.sh output.

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch. gfx950 correction (MI355X_MICROARCH.md,
HBM/rocprofv3 section): FETCH_SIZE reports half the bytes of a wide coalesced streaming
read, so it is doubled; WRITE_SIZE is taken as is. Per (shape, op) the median over the
timed dispatches of each kernel is used; the weight gradients are one grouped launch a step
(dw_grouped_kernel). Families are weighted by launches per training
step exactly as bench.py's roofline() weights its time and algorithmic bytes.

usage: python tools/traffic_json.py gpurun_out/TAG > profiles/pmc_traffic.json"""
import csv
import glob
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]

# launches per step (bench.py ql_shapes at Conformer-S: 16 blocks, 2 FFNs, 4 q/k/v/out)
COUNT = {"lin1": 32, "lin2": 32, "qkvo": 64, "pos": 16}
KERNELS = {"fwd": ("tgemm",), "dx": ("tgemm",)}


def per_dispatch(path, sub):
    vals = {}
    for f in glob.glob(f"{path}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if sub in r["Kernel_Name"]:
                vals.setdefault(r.get("Dispatch_Id", len(vals)), 0.0)
                vals[r.get("Dispatch_Id", len(vals))] += float(r["Counter_Value"])
    return statistics.median(vals.values()) if vals else None


def main():
    d = sys.argv[1]
    sys.path[:0] = [str(ROOT / "cmu-11785-idl-1.58bit-asr_amd")]
    from onebit_asr._lib import source_digest

    out, fam = {"source": d, "note": __doc__.split("\n\n")[1].replace("\n", " "),
                "csrc_sha256": source_digest()}, {}
    for shape, cnt in COUNT.items():
        for op, subs in KERNELS.items():
            if shape == "pos" and op == "dx":
                continue  # pos_emb needs no input gradient (bench.py n_dx)
            tot = 0.0
            for sub in subs:
                f = per_dispatch(f"{d}/{shape}_{op}_FETCH_SIZE", sub)
                w = per_dispatch(f"{d}/{shape}_{op}_WRITE_SIZE", sub)
                if f is None or w is None:
                    raise SystemExit(f"missing counters for {shape} {op} {sub}")
                tot += (2.0 * f + w) * 1024.0
            out[f"{shape}_{op}_hbm_bytes"] = int(tot)
            key = "ternary_gemm"
            b, n = fam.get(key, (0.0, 0))
            fam[key] = (b + cnt * tot, n + cnt)
    for key, (b, n) in fam.items():
        out[key] = {"hbm_bytes_per_launch": int(b / n), "launches_per_step": n}
    # the grouped dW launch: one a step (median over the eager dispatches of dwg_bench.py,
    # its composition recorded from a step's backward)
    f = per_dispatch(f"{d}/dwg_FETCH_SIZE", "dw_grouped")
    w = per_dispatch(f"{d}/dwg_WRITE_SIZE", "dw_grouped")
    if f is None or w is None:
        raise SystemExit("missing counters for dw_grouped")
    out["dw_grouped"] = {"hbm_bytes_per_launch": int((2.0 * f + w) * 1024.0),
                         "launches_per_step": 1}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
