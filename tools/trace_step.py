#!/usr/bin/env python3
"""Per-step kernel breakdown from a rocprofv3 kernel trace: takes the LAST `--steps`
occurrences of a per-step marker kernel window and groups kernel time by name/grid.
usage: trace_step.py run_kernel_trace.csv [--marker ctc_beta_kernel] [--per-step 3]"""
import argparse
import collections
import csv
import re


def short(name):
    """Kernel name without its parameter list (first '(' outside template brackets)."""
    name = name.replace("at::native::", "").replace("(anonymous namespace)::", "")
    depth = 0
    for i, c in enumerate(name):
        if c == "<":
            depth += 1
        elif c == ">":
            depth -= 1
        elif c == "(" and depth == 0 and i > 0 and not name[:i].endswith("operator"):
            name = name[:i]
            break
    name = re.sub(r"^void ", "", name)
    name = name.replace("at::native::", "").replace("(anonymous namespace)::", "")
    return name[:130]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="ctc_beta_kernel")
    ap.add_argument("--per-step", type=int, default=3, help="marker launches per step")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--by-grid", action="store_true")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    # last step = between the end of the marker group before the last and the last marker
    k = a.per_step
    last = marks[-1]
    prev = marks[-1 - k]
    sel = rows[prev + 1:last + 1]
    t0 = int(sel[0]["Start_Timestamp"])
    t1 = int(sel[-1]["End_Timestamp"])
    agg = collections.defaultdict(lambda: [0, 0.0])
    busy = 0.0
    for r in sel:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        key = short(r["Kernel_Name"])
        if a.by_grid:
            key += f" grid={r['Grid_Size_X']}x{r['Grid_Size_Y']} wg={r['Workgroup_Size_X']}"
        agg[key][0] += 1
        agg[key][1] += d
        busy += d
    print(f"window {len(sel)} kernels, span {(t1 - t0) / 1e3:.1f} us, busy {busy:.1f} us")
    for key, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"{t / 1e3:8.3f} ms {n:6d} {t / n:8.1f} us  {key}")


if __name__ == "__main__":
    main()
