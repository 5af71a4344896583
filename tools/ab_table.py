#!/usr/bin/env python3
"""Per-kernel table of tools/ab_prof.sh sides: average us per call of every kernel family
matching a pattern, one column per side, and each side's bench ms/step.
usage: ab_table.py DIR side1 side2 ... [--match tgemm,dgemm]"""
import csv
import json
import sys

d = sys.argv[1]
args = [a for a in sys.argv[2:] if not a.startswith("--")]
pat = next((a.split("=", 1)[1] for a in sys.argv[2:] if a.startswith("--match=")), "")
pats = [p for p in pat.split(",") if p]
tabs = {}
for s in args:
    t = {}
    for r in csv.DictReader(open(f"{d}/{s}/run_kernel_stats.csv")):
        t[r["Name"].replace("(anonymous namespace)::", "")[:88]] = (int(r["Calls"]), float(r["AverageNs"]) / 1e3)
    tabs[s] = t
    ms = None
    for line in open(f"{d}/{s}.log"):
        if line.startswith("{"):
            ms = json.loads(line).get("ms_per_step")
    print(f"{s}: {ms} ms/step")
keys = sorted({k for t in tabs.values() for k in t if not pats or any(p in k for p in pats)},
              key=lambda k: -max(t.get(k, (0, 0))[1] * t.get(k, (0, 0))[0] for t in tabs.values()))
print("| kernel | " + " | ".join(args) + " |")
print("|---|" + "---|" * len(args))
for k in keys[:40]:
    print(f"| `{k[:80]}` | " + " | ".join(f"{tabs[s][k][1]:.1f}" if k in tabs[s] else "" for s in args) + " |")
