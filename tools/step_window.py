#!/usr/bin/env python3
"""Kernel time of the LAST training step in a rocprofv3 kernel trace (window between the
last two AdamW launches), grouped by kernel. usage: step_window.py run_kernel_trace.csv [top]"""
import collections
import csv
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).parent))
from trace_step import short  # noqa: E402

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
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
    agg[names[i]][0] += d
    agg[names[i]][1] += 1
    tot += d
span = (int(rows[b]["End_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3
print(f"step window: {b - a + 1} kernels, kernel time {tot / 1e3:.2f} ms, span {span / 1e3:.2f} ms")
for n, (t, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:top]:
    print(f"{t / 1e3:8.3f} ms {c:5d} x {t / c:8.1f} us  {n[:110]}")
