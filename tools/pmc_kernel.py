#!/usr/bin/env python3
"""Median PMC counters per dispatch of kernels whose name contains a substring, plus derived
rates. usage: pmc_kernel.py DIR substring"""
import collections
import csv
import glob
import statistics
import sys

d, sub = sys.argv[1], sys.argv[2]
vals = collections.defaultdict(lambda: collections.defaultdict(float))
for f in sorted(glob.glob(f"{d}/p*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        if sub in r["Kernel_Name"]:
            vals[r["Counter_Name"]][(f, r["Dispatch_Id"])] += float(r["Counter_Value"])
med = {c: statistics.median(v.values()) for c, v in vals.items()}
for c in sorted(med):
    print(f"{c:28s} {med[c]:16.1f}")
if "SQ_WAVE_CYCLES" in med and med["SQ_WAVE_CYCLES"]:
    wc = med["SQ_WAVE_CYCLES"]
    for c in ["SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
              "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM"]:
        if c in med:
            print(f"  {c} / WAVE_CYCLES = {med[c] / wc:.3f}")
