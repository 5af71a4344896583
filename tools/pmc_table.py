#!/usr/bin/env python3
"""Per-kernel limiter table from tools/pmc_step.sh passes: median counters per dispatch of
each kernel (by full name, template arguments included) over the profiled step, and the
derived rates the limiter is read from. usage: pmc_table.py DIR [min_calls] [--json]

Units (MI355X_MICROARCH.md): SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count
quad-cycles; SQ_VALU_MFMA_BUSY_CYCLES counts cycles summed over SIMDs; GRBM_GUI_ACTIVE is
the sum over the 8 XCDs, so the kernel's span in cycles is GRBM_GUI_ACTIVE / 8.
  mfma_busy  = SQ_VALU_MFMA_BUSY_CYCLES / (span * 1024 SIMDs)
  waves/CU   = 4 * SQ_WAVE_CYCLES / (span * 256 CUs)     (mean resident waves per CU)
  wait/issue/active = SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES
  lds_conf   = SQ_LDS_BANK_CONFLICT / SQ_ACTIVE_INST_LDS (extra cycles per LDS-active cycle)
  hbm_MB     = (2 * FETCH_SIZE + WRITE_SIZE) KiB per dispatch (gfx950 FETCH x2 correction)
"""
import collections
import csv
import glob
import json
import re
import statistics
import sys


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*$", "", name)  # drop the argument list
    name = name.replace("void ", "")
    return name[:70]


def load(d):
    vals = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
    calls = collections.Counter()
    for f in sorted(glob.glob(f"{d}/p*/**/*counter_collection.csv", recursive=True)):
        seen = set()
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            key = (f, r["Dispatch_Id"])
            vals[k][r["Counter_Name"]][key] += float(r["Counter_Value"])
            if "p1/" in f and key not in seen:
                seen.add(key)
                calls[k] += 1
    return {k: {c: statistics.median(v.values()) for c, v in cs.items()} for k, cs in vals.items()}, calls


def derive(m):
    out = {}
    span = m.get("GRBM_GUI_ACTIVE", 0) / 8
    wc = m.get("SQ_WAVE_CYCLES", 0)
    if span:
        out["span_us@2.4GHz"] = span / 2400
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            out["mfma_busy"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (span * 1024)
        if wc:
            out["waves_per_CU"] = 4 * wc / (span * 256)
    if wc:
        for c, n in (("SQ_WAIT_ANY", "wait"), ("SQ_WAIT_INST_ANY", "issue_stall"),
                     ("SQ_ACTIVE_INST_ANY", "active"), ("SQ_ACTIVE_INST_VALU", "valu_active"),
                     ("SQ_ACTIVE_INST_LDS", "lds_active"), ("SQ_ACTIVE_INST_VMEM", "vmem_active")):
            if c in m:
                out[n] = m[c] / wc
    if m.get("SQ_INSTS_MFMA"):
        out["valu_per_mfma"] = m.get("SQ_INSTS_VALU", 0) / m["SQ_INSTS_MFMA"]
    if m.get("SQ_ACTIVE_INST_LDS"):
        out["lds_conf"] = m.get("SQ_LDS_BANK_CONFLICT", 0) / m["SQ_ACTIVE_INST_LDS"]
    if "FETCH_SIZE" in m or "WRITE_SIZE" in m:
        out["hbm_MB"] = (2 * m.get("FETCH_SIZE", 0) + m.get("WRITE_SIZE", 0)) * 1024 / 1e6
    h, mi = m.get("TCC_HIT_sum"), m.get("TCC_MISS_sum")
    if h is not None and mi:
        out["l2_hit"] = h / (h + mi)
    return out


def main():
    d = sys.argv[1]
    min_calls = int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2].isdigit() else 1
    med, calls = load(d)
    rows = []
    for k, m in med.items():
        if calls[k] < min_calls:
            continue
        dv = derive(m)
        rows.append((k, calls[k], m, dv))
    rows.sort(key=lambda r: -r[1] * r[3].get("span_us@2.4GHz", 0))
    if "--json" in sys.argv:
        print(json.dumps({k: {"calls": c, "counters": m, "derived": dv} for k, c, m, dv in rows}, indent=1))
        return
    cols = ["span_us@2.4GHz", "mfma_busy", "waves_per_CU", "active", "wait", "issue_stall",
            "valu_active", "lds_active", "lds_conf", "valu_per_mfma", "hbm_MB", "l2_hit"]
    print("| kernel | calls | " + " | ".join(cols) + " |")
    print("|---|---|" + "---|" * len(cols))
    for k, c, m, dv in rows:
        cells = [f"{dv[x]:.3g}" if x in dv else "" for x in cols]
        print(f"| `{k}` | {c} | " + " | ".join(cells) + " |")


if __name__ == "__main__":
    main()
