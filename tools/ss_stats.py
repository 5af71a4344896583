"""Per-call averages of the kernels matching a pattern in a rocprofv3 kernel_stats csv."""
import csv
import sys

path = sys.argv[1]
pats = sys.argv[2].split(",") if len(sys.argv) > 2 else ["ss_"]
rows = list(csv.DictReader(open(path)))
tot = 0.0
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    if any(p in r["Name"] for p in pats):
        avg = float(r["AverageNs"]) / 1e3
        tot += avg
        print(f"{avg:9.1f} us  x{int(r['Calls']):4d}  {r['Name'][:100]}")
print(f"sum of per-call averages: {tot:.1f} us")
