"""Print the top kernels of a rocprofv3 --stats kernel_stats.csv (per step if --steps)."""
import csv
import sys

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total {tot / 1e6:.2f} ms ({tot / 1e6 / steps:.2f} ms/step over {steps:g} steps)")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
    t = float(r["TotalDurationNs"]) / 1e6
    print(f"{t / steps:8.3f} ms/step {int(r['Calls']) / steps:7.1f} calls/step "
          f"{float(r['AverageNs']) / 1e3:9.2f} us avg {float(r['Percentage']):6.2f}%  {r['Name'][:100]}")
