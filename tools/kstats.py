#!/usr/bin/env python3
"""Print a rocprofv3 kernel_stats.csv sorted by total time. usage: kstats.py DIR [N]"""
import csv, glob, sys
f = glob.glob(f"{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)[0]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:n]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.3f} ms {int(r['Calls']):6d} calls "
          f"{float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:100]}")
