#!/usr/bin/env python
"""Summarise rocprofv3 --stats kernel tables (run_kernel_stats.csv): calls, avg and total time,
share, sorted by total. Usage: tools/kstats.py path/to/run_kernel_stats.csv [top]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"{len(rows)} kernels, {tot / 1e6:.3f} ms total")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
    print(f"{float(r['Percentage']):6.2f}% {int(r['Calls']):5d} x {float(r['AverageNs']) / 1e3:9.1f} us  {r['Name'][:100]}")
