#!/usr/bin/env python
"""Summarise a rocprofv3 kernel_stats CSV: top kernels by total time, per step.
Usage: tools/kstats.py run_kernel_stats.csv [steps]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total GPU kernel time {tot/1e6:.3f} ms  ({tot/1e6/steps:.3f} ms per step over {steps:g} steps)")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:28]:
    t = float(r["TotalDurationNs"])
    print(f"{t/1e6/steps:8.3f} ms/step {int(r['Calls'])/steps:6.1f} calls/step avg {float(r['AverageNs'])/1e3:8.2f} us "
          f"{100*t/tot:5.1f}%  {r['Name'][:95]}")
