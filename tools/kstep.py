#!/usr/bin/env python
"""Per-step kernel time from a rocprofv3 --stats kernel CSV: total / steps for the top kernels.
    python tools/kstep.py run_kernel_stats.csv STEPS [N]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2])
n = int(sys.argv[3]) if len(sys.argv) > 3 else 25
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total {tot / 1e6:.2f} ms over the profile, {tot / steps / 1e3:.1f} us per step ({steps:g} steps incl. warm-up)")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:n]:
    t = float(r["TotalDurationNs"])
    print(f"{t / steps / 1e3:9.1f} us/step {int(r['Calls']) / steps:6.1f}/step {float(r['AverageNs']) / 1e3:9.1f} us avg "
          f"{t / tot * 100:5.1f}%  {r['Name'][:100]}")
