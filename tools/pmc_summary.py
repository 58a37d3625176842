#!/usr/bin/env python
"""Summarise rocprofv3 --pmc CSVs (tools/pmc_profile.sh output): per kernel, the mean of
each counter per dispatch. Usage: tools/pmc_summary.py OUTDIR [kernel-substring ...]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    out = sys.argv[1]
    pats = sys.argv[2:]
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(out, "pass*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "")
            if pats and not any(p in name for p in pats):
                continue
            vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in vals.items():
        print(k[:120])
        for c, v in sorted(cs.items()):
            print(f"    {c:40s} {sum(v)/len(v):16.1f}   (n={len(v)})")


if __name__ == "__main__":
    main()
