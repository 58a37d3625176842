#!/usr/bin/env python
"""Median per-dispatch counters (and duration, clock) of the kernels matching the given
substrings, from tools/pmc_passes.sh output. Usage: tools/pmc_table.py OUTDIR pattern ..."""
import csv
import glob
import os
import statistics
import sys
from collections import defaultdict


def main():
    root, pats = sys.argv[1], sys.argv[2:]
    vals = defaultdict(lambda: defaultdict(list))
    durs = defaultdict(list)
    for d in sorted(glob.glob(os.path.join(root, "pass*"))):
        kt = {}
        for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                kt[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        per = defaultdict(lambda: defaultdict(float))
        names = {}
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if not any(p in r["Kernel_Name"] for p in pats):
                    continue
                per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
                names[r["Dispatch_Id"]] = r["Kernel_Name"]
        for did, cs in per.items():
            k = names[did]
            for c, v in cs.items():
                vals[k][c].append(v)
            if did in kt:
                durs[k].append(kt[did])
    for k, cs in vals.items():
        dur = statistics.median(durs[k]) if durs[k] else 0
        print(f"{k[:100]}  median {dur / 1e3:.1f} us")
        for c, v in sorted(cs.items()):
            m = statistics.median(v)
            extra = f"   -> {m / 8 / dur:.2f} GHz" if c == "GRBM_GUI_ACTIVE" and dur else ""
            print(f"    {c:42s} {m:18.1f}{extra}")


if __name__ == "__main__":
    main()
