#!/usr/bin/env python
"""Per-launch memory traffic of the bench's roofline kernels from rocprofv3 PMC passes.

Collect (two separate passes, counters only, program directly after `--`):
    rocprofv3 --pmc FETCH_SIZE --output-format csv -d OUT/fetch -o run -- python bench.py ...
    rocprofv3 --pmc WRITE_SIZE --output-format csv -d OUT/write -o run -- python bench.py ...
then:
    python tools/traffic.py OUT profiles/traffic_r01.json

FETCH_SIZE / WRITE_SIZE are in KiB. On gfx950 FETCH_SIZE reports half the bytes of 16-B/lane
streaming reads (MI355X_MICROARCH.md, HBM section), so traffic = 2 * FETCH + WRITE. Both count
memory-side (fabric) requests, which include Infinity Cache hits, so this is an upper bound on
HBM bytes.
"""
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict

# bench roofline kernels: key -> kernel-name substrings (either matches)
KERNELS = {
    "gemm_fwd_h3": ("k_gemm_x6<1, 0, 1, 256, 256, 4, 2, 0,",),   # f16x3 forward GEMM (256x256 tiles)
    "gemm_dgrad": ("k_gemm_h3p<128, 256, 2, 4, 4,", "k_gemm_x6<1, 0, 1, 128, 256, 2, 4, 8,",
                   "k_gemm_x6<1, 0, 1, 128, 256, 2, 4, 0,"),   # dgrad (pipelined kernel since round 6)
    "gemm_wgrad": ("k_gemm_x6<1, 1, 0, 256, 256, 4, 2, 0,",),   # wgrad (split-K partial products)
    "sage_fwd": ("k_seg_group<2, 0, 1,", "k_seg_sweep<2, 0, 1,"),   # fused SAGE forward aggregation
    "spmm_bwd": ("k_seg_group<2, 0, 0,", "k_seg_sweep<2, 0, 0,"),   # transpose aggregation
    "ea_edge_b16": ("k_gemm_b16<",),   # EA_GNN bf16 per-edge Linears (gathered and plain epilogues)
    "ea_wgrad_b16": ("k_gemm_x6<2, 1, 0, 256, 256, 4, 2, 19,",),   # EA_GNN bf16 per-edge weight gradients
}


def per_launch(pass_dir, counter):
    vals = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(os.path.join(pass_dir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            vals[r["Kernel_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    out = {}
    for key, pat in KERNELS.items():
        xs = [v for name, d in vals.items() if any(p in name for p in pat) for v in d.values()]
        if xs:
            out[key] = statistics.median(xs) * 1024.0
    return out


def main():
    root, dst = sys.argv[1], sys.argv[2]
    fetch = per_launch(os.path.join(root, "fetch"), "FETCH_SIZE")
    write = per_launch(os.path.join(root, "write"), "WRITE_SIZE")
    res = {"method": "2*FETCH_SIZE + WRITE_SIZE per launch (KiB->bytes, median over launches), "
                     "rocprofv3 --pmc, separate passes; fabric-side, includes Infinity Cache hits",
           "kernels": {}}
    for key in KERNELS:
        if key in fetch and key in write:
            res["kernels"][key] = {"kernel_pattern": list(KERNELS[key]), "fetch_bytes": 2 * fetch[key],
                                   "write_bytes": write[key], "bytes_per_launch": 2 * fetch[key] + write[key]}
    json.dump(res, open(dst, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
