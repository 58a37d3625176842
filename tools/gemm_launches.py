#!/usr/bin/env python
"""Per-family GEMM launch times of a bench run from its rocprofv3 kernel trace, so the bench's
`roofline` / `roofline_gemm` figures can be recomputed from profiles/ alone.

    python tools/gemm_launches.py gpurun_out/prof_TAG/.../run_kernel_trace.csv [N] [out.json]

The folded first layer's forward (K = 128) and the five K = 512 layers' forward run different
instantiations (the latter with the pre-split weights). N = nodes per batch (default cfg2: 80,656).
"""
import csv
import json
import statistics
import sys

H, K_IN = 512, 128
PEAK = 2500.0 / 3   # f16x3 f32-equivalent ceiling, TF

# (round 5: the names carry the variant parameter; the K = 512 forward and dgrad run the
# pre-split-weight instantiation, PPV 4, the folded layer's the plain one)
FAMS = {
    "gemm_fwd": ["k_gemm_x6<1, 0, 1, 256, 256, 4, 2, 0, 4>"],
    "gemm_fwd_fold": ["k_gemm_x6<1, 0, 1, 256, 256, 4, 2, 0, 0>"],
    # (round 6: the K = 512 input gradients run the pipelined kernel, gemm_h3p.hip)
    "gemm_dgrad": ["k_gemm_h3p<128, 256, 2, 4, 4, 8", "k_gemm_h3p<128, 256, 2, 4, 4, 0",
                   "k_gemm_x6<1, 0, 1, 128, 256, 2, 4, 8, 4>", "k_gemm_x6<1, 0, 1, 128, 256, 2, 4, 0, 4>"],
    "gemm_wgrad": ["k_gemm_x6<1, 1, 0, 256, 256, 4, 2, 0, 0>"],
    "gemm_dgrad_fold": ["k_gemm_x6<1, 0, 1, 256, 128, 4, 2, 0, 0>"],
    "gemm_wgrad_fold": ["k_gemm_x6<1, 1, 0, 256, 128, 4, 2, 0, 0>"],
}


def main():
    path = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 80656
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Dispatch_Id"]))
    dur = {k: [] for k in FAMS}
    for r in rows:
        name = r["Kernel_Name"]
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3   # us
        for fam, pats in FAMS.items():
            if any(p in name for p in pats):
                dur[fam].append(d)
                break
    flop = {"gemm_fwd": 2.0 * n * 2 * H * H, "gemm_dgrad": 2.0 * n * H * 2 * H, "gemm_wgrad": 2.0 * 2 * H * H * n,
            "gemm_fwd_fold": 2.0 * n * 2 * H * K_IN, "gemm_dgrad_fold": 2.0 * n * K_IN * 2 * H,
            "gemm_wgrad_fold": 2.0 * 2 * H * K_IN * n}
    out = {"source": path, "nodes": n, "peak_tfs": PEAK, "families": {}}
    for fam, ds in dur.items():
        if not ds:
            continue
        avg = statistics.fmean(ds)
        tf = flop[fam] / (avg * 1e-6) / 1e12
        out["families"][fam] = {"launches": len(ds), "avg_us": round(avg, 2), "median_us": round(statistics.median(ds), 2),
                                "achieved_tfs": round(tf, 1), "frac": round(tf / PEAK, 4)}
    if dur["gemm_fwd"] and dur["gemm_fwd_fold"]:
        out["fold_split_check"] = {"max_fold_us": round(max(dur["gemm_fwd_fold"]), 1),
                                   "min_k512_us": round(min(dur["gemm_fwd"]), 1),
                                   "ok": max(dur["gemm_fwd_fold"]) < 0.7 * min(dur["gemm_fwd"])}
    txt = json.dumps(out, indent=1)
    print(txt)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(txt + "\n")


if __name__ == "__main__":
    main()
