#!/usr/bin/env python
"""A/B the GEMM kernels and tile configurations (and torch.mm) on the SAGE layer shapes,
interleaved in one process; median per-launch HIP-event time, TFLOP/s, and the error
against an fp64 product as max_ij |c - c64|_ij / (|A| |B|)_ij.
Variants: "3" = f32 MFMA config 3, "h1" = f16x3 config 1 (bf16x6 "x" variants removed in ABI 9),
"torch" = torch.mm."""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "buck-gnn_amd"))
import torch  # noqa: E402

from bgnn import _lib, fused  # noqa: E402

SHAPES = {  # name: (M, N, K, trans_a, trans_b)
    "fwd": (80656, 1024, 512, False, True),
    "dgrad": (80656, 512, 1024, False, False),
    "wgrad": (1024, 512, 80656, True, False),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfgs", default="3,h0,h1,h2,h3,h4")
    ap.add_argument("--rounds", type=int, default=10)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    ops = {}
    for name, (M, N, K, ta, tb) in SHAPES.items():
        a = torch.randn((K, M) if ta else (M, K), device=dev)
        b = torch.randn((N, K) if tb else (K, N), device=dev)
        ops[name] = (a, b, ta, tb, 2.0 * M * N * K)
    exact = {}
    for name, (a, b, ta, tb, _) in ops.items():
        A = a.double().t() if ta else a.double()
        B = b.double().t() if tb else b.double()
        exact[name] = (A @ B, A.abs() @ B.abs())
    errs = {}
    variants = args.cfgs.split(",") + ["torch"]
    times = {(v, n): [] for v in variants for n in SHAPES}
    ref = {}
    for rnd in range(args.rounds + 1):
        for v in variants:
            for n, (a, b, ta, tb, fl) in ops.items():
                if v == "torch":
                    fused.GEMM_BACKEND = "torch"
                else:
                    fused.GEMM_BACKEND = "hip"
                    _lib.call("bgnn_set_tuning", 5, 2 if v[0] == "h" else 0)
                    _lib.call("bgnn_gemm_set_cfg", int(v.lstrip("xh")))
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                c = fused.gemm(a, b, ta, tb)
                e1.record()
                torch.cuda.synchronize()
                if rnd:
                    times[(v, n)].append(e0.elapsed_time(e1))
                else:
                    c64, mag = exact[n]
                    errs[(v, n)] = ((c.double() - c64).abs() / mag.clamp_min(1e-30)).max().item()
                    if n not in ref:
                        ref[n] = c
                    else:
                        err = (c - ref[n]).abs().max().item() / ref[n].abs().max().item()
                        if err > 1e-4:
                            print(f"MISMATCH cfg {v} {n}: rel {err:.2e}")
    _lib.call("bgnn_gemm_set_cfg", -1)
    _lib.call("bgnn_set_tuning", 5, 2)
    for v in variants:
        line = f"cfg {str(v):6s}"
        for n, (a, b, ta, tb, fl) in ops.items():
            t = statistics.median(times[(v, n)])
            line += f" | {n} {t*1e3:8.1f} us {fl/t/1e9:7.1f} TF err {errs[(v, n)]:.1e}"
        print(line)


if __name__ == "__main__":
    main()
