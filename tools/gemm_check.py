#!/usr/bin/env python
"""Per-element error class of bgnn GEMMs against fp64 on given shapes, with the split-K factor
the plan picks (from the workspace size). Usage: python tools/gemm_check.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "buck-gnn_amd"))
import torch  # noqa: E402

from bgnn import _lib, fused  # noqa: E402

SHAPES = [(1024, 128, 512, 0, 0), (1024, 1, 512, 0, 0), (512, 128, 1024, 1, 0), (512, 1, 1024, 1, 0),
          (1024, 512, 128, 0, 1), (300, 200, 64, 0, 0), (1024, 128, 2048, 0, 0)]


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    for (M, N, K, ta, tb) in SHAPES:
        a = torch.randn((K, M) if ta else (M, K), device=dev) * 0.05
        b = torch.randn((N, K) if tb else (K, N), device=dev) * 0.05
        c = fused.gemm(a, b, bool(ta), bool(tb))
        A = a.double().t() if ta else a.double()
        B = b.double().t() if tb else b.double()
        r, mag = A @ B, A.abs() @ B.abs()
        err = ((c.double() - r).abs() / mag).max().item()
        ws = _lib.query("bgnn_gemm_ws_bytes_ex", M, N, K, ta, tb, 0)
        split = max(1, (ws - 256) // (M * N * 4)) if ws > 256 else 1
        print(f"{M}x{N}x{K} ta={ta} tb={tb}: split {split}, max err/(|A||B|) {err:.2e}", flush=True)


if __name__ == "__main__":
    main()
