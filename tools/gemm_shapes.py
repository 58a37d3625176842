#!/usr/bin/env python
"""Per-shape GEMM timing of the step's small / skinny GEMMs under each tile config (medians of
HIP-event times, 20 launches each): which plan the shape gets by default (cfg -1) and what the
others would do. Usage: python tools/gemm_shapes.py"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "buck-gnn_amd"))
import torch  # noqa: E402

from bgnn import _lib, fused  # noqa: E402

SHAPES = [  # (M, N, K, ta, tb, what)
    (80656, 128, 64, 0, 1, "encoder L2 fwd"),
    (80656, 64, 128, 0, 1, "encoder L2 dgrad"),
    (80656, 1024, 128, 0, 1, "folded layer fwd"),
    (80656, 128, 1024, 0, 1, "folded layer dgrad"),
    (1024, 128, 80656, 1, 0, "folded layer wgrad"),
    (128, 64, 80656, 1, 0, "encoder L2 wgrad"),
    (80656, 64, 16, 0, 1, "encoder L1 fwd"),
]


def main():
    dev = torch.device("cuda", 0)
    for M, N, K, ta, tb, what in SHAPES:
        a = torch.randn((K, M) if ta else (M, K), device=dev)
        b = torch.randn((N, K) if tb else (K, N), device=dev)
        res = []
        for cfg in (-1, 0, 1, 2, 4):
            _lib.call("bgnn_gemm_set_cfg", cfg)
            try:
                ts = []
                for i in range(22):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    fused.gemm(a, b, bool(ta), bool(tb))
                    e1.record()
                    torch.cuda.synchronize()
                    if i >= 2:
                        ts.append(e0.elapsed_time(e1) * 1e3)
                res.append(f"cfg{cfg}:{statistics.median(ts):7.1f}")
            except Exception as ex:   # a config the shape cannot take
                res.append(f"cfg{cfg}: n/a ({str(ex)[:30]})")
        _lib.call("bgnn_gemm_set_cfg", -1)
        print(f"{what:20s} {M}x{N}x{K} " + "  ".join(res), flush=True)


if __name__ == "__main__":
    main()
