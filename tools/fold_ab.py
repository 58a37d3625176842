#!/usr/bin/env python
"""Folded-encoder gradient accuracy against fp64 (tests/test_gpu_fold.py's measure), per
parameter, for the fused path with the weight-by-weight products on torch.mm or on bgnn_gemm,
beside the unfolded path with f16x3 and with bf16x6 GEMMs (the spread of f32 rounding noise).

    python tools/fold_ab.py [model_name]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "buck-gnn_amd"), ROOT, os.path.join(ROOT, "tests")]
import torch  # noqa: E402

from bgnn import fused  # noqa: E402
import test_gpu_fold as T  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "GraphSage_meanAggr"
    dev = torch.device("cuda", 0)
    _, _, _, g_ref = T.run(dev, name, 512, False)
    res = {}
    for flag in (True, False):
        fused.FOLD_WEIGHTS_TORCH = flag
        b, sd, _, g = T.run(dev, name, 512, True)
        res[flag] = g
    # the unfolded path once more with the bf16x6 split GEMMs (same f32 error class, other rounding)
    from bgnn import _lib
    _lib.call("bgnn_set_tuning", 5, 1)
    _, _, _, g_x6 = T.run(dev, name, 512, False)
    _lib.call("bgnn_set_tuning", 5, 2)
    exact = T.oracle_grads(b, sd, name)
    print(f"{'param':45s} {'unfolded':>10s} {'unf/bf16x6':>10s} {'fold/torch':>10s} {'fold/bgnn':>10s}")
    for k in sorted(exact):
        print(f"{k:45s} {T.rel_err(g_ref[k], exact[k]):10.2e} {T.rel_err(g_x6[k], exact[k]):10.2e} "
              f"{T.rel_err(res[True][k], exact[k]):10.2e} {T.rel_err(res[False][k], exact[k]):10.2e}")


if __name__ == "__main__":
    main()
