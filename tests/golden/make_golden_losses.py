#!/usr/bin/env python
"""Generate tests/golden/heads/losses.npz from the REFERENCE's own per-graph losses and metrics
(Utils/Losses.py GraphRelativeError, GraphMixedError, GraphMSELoss, GraphMAELoss,
GraphMaxComponentRelativeError; Dataset_Preparation/Metrics.py MAPE_error, stress_errors).

Runs only in the build container, where /root/reference exists; the reference modules are
imported unchanged (torch_scatter, which Losses.py imports, comes from the oracle's CPU
restatement, oracle/shim.py). The fixture holds only data: the seeded inputs and the
reference's outputs.

    python tests/golden/make_golden_losses.py [--out tests/golden/heads/losses.npz]
"""
from __future__ import annotations

import argparse
import importlib.util
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, ROOT)


def load(path, name):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def inputs(seed, sizes, C):
    """Ragged batch: graph g has sizes[g] rows; targets spread over decades (some below the
    0.1 threshold), one exact tie of the largest |target| per graph (first index wins)."""
    g = torch.Generator().manual_seed(seed)
    batch = torch.cat([torch.full((n,), i, dtype=torch.long) for i, n in enumerate(sizes)])
    N = batch.numel()
    t = torch.randn(N, C, generator=g) * torch.pow(10.0, torch.rand(N, 1, generator=g) * 2 - 1.5)
    p = t + 0.05 * torch.randn(N, C, generator=g)
    off = 0
    for n in sizes:
        t[off + n - 1, 0] = t[off:off + n, 0].abs().max()   # tie with an earlier maximum
        off += n
    return p, t, batch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(HERE, "heads", "losses.npz"))
    args = ap.parse_args()
    from oracle import shim
    shim.install()
    L = load(os.path.join(REF, "Utils", "Losses.py"), "ref_losses")
    M = load(os.path.join(REF, "Dataset_Preparation", "Metrics.py"), "ref_metrics")
    shim.uninstall()
    out = {}
    for tag, (seed, sizes, C) in {"s3": (1, [37, 5, 64, 18], 3), "d3": (2, [23, 41, 9], 3),
                                  "v1": (3, [30, 12, 25], 1)}.items():
        p, t, b = inputs(seed, sizes, C)
        if C == 1:
            p, t = p[:, 0], t[:, 0]
        out[f"{tag}_pred"], out[f"{tag}_target"], out[f"{tag}_batch"] = p.numpy(), t.numpy(), b.numpy()
        for name, mod in (("rel", L.GraphRelativeError()), ("mixed", L.GraphMixedError()), ("mse", L.GraphMSELoss()),
                          ("mae", L.GraphMAELoss()), ("maxc", L.GraphMaxComponentRelativeError())):
            out[f"{tag}_{name}"] = np.float64(mod(p, t, b, None).item())
            out[f"{tag}_{name}_nobatch"] = np.float64(mod(p, t, None, None).item())
        if C == 3:
            for kind in ("static_stress", "static_disp"):
                d = M.stress_errors(p, t, b, prediction_type=kind)
                out[f"{tag}_{kind}_keys"] = np.array(sorted(d))
                out[f"{tag}_{kind}_vals"] = np.array([d[k] for k in sorted(d)], dtype=np.float64)
                out[f"{tag}_mape_{kind}"] = np.float64(M.MAPE_error(p, t, kind).item())
            out[f"{tag}_mape_mode_shape"] = np.float64(M.MAPE_error(p, t, "mode_shape").item())
    np.savez(args.out, **out)
    print("wrote", args.out, len(out), "arrays")


if __name__ == "__main__":
    main()
