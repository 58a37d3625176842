#!/usr/bin/env python
"""Host-side (Python) profile of the bench's cfg2 training step: cProfile over K steps after a
warm-up, sorted by cumulative and by own time, plus the host enqueue time per step against the
wall time (is the GPU waiting for the host?).

    python tools/host_profile.py [--steps 20]
"""
import argparse
import cProfile
import io
import itertools
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "buck-gnn_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bgnn  # noqa: E402
from bgnn import synthetic  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    c = synthetic.CONFIGS["cfg2"]
    pool = [synthetic.make_mesh_graph(c["n"], g, super_node=c["super_node"]) for g in range(64)]
    store = bgnn.GraphStore(pool, dev)
    torch.manual_seed(0)
    model = bgnn.BuckGNN(16, 5, hidden_channels=512, num_layers=6, dropout_rate=0.1,
                         model_name="GraphSage_addAggr").to(dev).train()
    opt = torch.optim.Adam(model.parameters(), lr=1e-2, weight_decay=1e-8, fused=True)
    crit, norm = bgnn.RelativeErrorLoss(), bgnn.EigenvalueScaler(1.0, 0.5)
    order = itertools.cycle(np.random.default_rng(0).permutation(64))

    def step():
        b = store.batch([next(order) for _ in range(16)])
        return bgnn.train_step(model, b, opt, crit, norm)

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    for _ in range(args.steps):
        step()
    pr.disable()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    n = args.steps
    print(f"per step (under cProfile): host {(t1 - t0) / n * 1e3:.2f} ms, wall {(t2 - t0) / n * 1e3:.2f} ms")
    for key in ("cumulative", "tottime"):
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats(key).print_stats(45)
        print(s.getvalue())


if __name__ == "__main__":
    main()
