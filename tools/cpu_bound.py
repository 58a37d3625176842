#!/usr/bin/env python
"""Is the training step CPU-launch-bound? Runs bench.py's store data path and reports, for K
steps, the host time to ENQUEUE them (Python + launches, measured before the final
synchronize) against the wall time until the GPU finishes, plus the host time of the batch
gather alone. Enqueue time close to the wall time means the GPU waits for the host.

    python tools/cpu_bound.py [--steps 20]
"""
import argparse
import itertools
import os
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
    rng = np.random.default_rng(0)
    order = itertools.cycle(rng.permutation(64))

    def step(t_batch):
        t = time.perf_counter()
        b = store.batch([next(order) for _ in range(16)])
        t_batch.append(time.perf_counter() - t)
        return bgnn.train_step(model, b, opt, crit, norm)
    tb = []
    for _ in range(5):
        step(tb)
    torch.cuda.synchronize()
    tb.clear()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(tb)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    n = args.steps
    print(f"per step: host enqueue {(t1 - t0) / n * 1e3:.2f} ms (batch gather {sum(tb) / n * 1e3:.2f} ms), "
          f"wall {(t2 - t0) / n * 1e3:.2f} ms", flush=True)


if __name__ == "__main__":
    main()
