#!/usr/bin/env python
"""Host issue time against GPU time of the bench's cfg2 training step (GraphStore batches, as
bench.py runs them): per step, the host time of step() (no synchronisation inside) and the GPU
time between HIP events at step boundaries. A host time close to the GPU time means the step is
host-bound at its start (the GPU idles while Python issues the next step's first kernels).
    python tools/host_lag.py [steps]"""
import os
import sys
import time

import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "buck-gnn_amd"))
import torch  # noqa: E402
import bgnn  # noqa: E402
from bgnn import synthetic  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    dev = torch.device("cuda", 0)
    c = synthetic.CONFIGS["cfg2"]
    pool = [synthetic.make_mesh_graph(c["n"], g) for g in range(64)]
    store = bgnn.GraphStore(pool, dev)
    torch.manual_seed(0)
    model = bgnn.BuckGNN(16, 5, hidden_channels=512, num_layers=6, dropout_rate=0.1,
                         model_name="GraphSage_addAggr").to(dev).train()
    opt = torch.optim.Adam(model.parameters(), lr=1e-2, weight_decay=1e-8, fused=True)
    crit, norm = bgnn.RelativeErrorLoss(), bgnn.EigenvalueScaler(1.0, 0.5)
    rng = np.random.default_rng(0)

    def step():
        ids = rng.permutation(len(pool))[:16]
        return bgnn.train_step(model, store.batch(ids), opt, crit, norm)

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    host = []
    evs[0].record()
    t0 = time.perf_counter()
    for i in range(steps):
        h0 = time.perf_counter()
        step()
        host.append(time.perf_counter() - h0)
        evs[i + 1].record()
    t_issue = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    gpu = [evs[i].elapsed_time(evs[i + 1]) for i in range(steps)]
    print(f"steps {steps}: host issue {t_issue * 1e3 / steps:.3f} ms/step, wall {t_all * 1e3 / steps:.3f} ms/step, "
          f"GPU {sum(gpu) / steps:.3f} ms/step")
    print("host ms per step:", " ".join(f"{h * 1e3:.2f}" for h in host))
    print("gpu  ms per step:", " ".join(f"{g:.2f}" for g in gpu))
    # where the host time goes in one step (no sync): batch assembly vs train_step
    h0 = time.perf_counter()
    b = store.batch(rng.permutation(len(pool))[:16])
    h1 = time.perf_counter()
    bgnn.train_step(model, b, opt, crit, norm)
    h2 = time.perf_counter()
    print(f"store.batch {1e3 * (h1 - h0):.3f} ms, train_step {1e3 * (h2 - h1):.3f} ms (host)")


if __name__ == "__main__":
    main()
