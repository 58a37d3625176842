#!/usr/bin/env python
"""Attribute a training step's small kernels to their Python call sites: torch.profiler over a
few cfg2 steps (bench.py's model and data path), events grouped by the innermost bgnn/ call
stack frames; prints kernels per step with their GPU time.

    python tools/step_profile.py [--steps 3] [--top 60]
"""
import argparse
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "buck-gnn_amd"))
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

import bgnn  # noqa: E402
from bgnn import synthetic  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--top", type=int, default=60)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    batch = synthetic.make_config_batch("cfg2").to(dev)
    torch.manual_seed(0)
    model = bgnn.BuckGNN(16, 5, hidden_channels=512, num_layers=6, dropout_rate=0.1,
                         model_name="GraphSage_addAggr").to(dev).train()
    opt = torch.optim.Adam(model.parameters(), lr=1e-2, weight_decay=1e-8, fused=True)
    crit, norm = bgnn.RelativeErrorLoss(), bgnn.EigenvalueScaler(1.0, 0.5)
    for _ in range(3):
        bgnn.train_step(model, batch, opt, crit, norm)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        for _ in range(args.steps):
            bgnn.train_step(model, batch, opt, crit, norm)
        torch.cuda.synchronize()
    # each CPU op's innermost bgnn frames; kernels launched under it inherit them
    agg = defaultdict(lambda: [0, 0.0])
    for e in prof.events():
        if e.device_type != torch.autograd.DeviceType.CPU or not e.kernels:
            continue
        frames = [f for f in (e.stack or []) if "bgnn" in f or "bench" in f]
        site = " <- ".join(f.split("/")[-1] for f in frames[:3]) or "(no bgnn frame)"
        for k in e.kernels:
            key = (k.name[:70], e.name[:40], site[:150])
            agg[key][0] += 1
            agg[key][1] += k.duration
    rows = sorted(agg.items(), key=lambda kv: -kv[1][1])
    print(f"{'n/step':>6s} {'us/step':>8s}  kernel | op | site")
    for (kn, op, site), (n, us) in rows[:args.top]:
        print(f"{n / args.steps:6.1f} {us / args.steps:8.1f}  {kn} | {op} | {site}")


if __name__ == "__main__":
    main()
