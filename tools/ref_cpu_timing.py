#!/usr/bin/env python
"""Time the REFERENCE's own training step on the CPU ("in this container").

The reference model class (Models/BuckGNN.py) is imported unchanged; its third-party PyG /
torch_scatter ops are supplied by the oracle's CPU restatement (oracle/shim.py), because PyG is
not installed -- the same mechanism tests/golden/make_golden.py uses. One step
follows TRAIN_FINAL.py:253-298: forward in train mode (BatchNorm batch statistics, dropout 0.1),
RelativeErrorLoss (Utils/Losses.py:755-761), backward, Adam step (lr 1e-3, weight decay 1e-8).
Inputs are the bench's synthetic meshes (bgnn.synthetic). Runs only here, where
/root/reference exists; nothing from the reference is written into the repository.

    python tools/ref_cpu_timing.py [--threads 8] [--warmup 3] [--steps 10] [--out FILE]
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "buck-gnn_amd"))

from bgnn import synthetic  # noqa: E402


def load_reference_model():
    from oracle import shim
    shim.install()
    sys.path.insert(0, REF)
    try:
        from Models.BuckGNN import BuckGNN  # the reference's model class, unchanged
    finally:
        sys.path.remove(REF)
    return BuckGNN


def time_config(BuckGNN, name, model_name, warmup, steps, graphs=None):
    c = dict(synthetic.CONFIGS[name])
    if graphs is not None:
        c["graphs"] = graphs
    b = synthetic.make_batch(c["n"], c["graphs"], c["super_node"])
    torch.manual_seed(0)
    model = BuckGNN(num_node_features=16, num_edge_features=5, hidden_channels=512, num_layers=6,
                    pooling_layer="mean", prediction_type="buckling", dropout_rate=0.1,
                    model_name=model_name).train()
    opt = torch.optim.Adam(model.parameters(), lr=1e-3, weight_decay=1e-8)
    single = c["graphs"] == 1
    batch = None if single else b.batch
    y = b.y if not single else b.y[0]

    def step():
        opt.zero_grad(set_to_none=True)
        pred, _ = model(b.x, b.edge_index, b.edge_attr, batch)
        loss = torch.mean(torch.abs(pred - y) / (torch.abs(y) + 1e-8))
        loss.backward()
        opt.step()
        return float(loss)

    for _ in range(warmup):
        step()
    ts = []
    for _ in range(steps):
        t0 = time.perf_counter()
        step()
        ts.append(time.perf_counter() - t0)
    ms = 1e3 * sum(ts) / len(ts)
    return {"config": name, "model_name": model_name, "graphs": c["graphs"], "nodes": int(b.x.size(0)),
            "edges": int(b.edge_index.size(1)), "ms_per_step": round(ms, 1),
            "ms_min": round(1e3 * min(ts), 1), "ms_max": round(1e3 * max(ts), 1),
            "graphs_per_s": round(c["graphs"] / (ms / 1e3), 3), "warmup": warmup, "steps": steps}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--configs", default="cfg1,cfg2,cfg3")
    ap.add_argument("--ea-graphs", type=int, default=4,
                    help="graphs of the EA_GNN (cfg5 model) sample; 64 does not fit this host's memory")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r03_ref_cpu_timing.json"))
    args = ap.parse_args()
    if not os.path.isdir(os.path.join(REF, "Models")):
        print("reference not present; nothing to do")
        return 0
    torch.set_num_threads(args.threads)
    BuckGNN = load_reference_model()
    rows = []
    for name in filter(None, args.configs.split(",")):
        if name == "cfg5":
            r = time_config(BuckGNN, "cfg5", "EA_GNN", 1, 2, graphs=args.ea_graphs)
            r["sample"] = f"{args.ea_graphs} of cfg5's 64 graphs per step, fp32 (the bf16 GPU config has no CPU analogue)"
        else:
            r = time_config(BuckGNN, name, "GraphSage_addAggr", args.warmup, args.steps)
        print(json.dumps(r), flush=True)
        rows.append(r)
    out = {"what": "reference Models/BuckGNN.py train step (fwd+loss+bwd+Adam) on the CPU, PyG ops from the "
                   "oracle's restatement", "threads": torch.get_num_threads(), "cpu_count": os.cpu_count(),
           "cpu": platform.processor() or platform.machine(), "torch": torch.__version__, "rows": rows}
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    print("->", args.out)
    return 0


if __name__ == "__main__":
    sys.exit(main())
