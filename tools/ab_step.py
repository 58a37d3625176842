#!/usr/bin/env python
"""Same-process A/B of whole training steps (cfg2): alternates settings for R rounds of S
steps and reports the median ms/step per setting. Settings are module attributes or C tuning knobs ("knob:5=1"):
    python tools/ab_step.py "bgnn.buckgnn.FUSED_ENCODER=True" "bgnn.buckgnn.FUSED_ENCODER=False"
"""
import importlib
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "buck-gnn_amd"))
import torch  # noqa: E402

import bgnn  # noqa: E402
from bgnn import synthetic  # noqa: E402


def apply(setting):
    """'mod.attr=expr' sets a module attribute; 'knob:K=V' calls bgnn_set_tuning(K, V)."""
    for kv in setting.split(";"):
        k, v = kv.split("=")
        if k.startswith("knob:"):
            bgnn._lib.call("bgnn_set_tuning", int(k[5:]), int(v))
            continue
        mod, attr = k.rsplit(".", 1)
        setattr(importlib.import_module(mod), attr, eval(v))


def main():
    settings = sys.argv[1:] or ["bgnn.fused.GEMM_BACKEND='hip'"]
    rounds, steps = int(os.environ.get("AB_ROUNDS", "5")), 8
    dev = torch.device("cuda", 0)
    batch = synthetic.make_config_batch(os.environ.get("AB_CONFIG", "cfg2")).to(dev)
    torch.manual_seed(0)
    model = bgnn.BuckGNN(16, 5, hidden_channels=512, num_layers=6, dropout_rate=0.1,
                         model_name=os.environ.get("AB_MODEL", "GraphSage_addAggr")).to(dev).train()
    opt = torch.optim.Adam(model.parameters(), lr=1e-2, weight_decay=1e-8, fused=True)
    crit, norm = bgnn.RelativeErrorLoss(), bgnn.EigenvalueScaler(1.0, 0.5)

    clear = os.environ.get("AB_CLEAR", "1") == "1"   # 0: keep the graph structure cached

    def step():
        if clear:
            bgnn.clear_caches()
        bgnn.train_step(model, batch, opt, crit, norm)

    res = {s: [] for s in settings}
    for s in settings:
        apply(s)
        for _ in range(3):
            step()
    for r in range(rounds):
        for s in (settings if r % 2 == 0 else settings[::-1]):   # (alternate the order: no position bias)
            apply(s)
            step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                step()
            torch.cuda.synchronize()
            res[s].append((time.perf_counter() - t0) / steps * 1e3)
    for s in settings:
        v = res[s]
        print(f"{statistics.median(v):8.3f} ms/step (min {min(v):.3f})  {s}")


if __name__ == "__main__":
    main()
