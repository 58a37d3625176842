#!/usr/bin/env python
"""Count the small torch fill / copy calls of one cfg2 train step by call site (which torch.zeros,
zero_, fill_, clone, .to() run per step on the fused path)."""
import collections
import itertools
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "buck-gnn_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bgnn  # noqa: E402
from bgnn import synthetic  # noqa: E402

counts = collections.Counter()
active = [False]


def wrap(obj, name):
    orig = getattr(obj, name)

    def f(*a, **k):
        if active[0]:
            st = traceback.extract_stack(limit=4)[-2]
            counts[(name, os.path.basename(st.filename), st.lineno)] += 1
        return orig(*a, **k)
    setattr(obj, name, f)


for n in ("zeros", "zeros_like", "ones", "full", "tensor", "cat", "stack"):
    wrap(torch, n)
for n in ("zero_", "fill_", "clone", "copy_", "to", "contiguous"):
    wrap(torch.Tensor, n)

dev = torch.device("cuda", 0)
c = synthetic.CONFIGS["cfg2"]
pool = [synthetic.make_mesh_graph(c["n"], g) for g in range(32)]
store = bgnn.GraphStore(pool, dev)
torch.manual_seed(0)
model = bgnn.BuckGNN(synthetic.NUM_NODE_FEATURES, synthetic.NUM_EDGE_FEATURES, hidden_channels=512, num_layers=6,
                     pooling_layer="mean", prediction_type="buckling", dropout_rate=0.1,
                     model_name="GraphSage_addAggr").to(dev).train()
opt = torch.optim.Adam(model.parameters(), lr=1e-2, weight_decay=1e-8, fused=True)
crit, norm = bgnn.RelativeErrorLoss(), bgnn.EigenvalueScaler(center=1.0, scale=0.5)
rng = np.random.default_rng(0)
for step in range(3):
    active[0] = step == 2
    ids = rng.permutation(32)[:16].tolist()
    bgnn.train_step(model, store.batch(ids), opt, crit, norm)
torch.cuda.synchronize()
for (n, f, l), v in counts.most_common(40):
    print(f"{v:4d}  {n:12s} {f}:{l}")
