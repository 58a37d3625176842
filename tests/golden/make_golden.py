#!/usr/bin/env python
"""Generate tests/golden/*.npz from the REFERENCE's own Models/BuckGNN.py.

Runs only in the build container, where /root/reference exists. The reference
model class is imported unchanged; the third-party ops it imports
(torch_geometric.nn.SAGEConv, global_mean_pool, torch_scatter.scatter_mean, ...)
are supplied by the oracle's CPU restatement (oracle/shim.py), because PyG is not
installed. Nothing from /root/reference is written into the
repository: each fixture holds only data — inputs, the weight-recipe seed, and the
reference's outputs (prediction, loss, gradients or gradient checksums, BatchNorm
running statistics, pooled features, eval-mode prediction).

    python tests/golden/make_golden.py [--out tests/golden]
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "buck-gnn_amd"))
sys.path.insert(0, HERE)

from recipe import grad_checksum, make_weights, meta_to_array  # noqa: E402

CASES = [
    # name, model_name, hidden, pooling, graphs [(n, super_node, seed)], full_grads
    ("add_h64", "GraphSage_addAggr", 64, "mean", [(5, False, 1), (6, False, 2), (4, False, 3)], True),
    ("sum_h64", "GraphSage_sumAggr", 64, "mean", [(5, False, 1), (6, False, 2), (4, False, 3)], True),
    ("mean_h64", "GraphSage_meanAggr", 64, "mean", [(5, False, 1), (6, False, 2), (4, False, 3)], True),
    ("max_h64", "GraphSage_maxAggr", 64, "mean", [(5, False, 1), (6, False, 2), (4, False, 3)], True),
    ("shared_h64", "GraphSage_addAggr_Shared", 64, "mean", [(5, False, 1), (6, False, 2), (4, False, 3)], True),
    ("add_super_h64", "GraphSage_addAggr", 64, "mean", [(5, True, 4), (7, True, 5)], True),
    ("add_super_nosuper_h64", "GraphSage_addAggr", 64, "mean_no_super", [(5, True, 4), (7, True, 5)], True),
    ("add_super_only_h64", "GraphSage_addAggr", 64, "supernode_only", [(5, True, 4), (7, True, 5)], True),
    ("add_super_withpool_h64", "GraphSage_addAggr", 64, "supernode_with_pooling", [(5, True, 4), (7, True, 5)],
     True),
    ("add_single_h64", "GraphSage_addAggr", 64, "mean", [(6, False, 7)], True),
    ("add_super_h512", "GraphSage_addAggr", 512, "mean", [(5, True, 8), (4, True, 9)], False),
    ("mean_h512", "GraphSage_meanAggr", 512, "mean", [(5, False, 10), (4, False, 11)], False),
    ("shared_h512", "GraphSage_addAggr_Shared", 512, "mean", [(6, False, 12)], False),
    ("add_h256", "GraphSage_addAggr", 256, "mean", [(5, False, 13), (5, True, 14)], False),
    ("ea_gnn_h64", "EA_GNN", 64, "mean", [(4, False, 15), (5, False, 16)], False),
    # round 4: EA_GNN_Shared (Models/BuckGNN.py:103-104,326-336; a TRAIN_FINAL.py:66,81 choice) and
    # max aggregation at the production size (aggregate-first hand-written path, super-node
    # heavy rows of the max kernel)
    ("ea_gnn_shared_h64", "EA_GNN_Shared", 64, "mean", [(4, False, 40), (5, False, 41)], True),
    ("max_h512_n1k", "GraphSage_maxAggr", 512, "mean", [(23, False, 42), (23, True, 43)], False),
    # SAGPooling variants (Models/BuckGNN.py:190-244,354-373,493-511)
    ("sag_h64", "GraphSAGE_SAG", 64, "mean", [(5, False, 17), (6, False, 18), (4, False, 19)], True),
    ("sag_super_h64", "GraphSAGE_SAG", 64, "mean", [(5, True, 20), (4, True, 21)], True),
    ("sag_single_h64", "GraphSAGE_SAG", 64, "mean", [(6, False, 22)], True),
    ("eagnn_sag_h64", "EAGNN_SAG", 64, "mean", [(4, False, 23), (5, False, 24)], False),
    # the production path (round 3): >= 1,024 nodes, where the fused model folds the node
    # encoder's last Linear into the first SAGE layer and runs the encoder head as bgnn_mlp2
    # (Models/BuckGNN.py:67-74,323,430-444); 23x23 + 22x22 meshes with virtual edges and an
    # 8x8 mesh with a super node: 1,078 nodes
    ("add_h512_n1k", "GraphSage_addAggr", 512, "mean", [(23, False, 30), (22, False, 31), (8, True, 32)], False),
    ("shared_h512_n1k", "GraphSage_addAggr_Shared", 512, "mean", [(23, False, 30), (22, False, 31), (8, True, 32)],
     False),
    ("mean_h512_n1k", "GraphSage_meanAggr", 512, "mean", [(23, False, 33), (23, True, 34)], False),
    ("sag_h512_n1k", "GraphSAGE_SAG", 512, "mean", [(23, False, 35), (23, False, 36)], False),
    # round 6: BASELINE configs[0] itself -- one 45x45 mesh (2,025 nodes, virtual edges), batch=None
    # (INFERENCE.py:261 at BATCH_SIZE = 1; global_mean_pool with batch=None, Models/BuckGNN.py:273-274),
    # h = 512, the add loop and TRAIN_FINAL.py's default Shared loop
    ("add_cfg1_h512", "GraphSage_addAggr", 512, "mean", [(45, False, 50)], False),
    ("shared_cfg1_h512", "GraphSage_addAggr_Shared", 512, "mean", [(45, False, 51)], False),
]


def build_inputs(graphs):
    from bgnn.synthetic import make_mesh_graph
    from oracle.pyg_ref import collate

    ds = []
    for n, sup, seed in graphs:
        d = make_mesh_graph(n, seed, super_node=sup)
        ds.append({"x": d.x.numpy(), "edge_index": d.edge_index.numpy(), "edge_attr": d.edge_attr.numpy(),
                   "y": d.y.numpy()})
    return collate(ds)


def run_case(BuckGNN, case):
    name, model_name, h, pooling, graphs, full = case
    torch.manual_seed(0)
    model = BuckGNN(num_node_features=16, num_edge_features=5, hidden_channels=h, num_layers=6,
                    pooling_layer=pooling, prediction_type="buckling", dropout_rate=0.0, model_name=model_name)
    sd = model.state_dict()
    shapes = {k: tuple(v.shape) for k, v in sd.items()}
    seed = 1000 + h
    w = make_weights(shapes, seed)
    model.load_state_dict({k: torch.from_numpy(w[k]) if k in w else sd[k] for k in sd})
    b = build_inputs(graphs)
    single = len(graphs) == 1
    batch = None if single else b["batch"]
    captured = {}
    model.decoder.register_forward_pre_hook(lambda m, inp: captured.__setitem__("pooled", inp[0].detach().clone()))
    if hasattr(model, "pool"):   # SAGPooling outputs: perm, score[perm], pooled edge count
        model.pool.register_forward_hook(lambda m, inp, o: captured.update(
            perm=o[4].clone(), score=o[5].detach().clone(), n_edges=o[1].size(1)))
    model.train()
    pred, _ = model(b["x"], b["edge_index"], b["edge_attr"], batch)
    y = b["y"] if not single else b["y"][0]
    loss = torch.mean(torch.abs(pred - y) / (torch.abs(y) + 1e-8))   # RelativeErrorLoss, Losses.py:755-761
    model.zero_grad(set_to_none=True)
    loss.backward()
    out = {
        "meta": meta_to_array({"name": name, "model_name": model_name, "hidden": h, "pooling": pooling,
                               "weight_seed": seed, "num_layers": 6, "single_graph": single,
                               "graphs": graphs}),
        "x": b["x"].numpy(), "edge_index": b["edge_index"].numpy(), "edge_attr": b["edge_attr"].numpy(),
        "batch": b["batch"].numpy(), "y": b["y"].numpy(),
        "pred_train": pred.detach().numpy().reshape(-1), "loss_train": np.array(loss.item()),
        "pooled_train": captured["pooled"].numpy(),
    }
    if "perm" in captured:
        out.update(pool_perm=captured["perm"].numpy(), pool_score=captured["score"].numpy(),
                   pool_edges=np.array(captured["n_edges"]))
    for k, p in model.named_parameters():
        if p.grad is None:
            continue
        g = p.grad.numpy()
        if full:
            out["grad/" + k] = g
        else:
            out["gradsum/" + k] = grad_checksum(g)
    for k, v in model.state_dict().items():
        if "running_" in k:
            out["state/" + k] = v.numpy()
    model.eval()
    with torch.no_grad():
        pe, _ = model(b["x"], b["edge_index"], b["edge_attr"], batch)
    out["pred_eval"] = pe.numpy().reshape(-1)
    out["pooled_eval"] = captured["pooled"].numpy()
    return name, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=HERE)
    ap.add_argument("--only", default="", help="comma-separated case names (default: all)")
    args = ap.parse_args()
    only = set(filter(None, args.only.split(",")))
    if not os.path.isdir(os.path.join(REF, "Models")):
        print("reference not present; nothing to do")
        return 0
    from oracle import shim
    shim.install()
    sys.path.insert(0, REF)
    try:
        from Models.BuckGNN import BuckGNN  # the reference's model class, unchanged
    finally:
        sys.path.remove(REF)
    total = 0
    for case in CASES:
        if only and case[0] not in only:
            continue
        name, out = run_case(BuckGNN, case)
        path = os.path.join(args.out, f"{name}.npz")
        np.savez_compressed(path, **out)
        total += os.path.getsize(path)
        print(f"{name}: pred={out['pred_train']} loss={float(out['loss_train']):.6f} -> {path}")
    print(f"total fixture bytes: {total}")
    shim.uninstall()
    return 0


if __name__ == "__main__":
    sys.exit(main())
