#!/usr/bin/env python
"""EA_GNN training trajectories on one cfg2 batch (16 meshes, h = 512, dropout 0): per-step
RelativeErrorLoss of the fused bgnn path (f32-accurate and bf16 GEMM operands) next to the
oracle's functional EA_GNN run in fp32 and under torch.autocast(bfloat16) (PyTorch's own bf16).
Diagnostic for ADVICE r01 (EA bench losses): is a divergence the model's or the kernels'?

    python tools/ea_trajectory.py [--lr 1e-3] [--steps 20]
"""
import argparse
import contextlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "buck-gnn_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bgnn  # noqa: E402
from bgnn import synthetic as S  # noqa: E402
from oracle import buckgnn_ref as R  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--config", default="cfg2")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    b = S.make_config_batch(args.config).to(dev)
    norm = bgnn.EigenvalueScaler(1.0, 0.5)
    torch.manual_seed(0)
    m0 = bgnn.BuckGNN(16, 5, hidden_channels=512, num_layers=6, dropout_rate=0.0, model_name="EA_GNN")
    sd0 = {k: v.detach().clone() for k, v in m0.state_dict().items()}
    runs = {}
    for bf16 in (False, True):
        m = bgnn.BuckGNN(16, 5, hidden_channels=512, num_layers=6, dropout_rate=0.0, model_name="EA_GNN")
        m.load_state_dict(sd0)
        m = m.to(dev).train()
        m.ea_bf16 = bf16
        opt = torch.optim.Adam(m.parameters(), lr=args.lr, weight_decay=1e-8)
        runs["fused_bf16" if bf16 else "fused_f32"] = [
            float(bgnn.train_step(m, b, opt, bgnn.RelativeErrorLoss(), norm)) for _ in range(args.steps)]
    for bf16 in (False, True):
        sd = {k: v.to(dev).clone() for k, v in sd0.items()}
        params = [v.requires_grad_(True) for k, v in sd.items() if v.is_floating_point() and "running" not in k]
        opt = torch.optim.Adam(params, lr=args.lr, weight_decay=1e-8)
        losses = []
        for _ in range(args.steps):
            ctx = torch.autocast("cuda", dtype=torch.bfloat16) if bf16 else contextlib.nullcontext()
            with ctx:
                pred = R.ea_forward(sd, b.x, b.edge_index, b.edge_attr, b.batch, True, 0.0)
            loss = R.relative_error_loss(norm.denormalize_eigenvalue(pred.float()), norm.denormalize_eigenvalue(b.y))
            opt.zero_grad(set_to_none=True)
            loss.backward()
            opt.step()
            losses.append(float(loss))
        runs["torch_autocast_bf16" if bf16 else "torch_f32"] = losses
    names = list(runs)
    print("step " + " ".join(f"{n:>20s}" for n in names))
    for s in range(args.steps):
        print(f"{s:4d} " + " ".join(f"{runs[n][s]:20.5g}" for n in names))


if __name__ == "__main__":
    main()
