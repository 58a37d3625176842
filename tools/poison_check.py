#!/usr/bin/env python
"""Uninitialised-memory check: run a model's forward + backward, then fill the caching
allocator's free blocks with a poison value (allocate everything we can, fill, free) and run
it again. Any difference means some kernel read memory it never wrote (torch.empty scratch).

    python tools/poison_check.py [--model EA_GNN] [--bf16] [--config cfg2]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "buck-gnn_amd"))

import torch  # noqa: E402

import bgnn  # noqa: E402
from bgnn import synthetic as S  # noqa: E402


def poison(value: float, gib: float):
    """Fill `gib` GiB of fresh allocations with `value` and free them back to the cache."""
    bufs = []
    left = int(gib * (1 << 30))
    while left > 0:
        n = min(left, 1 << 30)
        bufs.append(torch.full((n // 4,), value, dtype=torch.float32, device="cuda"))
        left -= n
    torch.cuda.synchronize()
    del bufs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="EA_GNN")
    ap.add_argument("--bf16", action="store_true")
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--gib", type=float, default=48.0)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    b = S.make_config_batch(args.config).to(dev)
    torch.manual_seed(0)
    m = bgnn.BuckGNN(16, 5, hidden_channels=512, num_layers=6, dropout_rate=0.0, model_name=args.model).to(dev)
    m.ea_bf16 = args.bf16
    m.train()

    def run():
        m.zero_grad(set_to_none=True)
        pred, _ = m(b.x, b.edge_index, b.edge_attr, b.batch)
        loss = bgnn.RelativeErrorLoss()(pred, b.y)
        loss.backward()
        torch.cuda.synchronize()
        return pred.detach().clone(), {k: p.grad.detach().clone() for k, p in m.named_parameters()
                                        if p.grad is not None}

    p0, g0 = run()
    for val in (float("nan"), 1e30, -7.0):
        torch.cuda.empty_cache()
        poison(val, args.gib)
        p1, g1 = run()
        bad = [k for k in g0 if not torch.equal(g0[k], g1[k])]
        same = torch.equal(p0, p1)
        print(f"poison {val}: prediction {'identical' if same else 'DIFFERS'}; "
              f"{len(bad)} gradients differ {bad[:6]}", flush=True)
        if not same:
            print("  pred", p0[:4].tolist(), p1[:4].tolist())


if __name__ == "__main__" and "--gemm" not in sys.argv:
    main()


def gemm_shapes():
    """Per-GEMM check: bf16 / f16x3 GEMMs of the EA_GNN shapes, poisoned between two calls."""
    from bgnn import fused
    from bgnn import ea
    from bgnn.graph import SegmentIndex
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    E, N = 715872, 80656
    shapes = [(E, 64, 5, 0, 1), (E, 128, 64, 0, 1), (E, 512, 128, 0, 1), (N, 1536, 512, 0, 1), (E, 512, 512, 0, 1),
              (E, 512, 512, 0, 0), (512, 512, E, 1, 0), (64, 5, E, 1, 0), (N, 512, 1024, 0, 1), (4000, 33, 70, 0, 1)]
    for bf16 in (True, False):
        for (M, Nn, K, ta, tb) in shapes:
            a = torch.randn(K, M, device=dev) if ta else torch.randn(M, K, device=dev)
            b = torch.randn(Nn, K, device=dev) if tb else torch.randn(K, Nn, device=dev)
            c0 = fused.gemm(a, b, bool(ta), bool(tb), bf16=bf16)
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
            poison(1e30, 24.0)
            c1 = fused.gemm(a, b, bool(ta), bool(tb), bf16=bf16)
            torch.cuda.synchronize()
            print(f"gemm bf16={bf16} {M}x{Nn}x{K} ta={ta} tb={tb}: "
                  f"{'ok' if torch.equal(c0, c1) else 'DIFFERS max ' + str((c0 - c1).abs().max().item())}", flush=True)
            del a, b, c0, c1
    # gather-add epilogue GEMM
    idx = torch.randint(0, N, (E,), device=dev)
    seg = SegmentIndex.build(idx, N)
    for bf16 in (True, False):
        e = torch.randn(E, 512, device=dev)
        W = torch.randn(512, 512, device=dev)
        p1 = torch.randn(N, 512, device=dev)
        o0 = ea._LinearGatherReLU.apply(e, W, None, p1, seg, None, None, bf16)
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        poison(1e30, 24.0)
        o1 = ea._LinearGatherReLU.apply(e, W, None, p1, seg, None, None, bf16)
        torch.cuda.synchronize()
        print(f"gather_add bf16={bf16}: {'ok' if torch.equal(o0, o1) else 'DIFFERS'}", flush=True)


if __name__ == "__main__" and "--gemm" in sys.argv:
    gemm_shapes()
