#!/usr/bin/env python
"""A/B of s_setprio around the f16x3 GEMM's MFMA block (k_gemm_x6 ablations 9 / 10 force it on
/ off; the default puts it on the single-register-set 256x256 tiles) on the cfg2 SAGE shapes:
fwd z = x Wcat^T, dgrad dx = dz Wcat, wgrad dWcat = dz^T x. Alternating launches, HIP events,
medians; cache flushed before each launch. Results must be bit-identical.

    python tools/prio_ab.py [R]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "buck-gnn_amd"))
from bgnn import _lib, fused  # noqa: E402

R = int(sys.argv[1]) if len(sys.argv) > 1 else 15
dev = torch.device("cuda", 0)
flush = torch.empty(128 * 1024 * 1024, dtype=torch.float32, device=dev)
N_NODES, H = 80656, 512

# (name, a shape, b shape, trans_a, trans_b, x6 tile config of the production plan)
SHAPES = [("fwd", (N_NODES, H), (2 * H, H), False, True, 4),
          ("dgrad", (N_NODES, 2 * H), (H, 2 * H), False, True, 2),
          ("wgrad", (N_NODES, 2 * H), (N_NODES, H), True, False, 4)]
for name, sa, sb, ta, tb, cfg in SHAPES:
    torch.manual_seed(0)
    A = torch.randn(*sa, device=dev)
    B = torch.randn(*sb, device=dev) * 0.05
    am, bm = fused.absmax(A), fused.absmax(B)
    outs, ts = {}, {}
    for mode in (-1, 900 + cfg, 1000 + cfg):
        ts[mode] = []
    for i in range(R):
        for mode in ts:
            _lib.call("bgnn_gemm_set_cfg", mode)
            flush.fill_(float(i))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            o = fused.gemm(A, B, ta, tb, a_amax=am, b_amax=bm)
            e1.record()
            torch.cuda.synchronize()
            ts[mode].append(e0.elapsed_time(e1) * 1e3)
            outs[mode] = o
    _lib.call("bgnn_gemm_set_cfg", -1)
    med = {m: sorted(v)[len(v) // 2] for m, v in ts.items()}
    same = all(torch.equal(outs[m], outs[-1]) for m in outs)
    print(f"{name}: default {med[-1]:7.1f} us | prio on {med[900 + cfg]:7.1f} us | prio off {med[1000 + cfg]:7.1f} us"
          f" | bit-identical {same}", flush=True)
