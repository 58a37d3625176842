#!/usr/bin/env python
"""Why is the transpose aggregation (bgnn_spmm_bwd) slower than the fused forward? A/B on
cfg2 in one process, cache flushed between launches (as inside a train step), medians of
HIP-event times:

  sage_fwd      bgnn_sage_fwd (forward CSR, z interleaved [N, 2H], SAGE epilogue)
  plain_fwd     bgnn_spmm_fwd SUM on z_l (forward CSR, interleaved in, dense out)
  bwd_t         bgnn_spmm_bwd SUM, transpose CSR, dh = dz[:, H:], out dz[:, :H] (the train step)
  bwd_fwdcsr    the same gather with the FORWARD CSR (= transpose as a multiset: symmetric graph)
  bwd_dense     transpose CSR, dense dh [N, H] in, dense out
  bwd_nt0       bwd_t with non-temporal hints off

Usage: python tools/agg_bwd_ab.py [--rounds 15]"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "buck-gnn_amd"))

import torch  # noqa: E402

from bgnn import _lib, synthetic  # noqa: E402
from bgnn.graph import Graph  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=15)
    ap.add_argument("--config", default="cfg2")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    b = synthetic.make_config_batch(args.config)
    g = Graph.build(b.edge_index.to(dev), b.num_nodes)
    N, E, H = b.num_nodes, b.num_edges, 512
    torch.manual_seed(0)
    z = torch.randn(N, 2 * H, device=dev)
    dz = torch.randn(N, 2 * H, device=dev)
    dh_dense = dz[:, H:].contiguous()
    bias = torch.randn(H, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    slots = _lib.query("bgnn_sage_fwd_slots", g.fwd.ref())
    o = torch.empty(N, H, device=dev)
    nrm = torch.empty(N, device=dev)
    bnp = torch.empty(slots, 2, H, device=dev)
    part = torch.empty(max(g.fwd.plan.n_chunks, g.bwd.plan.n_chunks, 1) * H, device=dev)
    out_dense = torch.empty(N, H, device=dev)

    def sage_fwd():
        _lib.call("bgnn_sage_fwd", g.fwd.ref(), z.data_ptr(), 2 * H, z[:, H:].data_ptr(), 2 * H, bias.data_ptr(), H,
                  0, o.data_ptr(), nrm.data_ptr(), bnp.data_ptr(), part.data_ptr(), None, 0, s)

    def plain_fwd():
        _lib.call("bgnn_spmm_fwd", g.fwd.ref(), z.data_ptr(), 2 * H, H, 0, out_dense.data_ptr(), H, None,
                  part.data_ptr(), s)

    def bwd(csr, src, ld_src, dst, ld_dst):
        def f():
            _lib.call("bgnn_spmm_bwd", csr.ref(), g.perm_t.data_ptr(), g.fwd.rowptr.data_ptr(), src.data_ptr(),
                      ld_src, H, 0, dst.data_ptr(), ld_dst, part.data_ptr(), None, 0, s)
        return f

    def nt0(f):
        def w():
            _lib.call("bgnn_set_tuning", 4, 0)
            f()
            _lib.call("bgnn_set_tuning", 4, 1)
        return w

    def knob(f, k, v):
        def w():
            old = _lib.query("bgnn_get_tuning", k)
            _lib.call("bgnn_set_tuning", k, v)
            f()
            _lib.call("bgnn_set_tuning", k, old)
        return w

    bwd_t = bwd(g.bwd, dz[:, H:], 2 * H, dz, 2 * H)
    variants = {
        "sage_fwd": sage_fwd,
        "plain_fwd": plain_fwd,
        "bwd_t": bwd_t,
        "bwd_fwdcsr": bwd(g.fwd, dz[:, H:], 2 * H, dz, 2 * H),
        "bwd_dense": bwd(g.bwd, dh_dense, H, out_dense, H),
        "bwd_nt0": nt0(bwd_t),
    }
    junk = torch.empty(1 << 28, device=dev)
    times = {k: [] for k in variants}
    for rnd in range(args.rounds + 2):
        for k, f in variants.items():
            junk.fill_(1.0)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            f()
            e1.record()
            torch.cuda.synchronize()
            if rnd >= 2:
                times[k].append(e0.elapsed_time(e1) * 1e3)
    res = {k: round(statistics.median(v), 1) for k, v in times.items()}
    for k, v in res.items():
        print(f"{k:12s} {v:8.1f} us")
    print(json.dumps({"config": args.config, "N": N, "E": E, "median_us": res}))


if __name__ == "__main__":
    main()
