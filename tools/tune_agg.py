#!/usr/bin/env python
"""A/B the aggregation kernel variants on cfg2/cfg3 in ONE process (interleaved rounds,
median of per-launch HIP-event times), checking that every variant agrees to fp32 rounding
results. Usage: python tools/tune_agg.py [--config cfg2] [--rounds 20]"""
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

KNOB = {"kernel": 1, "blocks": 2, "u": 3, "nt": 4, "gblocks": 7, "gu": 10, "gze": 11}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--rounds", type=int, default=20)
    ap.add_argument("--variants", default="sweep12,group8_b512,group8_b768,group8_b1024,group4_b512,group4_b1024")
    ap.add_argument("--no-virtual", action="store_true", help="cfg2 meshes without the random virtual edges")
    ap.add_argument("--flush", action="store_true",
                    help="write 1 GiB between launches (cold L2 / Infinity Cache, as inside a train step)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    if args.no_virtual:
        b = synthetic.Batch.from_data_list([synthetic.make_mesh_graph(71, g, virtual_edges=False) for g in range(16)])
    else:
        b = synthetic.make_config_batch(args.config)
    from bgnn import graph as Gm
    graphs = {}
    for rows in (0, 4, 8):
        Gm.GROUP_ROWS = rows
        graphs[rows] = Graph.build(b.edge_index.to(dev), b.num_nodes)
    Gm.GROUP_ROWS = 8
    cur = {"g": graphs[8]}
    N, E, H = b.num_nodes, b.num_edges, 512
    torch.manual_seed(0)
    z = torch.randn(N, 2 * H, device=dev)
    zp = z.view(N, 2, H).permute(1, 0, 2).contiguous()   # plane layout [z_l ; z_r], same values
    bias = torch.randn(H, device=dev)
    s = torch.cuda.current_stream().cuda_stream

    layout = {"il": True}

    def set_variant(v):
        # "blocked" | "sweep[U][_b<blocks>][_nt][_planes]" | "group<R>[_b<blocks>][_nt][_planes]"
        # (U = 0 auto, 8, 12, 16; R = 4 or 8 rows per group; planes = z as two [N, H] planes)
        kern, u, blocks, nt, rows, gu, gze = 2, 0, 1024, 1, 0, 8, 0
        layout["il"] = not v.endswith("_planes")
        parts = v.split("_")
        if v == "blocked":
            kern = 1
        elif parts[0].startswith("group"):
            kern, rows, blocks = 0, int(parts[0][5:] or 8), 1024
        else:
            u = int(parts[0][5:] or 0)
        for p in parts[1:]:
            if p.startswith("b"):
                blocks = int(p[1:])
            elif p == "nt0":
                nt = 0
            elif p == "u16":     # row-group kernel: 16 source rows per gather batch
                gu = 16
            elif p == "ze":      # row-group SAGE epilogue: z_r loads before the gathers
                gze = 1
        cur["g"] = graphs[rows]
        _lib.call("bgnn_set_tuning", KNOB["kernel"], kern)
        _lib.call("bgnn_set_tuning", KNOB["u"], u)
        _lib.call("bgnn_set_tuning", KNOB["blocks" if kern else "gblocks"], blocks)
        _lib.call("bgnn_set_tuning", KNOB["nt"], nt)
        _lib.call("bgnn_set_tuning", KNOB["gu"], gu)
        _lib.call("bgnn_set_tuning", KNOB["gze"], gze)

    def run_fwd():
        g = cur["g"]
        slots = _lib.query("bgnn_sage_fwd_slots", g.fwd.ref())
        o = torch.empty(N, H, device=dev)
        nrm = torch.empty(N, device=dev)
        bnp = torch.empty(slots, 2, H, device=dev)
        part = torch.empty(max(g.fwd.plan.n_chunks, 1) * H, device=dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        if layout["il"]:
            zl, zr, ld = z, z[:, H:], 2 * H
        else:
            zl, zr, ld = zp[0], zp[1], H
        _lib.call("bgnn_sage_fwd", g.fwd.ref(), zl.data_ptr(), ld, zr.data_ptr(), ld, bias.data_ptr(), H, 0,
                  o.data_ptr(), nrm.data_ptr(), bnp.data_ptr(), part.data_ptr(), None, 0, s)
        e1.record()
        return (e0, e1), (o, nrm, bnp.sum(0))

    def run_bwd():
        g = cur["g"]
        gx = torch.empty(N, 2 * H, device=dev)
        part = torch.empty(max(g.bwd.plan.n_chunks, 1) * H, device=dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        _lib.call("bgnn_spmm_bwd", g.bwd.ref(), g.perm_t.data_ptr(), g.fwd.rowptr.data_ptr(), z[:, H:].data_ptr(),
                  z.stride(0), H, 0, gx.data_ptr(), gx.stride(0), part.data_ptr(), None, 0, s)
        e1.record()
        return (e0, e1), (gx[:, :H],)

    variants = args.variants.split(",")
    times = {(v, k): [] for v in variants for k in ("fwd", "bwd")}
    ref = {}
    junk = torch.empty(1 << 28, device=dev) if args.flush else None
    for rnd in range(args.rounds + 2):
        for v in variants:
            set_variant(v)
            for k, fn in (("fwd", run_fwd), ("bwd", run_bwd)):
                if junk is not None:
                    junk.fill_(1.0)
                ev, outs = fn()
                torch.cuda.synchronize()
                if rnd >= 2:
                    times[(v, k)].append(ev[0].elapsed_time(ev[1]))
                if rnd == 0:
                    if k not in ref:
                        ref[k] = [t.clone() for t in outs]
                    else:
                        for a, bb in zip(ref[k], outs):
                            if a.dim() == 2 and not torch.allclose(a, bb, rtol=1e-5, atol=1e-5):
                                print(f"MISMATCH {v} {k}: max diff {(a - bb).abs().max().item()}")
    set_variant("group8")
    fwd_bytes = 3 * N * H * 4 + 4 * E + 4 * (N + 1) + 4 * N
    bwd_bytes = 2 * N * H * 4 + 4 * E + 4 * (N + 1)
    res = {}
    for v in variants:
        f = statistics.median(times[(v, "fwd")])
        bw = statistics.median(times[(v, "bwd")])
        res[v] = {"fwd_us": round(f * 1e3, 1), "fwd_GBs": round(fwd_bytes / f / 1e6, 1),
                  "bwd_us": round(bw * 1e3, 1), "bwd_GBs": round(bwd_bytes / bw / 1e6, 1)}
        print(f"{v:16s} fwd {f*1e3:8.1f} us {fwd_bytes/f/1e6:8.1f} GB/s | bwd {bw*1e3:8.1f} us "
              f"{bwd_bytes/bw/1e6:8.1f} GB/s")
    print(json.dumps({"config": args.config, "N": N, "E": E, "results": res}))


if __name__ == "__main__":
    main()
