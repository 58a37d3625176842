#!/usr/bin/env python
"""Experiment: row-group aggregation with deduplicated source lists (tools/proto/agg_group.hip)
against the production sweep kernel (bgnn_spmm_fwd, SUM), cfg2, H = 512, interleaved rounds."""
import argparse
import ctypes
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "buck-gnn_amd"))

import torch  # noqa: E402

from bgnn import _lib, synthetic  # noqa: E402
from bgnn.graph import Graph  # noqa: E402


def host_csr(ei, N):
    src, dst = ei[0], ei[1]
    order = np.argsort(dst, kind="stable")
    col = src[order].astype(np.int32)
    rowptr = np.zeros(N + 1, dtype=np.int64)
    np.add.at(rowptr, dst + 1, 1)
    return np.cumsum(rowptr).astype(np.int32), col


def group_plan(rowptr, col, N, R):
    G = (N + R - 1) // R
    gptr = np.zeros(G + 1, dtype=np.int32)
    srcs, masks = [], []
    for g in range(G):
        d = {}
        s_l, m_l = [], []
        for t in range(R):
            r = g * R + t
            if r >= N:
                break
            occ = {}
            for e in range(rowptr[r], rowptr[r + 1]):
                s = int(col[e])
                k = occ.get(s, 0)
                occ[s] = k + 1
                i = d.get((s, k))
                if i is None:
                    d[(s, k)] = len(s_l)
                    s_l.append(s)
                    m_l.append(1 << t)
                else:
                    m_l[i] |= 1 << t
        srcs.extend(s_l)
        masks.extend(m_l)
        gptr[g + 1] = len(srcs)
    return gptr, np.array(srcs, dtype=np.int32), np.array(masks, dtype=np.uint32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--rounds", type=int, default=15)
    ap.add_argument("--variants", default="4x2x8x1,8x2x8x1")
    ap.add_argument("--blocks", default="256,512,1024")
    ap.add_argument("--flush", action="store_true", help="write 1 GiB between launches (cold caches)")
    ap.add_argument("--qvariants", default="0x4x1x12x1024,0x4x1x12x2048,0x4x1x16x2048,0x2x1x12x1024,0x2x1x12x2048,"
                    "1x4x4x12x1024,1x4x4x12x2048,1x4x8x12x1024,1x4x8x12x2048,1x4x8x16x1024,1x2x4x12x1024,"
                    "1x2x8x12x1024,1x2x4x12x512")
    args = ap.parse_args()
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "proto", "libproto.so"))
    lib.proto_grp.restype = ctypes.c_int
    lib.proto_grp.argtypes = [ctypes.c_int] * 5 + [ctypes.c_void_p] * 5 + [ctypes.c_int64, ctypes.c_int64,
                                                                            ctypes.c_int, ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    b = synthetic.make_config_batch(args.config)
    N, E, H = b.num_nodes, b.num_edges, 512
    ei = b.edge_index.numpy()
    rowptr, col = host_csr(ei, N)
    plans = {}
    t0 = time.time()
    for R in sorted({int(v.split("x")[0]) for v in args.variants.split(",")}):
        gptr, gsrc, gmask = group_plan(rowptr, col, N, R)
        plans[R] = (torch.from_numpy(gptr).to(dev), torch.from_numpy(gsrc).to(dev),
                    torch.from_numpy(gmask.view(np.int32)).to(dev), len(gptr) - 1)
        print(f"R={R}: groups {len(gptr)-1} entries {len(gsrc)} ({len(gsrc)/N:.2f}/row vs {E/N:.2f} refs/row)",
              flush=True)
    print(f"plans built in {time.time()-t0:.1f}s", flush=True)
    g = Graph.build(b.edge_index.to(dev), N)
    torch.manual_seed(0)
    x = torch.randn(N, H, device=dev)
    ref = torch.zeros(N, H, device=dev, dtype=torch.float64).index_add_(
        0, b.edge_index[1].to(dev), x.double()[b.edge_index[0].to(dev)]).float()
    s = torch.cuda.current_stream().cuda_stream

    def run_base():
        out = torch.empty(N, H, device=dev)
        part = torch.empty(max(g.fwd.plan.n_chunks, 1) * H, device=dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        _lib.call("bgnn_spmm_fwd", g.fwd.ref(), x.data_ptr(), H, H, 0, out.data_ptr(), H, None, part.data_ptr(), s)
        e1.record()
        return (e0, e1), out

    def mk(v, blocks):
        R, nv, u, mode = (int(t) for t in v.split("x"))
        gptr, gsrc, gmask, G = plans[R]

        def run():
            out = torch.empty(N, H, device=dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            rc = lib.proto_grp(R, nv, u, mode, blocks, x.data_ptr(), out.data_ptr(), gptr.data_ptr(), gsrc.data_ptr(),
                               gmask.data_ptr(), G, N, H, s)
            e1.record()
            assert rc == 0, rc
            return (e0, e1), out
        return run

    lib.proto_q.restype = ctypes.c_int
    lib.proto_q.argtypes = [ctypes.c_int] * 5 + [ctypes.c_void_p] * 7 + [ctypes.c_int64, ctypes.c_int64,
                                                                       ctypes.c_int, ctypes.c_void_p]

    def mkq(kind, cs, R, u, blocks):
        gptr, gsrc, gmask, G = plans.get(R, (None, None, None, 0))

        def run():
            out = torch.empty(N, H, device=dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            rc = lib.proto_q(kind, cs, R, u, blocks, x.data_ptr(), out.data_ptr(), g.fwd.rowptr.data_ptr(),
                             g.fwd.col.data_ptr(), gptr.data_ptr() if gptr is not None else None,
                             gsrc.data_ptr() if gsrc is not None else None,
                             gmask.data_ptr() if gmask is not None else None, N, G, H, s)
            e1.record()
            assert rc == 0, rc
            return (e0, e1), out
        return run

    runs = {"base": run_base}
    for q in args.qvariants.split(","):
        if not q:
            continue
        kind, cs, R, u, bl = (int(t) for t in q.split("x"))
        runs[f"q{q}"] = mkq(kind, cs, R, u, bl)
    for v in args.variants.split(","):
        for bl in args.blocks.split(","):
            runs[f"grp{v}_b{bl}"] = mk(v, int(bl))
    times = {k: [] for k in runs}
    junk = torch.empty(1 << 28, device=dev) if args.flush else None
    for rnd in range(args.rounds + 2):
        for k, fn in runs.items():
            if junk is not None:
                junk.fill_(1.0)
            ev, out = fn()
            torch.cuda.synchronize()
            if rnd >= 2:
                times[k].append(ev[0].elapsed_time(ev[1]))
            if rnd == 0:
                err = ((out - ref).abs().max() / ref.abs().max()).item()
                print(f"{k:20s} max rel err {err:.2e}", flush=True)
    nbytes = 2 * N * H * 4 + 4 * E + 4 * (N + 1)
    for k in runs:
        t = statistics.median(times[k])
        print(f"{k:20s} {t*1e3:8.1f} us  {nbytes/t/1e6:8.1f} GB/s (alg)  min {min(times[k])*1e3:8.1f}", flush=True)


if __name__ == "__main__":
    main()
