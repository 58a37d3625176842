#!/usr/bin/env python
"""Interleaved A/B of aggregation-kernel settings (bgnn_set_tuning knobs) on a config's batch as the
training step runs them: the fused SAGE forward (bgnn_sage_fwd, z interleaved [N, 2H]) and the
transpose aggregation (bgnn_spmm_bwd, dh = dz[:, H:] -> dz[:, :H]); 1 GiB cache flush between
launches, median HIP-event times, bit-identity against the first setting.
    python tools/agg_knob_ab.py [--config cfg2] [--rounds 15] "" "7=2048" ..."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "buck-gnn_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from bgnn import _lib, synthetic  # noqa: E402
from bgnn.graph import Graph  # noqa: E402


def cluster_order(src: np.ndarray, dst: np.ndarray, n: int, strip: int = 4) -> np.ndarray:
    """(Round-4 experiment, not adopted: R = 8 groups over this order ran slower than R = 4 in
    dataset order, profiles/r04_ab_agg_knobs.txt.) A node order for row groups of 2 * strip rows (graph-local; returns new -> old node ids).

    The row-group aggregation kernels (csrc/spmm.hip k_seg_group) fetch every distinct source
    row of a group of consecutive target rows once. In the order a mesh is numbered (sorted
    Nastran ids, GraphCreate.py:150: row-major), consecutive rows are a 1-D strip of the mesh,
    whose neighbourhoods overlap along one direction only. Here the graph's strips of `strip`
    consecutive rows are paired greedily, each with the not yet paired strip that shares the most
    source rows (on a mesh: the strip one mesh row away), and each pair is placed consecutively,
    so a group of 2 * strip rows is a 2-D patch: cfg2 meshes fetch 4.23 source rows per target row
    in groups of 8 instead of 4.74 (1-D strips of 8) or 5.47 (strips of 4). Strips left unpaired
    (and a last partial strip) go to the end. Generic: uses the edge list only."""
    n = int(n)
    order = np.argsort(dst, kind="stable")
    rp = np.zeros(n + 1, np.int64)
    np.add.at(rp, dst + 1, 1)
    rp = np.cumsum(rp)
    s_sorted = src[order]
    G = (n + strip - 1) // strip
    keys = [set(s_sorted[rp[g * strip]:rp[min(n, g * strip + strip)]].tolist()) for g in range(G)]
    full = [min(n, g * strip + strip) - g * strip == strip for g in range(G)]
    partner = [-1] * G
    for g in range(G):
        if partner[g] >= 0 or not full[g]:
            continue
        best, bs = -1, 0
        for c in sorted({k // strip for k in keys[g]}):
            if c == g or partner[c] >= 0 or not full[c]:
                continue
            sh = len(keys[g] & keys[c])
            if sh > bs:
                bs, best = sh, c
        if best >= 0:
            partner[g], partner[best] = best, g
    perm, rest, done = [], [], [False] * G
    for g in range(G):
        if done[g]:
            continue
        done[g] = True
        rows = list(range(g * strip, min(n, g * strip + strip)))
        if partner[g] >= 0:
            p = partner[g]
            done[p] = True
            perm += rows + list(range(p * strip, p * strip + strip))
        else:
            rest += rows
    return np.asarray(perm + rest, dtype=np.int64)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=15)
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--group-rows", type=int, default=4)
    ap.add_argument("--reorder", action="store_true", help="strip-pair node order (bgnn.store.cluster_order)")
    ap.add_argument("settings", nargs="*", default=[""])
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    from bgnn import graph as G_
    G_.GROUP_ROWS = args.group_rows
    b = synthetic.make_config_batch(args.config)
    ei = b.edge_index
    if args.reorder:
        import numpy as np
        src, dst = ei.numpy()
        inv = np.empty(b.num_nodes, np.int64)
        ptr = b.ptr.numpy()
        for k in range(b.num_graphs):   # per graph (graphs are contiguous node ranges)
            lo, hi = int(ptr[k]), int(ptr[k + 1])
            m = (dst >= lo) & (dst < hi)
            perm = cluster_order(src[m] - lo, dst[m] - lo, hi - lo)
            inv[lo + perm] = lo + np.arange(hi - lo)
        ei = torch.from_numpy(np.stack([inv[src], inv[dst]]))
    g = Graph.build(ei.to(dev), b.num_nodes)
    N, E, H = b.num_nodes, b.num_edges, 512
    torch.manual_seed(0)
    z = torch.randn(N, 2 * H, device=dev)
    dz = torch.randn(N, 2 * H, device=dev)
    bias = torch.randn(H, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    slots = _lib.query("bgnn_sage_fwd_slots", g.fwd.ref())
    o = torch.empty(N, H, device=dev)
    nrm = torch.empty(N, device=dev)
    bnp = torch.empty(max(slots, 2048), 2, H, device=dev)
    part = torch.empty(max(g.fwd.plan.n_chunks, g.bwd.plan.n_chunks, 1) * H, device=dev)
    flush = torch.empty(1 << 28, device=dev)
    fwd_bytes = 3 * N * H * 4 + 4 * E + 4 * (N + 1) + 4 * N
    bwd_bytes = 2 * N * H * 4 + 4 * E + 4 * (N + 1)

    def sage_fwd():
        _lib.call("bgnn_sage_fwd", g.fwd.ref(), z.data_ptr(), 2 * H, z[:, H:].data_ptr(), 2 * H, bias.data_ptr(), H,
                  0, o.data_ptr(), nrm.data_ptr(), bnp.data_ptr(), part.data_ptr(), None, 0, s)
        return o

    def bwd_t():
        _lib.call("bgnn_spmm_bwd", g.bwd.ref(), g.perm_t.data_ptr(), g.fwd.rowptr.data_ptr(), dz[:, H:].data_ptr(),
                  2 * H, H, 0, dz.data_ptr(), 2 * H, part.data_ptr(), None, 0, s)
        return dz[:, :H]

    def apply(setting, undo=None):
        for kv in filter(None, setting.split(";")):
            k, v = (int(t) for t in kv.split("="))
            if undo is not None:
                undo.append((k, _lib.query("bgnn_get_tuning", k)))
            _lib.call("bgnn_set_tuning", k, v)

    kernels = {"sage_fwd": (sage_fwd, fwd_bytes), "spmm_bwd": (bwd_t, bwd_bytes)}
    times = {(k, st): [] for k in kernels for st in args.settings}
    ref = {}
    for rnd in range(args.rounds + 2):
        for kname, (fn, _) in kernels.items():
            for st in args.settings:
                undo = []
                apply(st, undo)
                flush.fill_(float(rnd))
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                out = fn()
                e1.record()
                torch.cuda.synchronize()
                for k, v in reversed(undo):
                    _lib.call("bgnn_set_tuning", k, v)
                if rnd == 1:
                    ref[(kname, st)] = out.clone()
                if rnd >= 2:
                    times[(kname, st)].append(e0.elapsed_time(e1) * 1e3)
    for kname, (_, nbytes) in kernels.items():
        for st in args.settings:
            ts = sorted(times[(kname, st)])
            med = ts[len(ts) // 2]
            same = torch.equal(ref[(kname, st)], ref[(kname, args.settings[0])])
            print(f"{args.config} R{args.group_rows}{'r' if args.reorder else ''} {kname:8s} [{st or 'default':>16s}] median {med:7.1f} us  min {ts[0]:7.1f}  "
                  f"{nbytes / med / 1e6:7.1f} GB/s = {nbytes / med / 1e6 / 8000:.3f} of 8 TB/s  "
                  f"{'bit-identical' if same else 'DIFFERS'}", flush=True)


if __name__ == "__main__":
    main()
