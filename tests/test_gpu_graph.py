"""GPU: edge_index -> CSR / transpose CSR / heavy-row plan, bit-exact against numpy."""
import numpy as np
import pytest
import torch

import bgnn
from bgnn.graph import Graph, SegmentIndex, make_plan
from bgnn import synthetic as S

pytestmark = pytest.mark.gpu


def np_csr(keys, vals, n):
    order = np.argsort(keys, kind="stable")
    rowptr = np.zeros(n + 1, dtype=np.int64)
    np.add.at(rowptr, keys + 1, 1)
    return np.cumsum(rowptr), vals[order], order


def np_groups(rowptr, col, n, chunk, R, grow=None):
    """Host restatement of bgnn_group_plan's rule (include/bgnn.h): per group of at most R rows
    (rows [g*R, g*R+R), or [grow[g], grow[g+1])), the light rows' entries keyed by (source,
    occurrence within the row), numbered by first appearance, with the mask of the rows holding
    each key."""
    if grow is None:
        grow = list(range(0, n, R)) + [n]
    G = len(grow) - 1
    gsrc, gmask, gcnt = {}, {}, np.zeros(G, dtype=np.int64)
    for g in range(G):
        keys, src, mask = {}, [], []
        for t in range(grow[g + 1] - grow[g]):
            r = grow[g] + t
            b, e = int(rowptr[r]), int(rowptr[r + 1])
            if e - b > chunk:
                continue
            occ = {}
            for q in range(b, e):
                s_ = int(col[q])
                k = (s_, occ.get(s_, 0))
                occ[s_] = k[1] + 1
                if k not in keys:
                    keys[k] = len(src)
                    src.append(s_)
                    mask.append(0)
                mask[keys[k]] |= 1 << t
        base = int(rowptr[grow[g]])
        for i, (s_, m) in enumerate(zip(src, mask)):
            gsrc[base + i], gmask[base + i] = s_, m
        gcnt[g] = len(src)
    return gsrc, gmask, gcnt


def check_groups(csr, n, chunk):
    gr = csr.groups
    if gr is None:
        return
    rp, col = csr.rowptr.cpu().numpy(), csr.col.cpu().numpy()
    grow = gr.grow.cpu().tolist() if gr.grow is not None else None
    gsrc, gmask, gcnt = np_groups(rp, col, n, chunk, gr.rows, grow)
    assert np.array_equal(gr.gcnt.cpu().numpy(), gcnt)
    got_s, got_m = gr.gsrc.cpu().numpy(), gr.gmask.cpu().numpy()
    for pos, s_ in gsrc.items():
        assert got_s[pos] == s_ and got_m[pos] == gmask[pos], pos


def check_graph(ei_np, n, dev, chunk=64):
    ei = torch.from_numpy(ei_np).to(dev)
    g = Graph.build(ei, n, chunk=chunk)
    src, dst = ei_np[0], ei_np[1]
    rp, col, order = np_csr(dst, src, n)
    assert np.array_equal(g.fwd.rowptr.cpu().numpy(), rp)
    E = ei_np.shape[1]
    assert np.array_equal(g.fwd.col[:E].cpu().numpy(), col)
    # transpose: rows = sources, entries in forward-CSR order
    rpt, pos, _ = np_csr(col, np.arange(E), n)
    assert np.array_equal(g.bwd.rowptr.cpu().numpy(), rpt)
    assert np.array_equal(g.perm_t[:E].cpu().numpy(), pos)
    assert np.array_equal(g.bwd.col[:E].cpu().numpy(), dst[order][pos])
    # heavy plan
    deg = np.diff(rp)
    heavy = np.nonzero(deg > chunk)[0]
    p = g.fwd.plan
    assert p.n_heavy == len(heavy)
    assert np.array_equal(p.heavy_row[:len(heavy)].cpu().numpy(), heavy)
    nch = (deg[heavy] + chunk - 1) // chunk
    assert p.n_chunks == int(nch.sum())
    c0 = np.concatenate([[0], np.cumsum(nch)])
    assert np.array_equal(p.heavy_chunk0[:len(heavy) + 1].cpu().numpy(), c0)
    # row-group plans of both CSRs
    check_groups(g.fwd, n, chunk)
    check_groups(g.bwd, n, chunk)
    return g


def test_random_graph_with_duplicates_and_self_loops(dev):
    rng = np.random.default_rng(0)
    n, E = 300, 4000
    ei = rng.integers(0, n, size=(2, E))
    ei[:, :50] = ei[:, 50:100]                 # duplicates
    ei[1, 100:120] = ei[0, 100:120]            # self loops
    check_graph(ei, n, dev, chunk=8)


def test_isolated_nodes_and_empty_graph(dev):
    ei = np.array([[0, 5], [5, 0]])
    g = check_graph(ei, 10, dev)
    assert g.fwd.degree().cpu().tolist() == [1, 0, 0, 0, 0, 1, 0, 0, 0, 0]
    g0 = Graph.build(torch.zeros(2, 0, dtype=torch.long, device=dev), 7)
    assert g0.fwd.rowptr.cpu().tolist() == [0] * 8 and g0.fwd.plan.n_heavy == 0


def test_mesh_with_super_node_plan(dev):
    b = S.make_batch(20, 3, super_node=True)
    g = check_graph(b.edge_index.numpy(), b.num_nodes, dev, chunk=64)
    assert g.fwd.plan.n_heavy == 3 and g.bwd.plan.n_heavy == 3   # the three super nodes


def test_out_of_range_index_raises(dev):
    ei = torch.tensor([[0, 1], [1, 9]], device=dev)
    with pytest.raises(IndexError):
        Graph.build(ei, 5)


def test_segment_index_unsorted(dev):
    idx = np.array([2, 0, 2, 1, 0, 2, 4])
    s = SegmentIndex.build(torch.from_numpy(idx).to(dev), 6)
    rp, col, _ = np_csr(idx, np.arange(len(idx)), 6)
    assert np.array_equal(s.fwd.rowptr.cpu().numpy(), rp)
    assert np.array_equal(s.fwd.col[:len(idx)].cpu().numpy(), col)


@pytest.mark.parametrize("rows", [4, 8])
def test_group_plan_meshes(dev, rows):
    from bgnn import graph as G
    old = G.GROUP_ROWS
    G.GROUP_ROWS = rows
    try:
        b = S.make_batch(23, 3)
        g = check_graph(b.edge_index.numpy(), b.num_nodes, dev)
        assert g.fwd.groups is not None and g.fwd.groups.rows == rows
        # fewer fetched source rows than edges (neighbours shared inside a group)
        assert int(g.fwd.groups.gcnt.sum()) < 0.75 * b.num_edges
    finally:
        G.GROUP_ROWS = old


def test_group_plan_explicit_group_starts(dev):
    """bgnn_group_plan with caller-given group starts (groups of 1..R rows, as the GraphStore
    uses to align groups with graph starts), against the host restatement."""
    from bgnn.graph import Csr, enqueue_groups
    rng = np.random.default_rng(7)
    n, E, R = 500, 6000, 8
    ei = rng.integers(0, n, size=(2, E))
    ei[:, :40] = ei[:, 40:80]                  # duplicate edges
    g = Graph.build(torch.from_numpy(ei).to(dev), n, chunk=32)
    sizes = rng.integers(1, R + 1, size=n)
    starts = np.concatenate([[0], np.cumsum(sizes)])
    grow = starts[starts < n].tolist() + [n]
    grow_d = torch.tensor(grow, dtype=torch.int32, device=dev)
    for csr in (g.fwd, g.bwd):
        gr = enqueue_groups(csr.rowptr, csr.col, n, E, 32, R, grow_d, len(grow) - 1)
        check_groups(Csr(csr.rowptr, csr.col, n, E, csr.plan, gr), n, 32)
