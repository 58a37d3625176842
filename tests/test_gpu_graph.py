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
