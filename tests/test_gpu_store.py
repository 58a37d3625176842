"""GPU: device-resident graph store (bgnn.GraphStore).

A batch gathered on the device must be bit-identical to the host collation
(Batch.from_data_list, PyG rules) of the same graphs, and its graph structure bit-identical
to Graph.build / SegmentIndex.build of the collated edge_index / batch vector, including the
heavy-row plan counts the store derives on the host. A train step on a store batch gives
exactly the same loss and gradients as on the host-collated batch."""
import numpy as np
import pytest
import torch

import bgnn
from bgnn import synthetic as S
from bgnn.data import Batch, Data
from bgnn.graph import Graph, SegmentIndex, _graph_cache, _index_cache

pytestmark = pytest.mark.gpu


def dataset():
    gs = []
    for i in range(7):   # mixed sizes: meshes with random virtual edges and super-node meshes
        gs.append(S.make_mesh_graph(6 + 3 * i, seed=i, super_node=(i % 3 == 2)))
    # a graph without edges and a one-node graph (edge cases of the collation)
    gs.append(Data(x=torch.randn(3, 16), edge_index=torch.zeros(2, 0, dtype=torch.int64),
                   edge_attr=torch.zeros(0, 5), y=torch.rand(1)))
    gs.append(Data(x=torch.randn(1, 16), edge_index=torch.tensor([[0], [0]]), edge_attr=torch.rand(1, 5),
                   y=torch.rand(1)))
    return gs


def csr_equal(a, b):
    n = a.n_rows if hasattr(a, "n_rows") else None
    assert torch.equal(a.rowptr, b.rowptr)
    nnz = int(b.rowptr[-1])
    assert torch.equal(a.col[:nnz], b.col[:nnz])
    assert (a.plan.n_heavy, a.plan.n_chunks) == (b.plan.n_heavy, b.plan.n_chunks)
    nh, nc = b.plan.n_heavy, b.plan.n_chunks
    assert torch.equal(a.plan.heavy_row[:nh], b.plan.heavy_row[:nh])
    assert torch.equal(a.plan.heavy_chunk0[:nh + 1], b.plan.heavy_chunk0[:nh + 1])
    assert torch.equal(a.plan.chunk_heavy[:nc], b.plan.chunk_heavy[:nc])


def groups_equal(a, b, rowptr):
    """Same row-group plan: same group starts, counts and keys in every group's range."""
    assert (a is None) == (b is None)
    if b is None:
        return
    assert a.n_groups == b.n_groups and a.rows == b.rows
    assert torch.equal(a.gcnt[:b.n_groups], b.gcnt[:b.n_groups])
    if b.grow is not None:
        assert torch.equal(a.grow, b.grow)
    rp, cnt = rowptr.cpu(), b.gcnt.cpu()
    starts = b.grow.cpu() if b.grow is not None else torch.arange(b.n_groups) * b.rows
    for g in range(b.n_groups):
        lo = int(rp[int(starts[g])])
        hi = lo + int(cnt[g])
        assert torch.equal(a.gsrc[lo:hi], b.gsrc[lo:hi])
        assert torch.equal(a.gmask[lo:hi], b.gmask[lo:hi])


@pytest.mark.parametrize("ids", [[0, 1, 2, 3, 4, 5, 6, 7, 8], [6, 2, 2, 8, 0], [7], [5, 7, 3]])
def test_store_batch_matches_host_collation(dev, ids):
    gs = dataset()
    store = bgnn.GraphStore(gs, dev, chunk=16)
    b = store.batch(ids)
    ref = Batch.from_data_list([gs[i] for i in ids]).to(dev)
    for k in ("x", "edge_index", "edge_attr", "y", "batch", "ptr"):
        assert torch.equal(b[k], ref[k]), k
    assert b.num_graphs == len(ids) and b.num_nodes == ref.num_nodes
    # graph structure registered for prepare() equals a fresh build from the collated edge_index
    g = _graph_cache.peek(b.edge_index, (b.num_nodes, 16))
    assert g is not None
    r = Graph.build(ref.edge_index, ref.num_nodes, chunk=16)
    csr_equal(g.fwd, r.fwd)
    csr_equal(g.bwd, r.bwd)
    assert torch.equal(g.perm_t[:r.num_edges], r.perm_t[:r.num_edges])
    # row-group plans: groups start at every graph's first node; the gathered per-graph plans
    # equal a plan built on the collated CSR with the same group starts
    from bgnn.graph import enqueue_groups
    gf = g.fwd.groups
    assert gf is not None and gf.grow is not None
    R, ptr = gf.rows, ref.ptr.cpu().tolist()
    want = [p + k * R for p, q in zip(ptr[:-1], ptr[1:]) for k in range((q - p + R - 1) // R)] + [ptr[-1]]
    assert gf.grow.cpu().tolist() == want
    for mine, csr in ((g.fwd, r.fwd), (g.bwd, r.bwd)):
        want_g = enqueue_groups(csr.rowptr, csr.col, r.num_nodes, r.num_edges, 16, R, gf.grow, gf.n_groups)
        groups_equal(mine.groups, want_g, csr.rowptr)
    seg = _index_cache.peek(b.batch, ("batch",))
    rs = SegmentIndex.build(ref.batch, len(ids), chunk=16)
    csr_equal(seg.fwd, rs.fwd)
    assert torch.equal(seg.bwd.col[:rs.n], rs.bwd.col[:rs.n])
    # prepare() must reuse the registered structures (no rebuild)
    g2, s2 = bgnn.prepare(b.edge_index, b.num_nodes, b.batch, b.num_graphs, chunk=16)
    assert g2 is g and s2 is seg


def test_store_loader_epoch_and_shards(dev):
    gs = dataset()
    store = bgnn.GraphStore(gs, dev)
    seen = []
    for b in store.loader(batch_size=4, shuffle=True, seed=3):
        seen.append(b.num_graphs)
    assert sum(seen) == len(gs) and seen[:-1] == [4] * (len(seen) - 1)
    # DistributedSampler-style shards are disjoint and cover the epoch
    n0 = sum(b.num_graphs for b in store.loader(4, shuffle=True, seed=3, rank=0, world_size=2))
    n1 = sum(b.num_graphs for b in store.loader(4, shuffle=True, seed=3, rank=1, world_size=2))
    assert n0 + n1 == len(gs)


def test_store_rejects_bad_ids(dev):
    store = bgnn.GraphStore(dataset(), dev)
    with pytest.raises(IndexError):
        store.batch([0, 99])
    with pytest.raises(ValueError):
        store.batch([])


@pytest.mark.parametrize("super_node", [False, True])
def test_train_step_on_store_batch_equals_host_batch(dev, super_node):
    """A train step on a store batch equals one on the host-collated batch. The graph structure is
    bit-identical; the row-group plans start groups at graph starts on the store path and every
    R rows on the host path, so the aggregation sums in a different order: loss and gradients
    agree to fp32 rounding (compared before the optimizer update, whose first Adam step would
    amplify sign flips of near-zero gradients)."""
    gs = [S.make_mesh_graph(20, seed=s, super_node=super_node) for s in range(4)]
    store = bgnn.GraphStore(gs, dev)
    results = []
    for use_store in (True, False):
        bgnn.clear_caches()
        torch.manual_seed(0)
        model = bgnn.BuckGNN(16, 5, hidden_channels=128, num_layers=6, dropout_rate=0.0,
                             model_name="GraphSage_addAggr").to(dev).train()

        class NoStep:
            def zero_grad(self, set_to_none=True):
                model.zero_grad(set_to_none=set_to_none)

            def step(self):
                pass

        batch = store.batch([0, 1, 2, 3]) if use_store else Batch.from_data_list(gs).to(dev)
        loss = bgnn.train_step(model, batch, NoStep(), bgnn.RelativeErrorLoss(), bgnn.EigenvalueScaler(1.0, 0.5))
        results.append((float(loss), [p.grad.detach().clone() for p in model.parameters() if p.grad is not None]))
    assert results[0][0] == pytest.approx(results[1][0], rel=1e-5)
    assert len(results[0][1]) == len(results[1][1])
    for a, b in zip(results[0][1], results[1][1]):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-4 * float(b.abs().max()) + 1e-12)

