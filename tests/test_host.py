"""Host-side logic (CPU only): synthetic inputs, PyG-compatible containers and
collation, the PyG shim, BuckGNN module/state-dict layout, and 'no CPU fallback'."""
import os
import sys

import numpy as np
import pytest
import torch

import bgnn
from bgnn import synthetic as S
from oracle import pyg_ref as P

REF = "/root/reference"


def test_mesh_config_sizes_match_survey():
    # per-graph node/edge counts of cfg1/cfg2/cfg3
    g1 = S.make_mesh_graph(45, 0)
    assert (g1.num_nodes, g1.num_edges) == (2025, 17752)
    g2 = S.make_mesh_graph(71, 0)
    assert (g2.num_nodes, g2.num_edges) == (5041, 44742)
    g3 = S.make_mesh_graph(71, 0, super_node=True)
    assert (g3.num_nodes, g3.num_edges) == (5042, 49562)


def test_mesh_graph_structure():
    g = S.make_mesh_graph(6, 3)
    ei = g.edge_index.numpy()
    # both directions, interleaved (GraphCreate.py:420-422)
    assert np.array_equal(ei[0, 0::2], ei[1, 1::2]) and np.array_equal(ei[1, 0::2], ei[0, 1::2])
    pairs = {tuple(sorted(p)) for p in ei.T.tolist()}
    assert len(pairs) * 2 == ei.shape[1]            # no duplicate undirected edges
    assert all(a != b for a, b in pairs)            # no self loops
    assert g.x.shape == (36, 16) and float(g.x[:, -1].abs().sum()) == 0.0
    assert g.edge_attr.shape == (ei.shape[1], 5)
    gs = S.make_mesh_graph(6, 3, super_node=True)
    s = gs.num_nodes - 1
    deg_s = int((gs.edge_index[1] == s).sum())
    assert deg_s == 36 and float(gs.x[s, -1]) == 1.0


def test_batch_collation_matches_oracle():
    ds = [S.make_mesh_graph(n, seed) for n, seed in ((4, 1), (5, 2), (3, 3))]
    b = bgnn.Batch.from_data_list(ds)
    ref = P.collate([{"x": d.x, "edge_index": d.edge_index, "edge_attr": d.edge_attr, "y": d.y} for d in ds])
    for k in ("x", "edge_index", "edge_attr", "y", "batch"):
        assert torch.equal(getattr(b, k), ref[k]), k
    assert b.num_graphs == 3 and b.ptr.tolist() == [0, 16, 41, 50]
    assert b.num_node_features == 16 and b.num_edge_features == 5
    loader = bgnn.DataLoader(ds, batch_size=2, shuffle=False)
    batches = list(loader)
    assert [bb.num_graphs for bb in batches] == [2, 1]


def test_data_attributes_and_clone():
    d = bgnn.Data(x=torch.zeros(3, 2), edge_index=torch.tensor([[0], [1]]), file_path="a.bdf",
                  mode_shapes=torch.ones(3, 3))
    c = d.clone()
    c.x[0, 0] = 5
    assert float(d.x[0, 0]) == 0.0
    assert d.file_path == "a.bdf" and d.num_nodes == 3 and d.edge_attr is None
    b = bgnn.Batch.from_data_list([d, d])
    assert b.file_path == ["a.bdf", "a.bdf"] and b.mode_shapes.shape == (6, 3)


@pytest.mark.parametrize("fn", [
    lambda: bgnn.aggregate(torch.zeros(3, 4), None),
    lambda: bgnn.Graph.build(torch.zeros(2, 3, dtype=torch.long), 3),
    lambda: bgnn.SAGEConv(4, 4, aggr="sum")(torch.zeros(3, 4), torch.zeros(2, 3, dtype=torch.long)),
    lambda: bgnn.global_mean_pool(torch.zeros(3, 4), torch.zeros(3, dtype=torch.long)),
])
def test_no_cpu_fallback(fn):
    with pytest.raises((RuntimeError, AttributeError)):
        fn()


VARIANTS = ["GraphSage_addAggr", "GraphSage_sumAggr", "GraphSage_meanAggr", "GraphSage_maxAggr",
            "GraphSage_addAggr_Shared", "EA_GNN", "EA_GNN_Shared", "GraphSAGE_MLP", "GraphSAGE_SAG", "EAGNN_SAG"]


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference not present")
@pytest.mark.parametrize("hidden", [64, 512])
@pytest.mark.parametrize("name", VARIANTS)
def test_state_dict_layout_matches_reference(name, hidden):
    """The reference's BuckGNN (imported unchanged through bgnn's PyG shim) and bgnn.BuckGNN
    have identical state-dict keys and shapes, so checkpoints load both ways."""
    bgnn.install_pyg_shim(batchnorm=False, fused_model=False)
    sys.path.insert(0, REF)
    try:
        from Models.BuckGNN import BuckGNN as RefBuckGNN
    finally:
        sys.path.remove(REF)
    kw = dict(hidden_channels=hidden, num_layers=6, pooling_layer="mean", dropout_rate=0.1, model_name=name)
    ref = RefBuckGNN(16, 5, **kw).state_dict()
    mine = bgnn.BuckGNN(16, 5, **kw).state_dict()
    assert list(ref.keys()) == list(mine.keys())
    for k in ref:
        assert ref[k].shape == mine[k].shape, k
    bgnn.BuckGNN(16, 5, **kw).load_state_dict(ref)
    bgnn.uninstall_pyg_shim()


def test_reference_defects_reproduced():
    m = bgnn.BuckGNN(16, 5, hidden_channels=64, model_name="GraphSage_MLP")
    with pytest.raises(AttributeError):
        m(torch.zeros(4, 16), torch.zeros(2, 0, dtype=torch.long), None)
    # hidden in (128, 256): no encoder is built (Models/BuckGNN.py:41,67)
    m2 = bgnn.BuckGNN(16, 5, hidden_channels=192, model_name="GraphSage_addAggr")
    assert not hasattr(m2, "node_encoder")


def test_super_node_index_vectorised():
    from bgnn.buckgnn import super_node_index
    from oracle.buckgnn_ref import super_index

    b = torch.tensor([0, 0, 0, 1, 1, 2, 2, 2, 2])
    assert super_node_index(b, 9, "cpu").tolist() == super_index(b, 9).tolist() == [2, 4, 8]
    assert super_node_index(None, 5, "cpu").tolist() == [4]


def test_graph_store_requires_gpu():
    """GraphStore lives in HBM: a CPU device is rejected (no CPU fallback)."""
    import bgnn
    from bgnn import synthetic as S
    with pytest.raises(RuntimeError):
        bgnn.GraphStore([S.make_mesh_graph(5, seed=0)], device="cpu")


def test_column_blocks_backward_is_one_concat():
    """bgnn.ea._ColumnBlocks: the k column views of P, with an unused block's gradient zero."""
    from bgnn.ea import _ColumnBlocks
    P = torch.randn(7, 12, dtype=torch.float64, requires_grad=True)
    a, b, c = _ColumnBlocks.apply(P, 3)
    assert torch.equal(torch.cat([a, b, c], 1), P.detach())
    w = torch.randn(7, 4, dtype=torch.float64)
    ((a * w).sum() + (c * 2 * w).sum()).backward()
    assert torch.equal(P.grad, torch.cat([w, torch.zeros_like(w), 2 * w], 1))


def test_column_blocks_unused_blocks_get_no_buffers():
    """An unused block's gradient arrives as None (no materialized zeros); the only used block
    still yields the full-width gradient, and P gets no gradient through unused outputs."""
    from bgnn.ea import _ColumnBlocks
    P = torch.randn(5, 9, dtype=torch.float64, requires_grad=True)
    a, b, c = _ColumnBlocks.apply(P, 3)
    (3 * b).sum().backward()
    assert torch.equal(P.grad, torch.cat([torch.zeros(5, 3), torch.full((5, 3), 3.0), torch.zeros(5, 3)], 1).double())
    # every block unused by the loss: backward returns None for P (no StopIteration)
    Q = torch.randn(4, 6, requires_grad=True)
    x, y = _ColumnBlocks.apply(Q, 2)
    z = torch.randn(1, requires_grad=True)
    (z * 2).sum().backward(inputs=[z])
    out = _ColumnBlocks.backward(type("Ctx", (), {"k": 2, "cg": None})(), None, None)
    assert out == (None, None, None)


def test_column_blocks_shared_buffer_returned_without_copy():
    """EA_GNN's ColGrad: when every block's gradient is that block of the shared buffer, the
    backward hands the buffer on (no concatenation); otherwise it concatenates."""
    from bgnn.ea import ColGrad, _ColumnBlocks
    cg = ColGrad((4, 6), torch.device("cpu"))
    b0, b1 = cg.block(0, 3), cg.block(1, 3)
    b0.fill_(1.0)
    b1.fill_(2.0)
    buf = cg.buf
    out = _ColumnBlocks.backward(type("Ctx", (), {"k": 2, "cg": cg})(), b0, b1)
    assert out[0] is buf and cg.buf is None
    cg2 = ColGrad((4, 6), torch.device("cpu"))
    g0 = cg2.block(0, 3)
    g1 = torch.full((4, 3), 5.0)   # not the buffer's block: concatenated
    out = _ColumnBlocks.backward(type("Ctx", (), {"k": 2, "cg": cg2})(), g0, g1)
    assert out[0] is not cg2.buf and torch.equal(out[0][:, 3:], g1)


def test_relu_mask_matches_reference_form():
    """threshold_backward (the backward ReLU mask of bgnn.ea / bgnn.fused) == g * (out > 0)."""
    g, out = torch.randn(64, 33), torch.randn(64, 33)
    out[0, :5] = 0.0
    assert torch.equal(torch.ops.aten.threshold_backward(g, out, 0.0), g * (out > 0))


def test_pyg_shim_batchnorm_patches_and_restores():
    """install_pyg_shim() (batchnorm=True, the default since round 5) makes torch.nn.BatchNorm1d
    bgnn's subclass (same state-dict keys) for modules built while it is installed; uninstall
    restores torch's class."""
    import torch
    import bgnn
    from bgnn import nn as bnn
    orig = torch.nn.BatchNorm1d
    bgnn.install_pyg_shim(batchnorm=True)
    try:
        assert torch.nn.BatchNorm1d is bnn.BatchNorm1d
        m = torch.nn.BatchNorm1d(8)
        assert isinstance(m, orig) and set(m.state_dict()) == set(orig(8).state_dict())
        y = m(torch.randn(4, 8))   # CPU input: torch's own forward
        assert y.shape == (4, 8)
    finally:
        bgnn.uninstall_pyg_shim()
    assert torch.nn.BatchNorm1d is orig


@pytest.mark.skipif(not os.path.isdir(REF), reason="needs the reference checkout")
def test_pyg_shim_binds_fused_model_class():
    """install_pyg_shim()'s import hook: the reference's unchanged Models/BuckGNN.py, imported the way
    TRAIN_FINAL.py / INFERENCE.py import it, exports bgnn.BuckGNN as BuckGNN (same constructor and
    state-dict keys as the reference class, kept as BuckGNN_reference); a module imported before the
    shim is rebound in place; uninstall restores the reference class."""
    for k in [k for k in sys.modules if k == "Models" or k.startswith("Models.")]:
        del sys.modules[k]
    sys.path.insert(0, REF)
    try:
        bgnn.install_pyg_shim(batchnorm=False)
        try:
            from Models.BuckGNN import BuckGNN
            import Models.BuckGNN as M
            assert BuckGNN is bgnn.BuckGNN and M.BuckGNN is bgnn.BuckGNN
            ref_cls = M.BuckGNN_reference
            assert ref_cls is not bgnn.BuckGNN and ref_cls.__module__ == "Models.BuckGNN"
            kw = dict(hidden_channels=64, num_layers=6, pooling_layer="mean", dropout_rate=0.1,
                      model_name="GraphSage_addAggr_Shared")
            ours, ref = BuckGNN(16, 5, **kw), ref_cls(16, 5, **kw)
            assert list(ours.state_dict()) == list(ref.state_dict())
            ours.load_state_dict(ref.state_dict())   # a reference checkpoint loads unchanged (strict)
        finally:
            bgnn.uninstall_pyg_shim()
        assert M.BuckGNN is ref_cls
        # imported first (with the shim's PyG modules but without the hook), then rebound in place
        bgnn.install_pyg_shim(batchnorm=False, fused_model=False)
        assert sys.modules["Models.BuckGNN"].BuckGNN is ref_cls
        bgnn.uninstall_pyg_shim()
        bgnn.install_pyg_shim(batchnorm=False)
        try:
            assert sys.modules["Models.BuckGNN"].BuckGNN is bgnn.BuckGNN
        finally:
            bgnn.uninstall_pyg_shim()
        assert sys.modules["Models.BuckGNN"].BuckGNN is ref_cls
    finally:
        sys.path.remove(REF)
        for k in [k for k in sys.modules if k == "Models" or k.startswith("Models.")]:
            del sys.modules[k]
