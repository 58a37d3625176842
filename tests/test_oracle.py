"""Pin the oracle (CPU restatement) before trusting it:
1. hand-derived known-answer tests of PyG's SAGEConv / pooling / scatter formula;
2. golden vectors produced by the reference's own Models/BuckGNN.py (tests/golden).
CPU only."""
import glob
import os

import numpy as np
import pytest
import torch

from oracle import buckgnn_ref as R
from oracle import pyg_ref as P
from recipe import grad_checksum, make_weights, meta_from_array

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


# --------------------------------------------------------------------------- KATs
def path_graph():
    # 0 -> 1 -> 2 and 2 -> 1 ; node 0 has no in-edges
    return torch.tensor([[0, 1, 2], [1, 2, 1]])


def test_kat_sum_mean_max_on_path_graph():
    x = torch.tensor([[1.0, -2.0], [3.0, 4.0], [-5.0, 6.0]])
    ei = path_graph()
    s = P.sage_aggregate(x, ei, "sum")
    m = P.sage_aggregate(x, ei, "mean")
    mx = P.sage_aggregate(x, ei, "max")
    # target 1 receives x0 + x2, target 2 receives x1, target 0 nothing
    assert torch.equal(s, torch.tensor([[0.0, 0.0], [-4.0, 4.0], [3.0, 4.0]]))
    assert torch.equal(m, torch.tensor([[0.0, 0.0], [-2.0, 2.0], [3.0, 4.0]]))
    assert torch.equal(mx, torch.tensor([[0.0, 0.0], [1.0, 6.0], [3.0, 4.0]]))
    assert torch.equal(P.sage_aggregate(x, ei, "add"), s)


def test_kat_max_ties_first_occurrence_gets_gradient():
    """Tie convention of max aggregation (oracle/pyg_ref._ScatterMaxFirst): the first edge in
    edge_index order that attains the maximum of its (target, column) takes the whole gradient
    (torch_scatter's argmax form; ReLU zeros tie in practice). Targets: 0 <- {1, 2, 3},
    1 <- {2, 0}; node 2 has no in-edges."""
    x = torch.tensor([[0.0, 5.0], [0.0, 1.0], [0.0, 5.0], [-1.0, 5.0]], requires_grad=True)
    ei = torch.tensor([[1, 2, 3, 2, 0], [0, 0, 0, 1, 1]])
    out = P.sage_aggregate(x, ei, "max")
    assert torch.equal(out.detach(), torch.tensor([[0.0, 5.0], [0.0, 5.0], [0.0, 0.0], [0.0, 0.0]]))
    g = torch.tensor([[1.0, 10.0], [100.0, 1000.0], [7.0, 7.0], [9.0, 9.0]])
    out.backward(g)
    # target 0: column 0 ties at 0 between sources 1 and 2 -> source 1 (first edge); column 1
    # ties at 5 between sources 2 and 3 -> source 2. Target 1: both columns tie between sources
    # 2 and 0 -> source 2 (the first edge, although node 0 has the lower index)
    exp = torch.tensor([[0.0, 0.0], [1.0, 0.0], [100.0, 10.0 + 1000.0], [0.0, 0.0]])
    assert torch.equal(x.grad, exp)


def test_kat_duplicate_edges_count_twice_and_self_loops():
    x = torch.tensor([[1.0], [10.0]])
    ei = torch.tensor([[1, 1, 0], [0, 0, 0]])   # 1->0 twice, self loop 0->0
    assert torch.equal(P.sage_aggregate(x, ei, "sum"), torch.tensor([[21.0], [0.0]]))
    assert torch.equal(P.sage_aggregate(x, ei, "mean"), torch.tensor([[7.0], [0.0]]))


def test_kat_sageconv_identity_weights_and_normalize():
    conv = P.SAGEConv(2, 2, aggr="sum", normalize=True)
    with torch.no_grad():
        conv.lin_l.weight.copy_(torch.eye(2))
        conv.lin_l.bias.zero_()
        conv.lin_r.weight.copy_(2 * torch.eye(2))
    x = torch.tensor([[3.0, 0.0], [0.0, 4.0], [0.0, 0.0]])
    ei = torch.tensor([[0, 1], [1, 0]])
    out = conv(x, ei)
    # node0: agg = x1 = (0,4) + 2*x0 = (6,4) -> /|.|; node2: zero row -> normalize gives 0
    exp0 = torch.tensor([6.0, 4.0]) / np.sqrt(52.0)
    exp1 = torch.tensor([3.0, 8.0]) / np.sqrt(73.0)
    assert torch.allclose(out[0], exp0, atol=1e-7)
    assert torch.allclose(out[1], exp1, atol=1e-7)
    assert torch.equal(out[2], torch.zeros(2))
    assert set(conv.state_dict()) == {"lin_l.weight", "lin_l.bias", "lin_r.weight"}


def test_kat_pools_and_scatter():
    x = torch.tensor([[1.0], [3.0], [5.0], [7.0]])
    b = torch.tensor([0, 0, 2, 2])
    assert torch.equal(P.global_mean_pool(x, b), torch.tensor([[2.0], [0.0], [6.0]]))
    assert torch.equal(P.global_add_pool(x, b), torch.tensor([[4.0], [0.0], [12.0]]))
    assert torch.equal(P.global_max_pool(x, b), torch.tensor([[3.0], [0.0], [7.0]]))
    assert torch.equal(P.global_mean_pool(x, None), torch.tensor([[4.0]]))
    assert torch.equal(P.scatter_mean(x, b, dim_size=4), torch.tensor([[2.0], [0.0], [6.0], [0.0]]))


def test_collate_offsets_edge_index():
    g1 = {"x": np.zeros((2, 1)), "edge_index": np.array([[0], [1]]), "y": np.array([1.0])}
    g2 = {"x": np.zeros((3, 1)), "edge_index": np.array([[2], [0]]), "y": np.array([2.0])}
    b = P.collate([g1, g2])
    assert b["edge_index"].tolist() == [[0, 4], [1, 2]]
    assert b["batch"].tolist() == [0, 0, 1, 1, 1]


# --------------------------------------------------------------------------- golden
def golden_files():
    return sorted(glob.glob(os.path.join(GOLDEN, "*.npz")))


def load_case(path):
    z = np.load(path)
    meta = meta_from_array(z["meta"])
    return z, meta


def oracle_state(meta, keys_shapes):
    return {k: torch.from_numpy(v) for k, v in make_weights(keys_shapes, meta["weight_seed"]).items()}


def reference_shapes(meta):
    """State-dict shapes the reference model has, derived from bgnn.BuckGNN (same layout, checked
    against the reference class itself in test_host.py)."""
    import bgnn
    m = bgnn.BuckGNN(16, 5, hidden_channels=meta["hidden"], num_layers=meta["num_layers"],
                     pooling_layer=meta["pooling"], dropout_rate=0.0, model_name=meta["model_name"])
    return {k: tuple(v.shape) for k, v in m.state_dict().items()}


def _is_sag(p):
    return os.path.basename(p).startswith(("sag_", "eagnn_sag"))


@pytest.mark.parametrize("path", [p for p in golden_files() if "ea_gnn" not in p and not _is_sag(p)],
                         ids=os.path.basename)
def test_oracle_matches_reference_golden(path):
    z, meta = load_case(path)
    sd = oracle_state(meta, reference_shapes(meta))
    x = torch.from_numpy(z["x"])
    ei = torch.from_numpy(z["edge_index"])
    batch = None if meta["single_graph"] else torch.from_numpy(z["batch"])
    y = torch.from_numpy(z["y"])
    if meta["single_graph"]:
        y = y[0]
    step = {k: v.clone().requires_grad_(v.is_floating_point() and "running" not in k) for k, v in sd.items()}
    pred = R.forward(step, meta["model_name"], x, ei, batch, True, meta["pooling"], 0.0)
    loss = R.relative_error_loss(pred, y)
    loss.backward()
    tol = 2e-5 if meta["hidden"] <= 64 else 1e-4
    np.testing.assert_allclose(pred.detach().numpy().reshape(-1), z["pred_train"], rtol=tol, atol=tol)
    np.testing.assert_allclose(loss.item(), float(z["loss_train"]), rtol=tol, atol=tol)
    for k in z.files:
        if k.startswith("grad/"):
            g = step[k[5:]].grad
            assert g is not None, k
            np.testing.assert_allclose(g.numpy(), z[k], rtol=1e-4, atol=1e-5, err_msg=k)
        elif k.startswith("gradsum/"):
            g = step[k[8:]].grad
            assert g is not None, k
            np.testing.assert_allclose(grad_checksum(g.numpy()), z[k], rtol=1e-3, atol=1e-4, err_msg=k)
        elif k.startswith("state/"):
            np.testing.assert_allclose(step[k[6:]].detach().numpy(), z[k], rtol=1e-5, atol=1e-6, err_msg=k)
    with torch.no_grad():
        pe = R.forward(step, meta["model_name"], x, ei, batch, False, meta["pooling"], 0.0)
    np.testing.assert_allclose(pe.numpy().reshape(-1), z["pred_eval"], rtol=tol, atol=tol)


@pytest.mark.parametrize("path", [p for p in golden_files() if "ea_gnn" in p], ids=os.path.basename)
def test_ea_oracle_matches_reference_golden(path):
    """oracle.buckgnn_ref.ea_forward (EA_GNN, Models/BuckGNN.py:375-387,528-566) against the
    golden vectors of the reference's own EA_GNN: prediction, loss, every gradient."""
    z, meta = load_case(path)
    assert meta["model_name"] in ("EA_GNN", "EA_GNN_Shared")
    shared = meta["model_name"] == "EA_GNN_Shared"
    sd = oracle_state(meta, reference_shapes(meta))
    x = torch.from_numpy(z["x"])
    ei = torch.from_numpy(z["edge_index"])
    ea = torch.from_numpy(z["edge_attr"])
    batch = torch.from_numpy(z["batch"])
    y = torch.from_numpy(z["y"])
    step = {k: v.clone().requires_grad_(v.is_floating_point() and "running" not in k) for k, v in sd.items()}
    pred = R.ea_forward(step, x, ei, ea, batch, True, 0.0, meta["num_layers"], shared)
    loss = R.relative_error_loss(pred, y)
    loss.backward()
    np.testing.assert_allclose(pred.detach().numpy().reshape(-1), z["pred_train"], rtol=2e-5, atol=2e-5)
    np.testing.assert_allclose(loss.item(), float(z["loss_train"]), rtol=2e-5, atol=2e-5)
    n = 0
    for k in z.files:
        if k.startswith("grad/"):
            np.testing.assert_allclose(step[k[5:]].grad.numpy(), z[k], rtol=1e-4, atol=1e-5, err_msg=k)
            n += 1
        elif k.startswith("gradsum/"):
            np.testing.assert_allclose(grad_checksum(step[k[8:]].grad.numpy()), z[k], rtol=1e-3, atol=1e-4, err_msg=k)
            n += 1
    assert n > 0
    with torch.no_grad():
        pe = R.ea_forward(step, x, ei, ea, batch, False, 0.0, meta["num_layers"], shared)
    np.testing.assert_allclose(pe.numpy().reshape(-1), z["pred_eval"], rtol=2e-5, atol=2e-5)


@pytest.mark.parametrize("path", [p for p in golden_files() if _is_sag(p)], ids=os.path.basename)
def test_sag_oracle_matches_reference_golden(path):
    """oracle.buckgnn_ref.sag_forward (GraphSAGE_SAG / EAGNN_SAG with SAGPooling,
    Models/BuckGNN.py:190-244,354-373,493-511) against the golden vectors of the reference's own
    model: the pooled node selection (perm, scores), prediction, loss, gradients, BN state."""
    z, meta = load_case(path)
    sd = oracle_state(meta, reference_shapes(meta))
    x = torch.from_numpy(z["x"])
    ei = torch.from_numpy(z["edge_index"])
    ea = torch.from_numpy(z["edge_attr"])
    batch = None if meta["single_graph"] else torch.from_numpy(z["batch"])
    y = torch.from_numpy(z["y"])
    if meta["single_graph"]:
        y = y[0]
    step = {k: v.clone().requires_grad_(v.is_floating_point() and "running" not in k) for k, v in sd.items()}
    pred, perm = R.sag_forward(step, meta["model_name"], x, ei, ea, batch, True, 0.0, meta["num_layers"])
    np.testing.assert_array_equal(perm.numpy(), z["pool_perm"])
    loss = R.relative_error_loss(pred, y)
    loss.backward()
    np.testing.assert_allclose(pred.detach().numpy().reshape(-1), z["pred_train"], rtol=2e-5, atol=2e-5)
    np.testing.assert_allclose(loss.item(), float(z["loss_train"]), rtol=2e-5, atol=2e-5)
    n = 0
    for k in z.files:
        if k.startswith("grad/"):
            np.testing.assert_allclose(step[k[5:]].grad.numpy(), z[k], rtol=1e-4, atol=1e-5, err_msg=k)
            n += 1
        elif k.startswith("gradsum/"):
            np.testing.assert_allclose(grad_checksum(step[k[8:]].grad.numpy()), z[k], rtol=1e-3, atol=1e-4,
                                       err_msg=k)
            n += 1
        elif k.startswith("state/"):
            np.testing.assert_allclose(step[k[6:]].detach().numpy(), z[k], rtol=1e-5, atol=1e-6, err_msg=k)
    assert n > 0
    with torch.no_grad():
        pe, _ = R.sag_forward(step, meta["model_name"], x, ei, ea, batch, False, 0.0, meta["num_layers"])
    np.testing.assert_allclose(pe.numpy().reshape(-1), z["pred_eval"], rtol=2e-5, atol=2e-5)


def test_kat_topk_and_filter_adj():
    """Hand-derived known answers for PyG's topk / filter_adj (ratio 0.5: ceil(n/2) per graph,
    descending, ties to the lower index; kept edges in order, relabelled)."""
    from oracle.pyg_ref import filter_adj, topk
    score = torch.tensor([0.1, 0.9, 0.5, 0.5, -1.0, 0.3, 0.3, 0.3])
    batch = torch.tensor([0, 0, 0, 0, 0, 1, 1, 1])
    perm = topk(score, 0.5, batch)
    assert perm.tolist() == [1, 2, 3, 5, 6]    # graph 0: k=3 of 5; graph 1: k=2 of 3 (ties)
    ei = torch.tensor([[1, 2, 0, 3, 5, 6, 7], [2, 1, 1, 5, 6, 5, 5]])
    ea = torch.arange(7.0).view(7, 1)
    e2, a2 = filter_adj(ei, ea, perm, 8)
    assert e2.tolist() == [[0, 1, 2, 3, 4], [1, 0, 3, 4, 3]]
    assert a2.view(-1).tolist() == [0.0, 1.0, 3.0, 4.0, 5.0]
