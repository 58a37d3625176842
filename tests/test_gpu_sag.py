"""GPU: SAGPooling (GraphSAGE_SAG / EAGNN_SAG, Models/BuckGNN.py:190-244,354-373,493-511) on
the bgnn kernels (bgnn_topk_rank / _select, bgnn_gather_scale / _bwd, bgnn_filter_edges)
against the oracle's restatement of PyG's topk / filter_adj / SAGPooling (oracle/pyg_ref.py).

Whole-model parity of the SAG variants against the reference's own golden vectors runs in
test_gpu_model.py (sag_*.npz, eagnn_sag_h64.npz); here: the selected nodes of those
fixtures, the ops one by one (bit-exact for the integer work), edge cases (ties, one-node
graphs, ratio >= 1, no kept edges), and a cfg-sized pooled model against the oracle."""
import os

import numpy as np
import pytest
import torch

import bgnn
from bgnn import pool as P
from bgnn import synthetic as S
from bgnn.data import Batch
from oracle import buckgnn_ref as R
from oracle import pyg_ref
from recipe import make_weights, meta_from_array

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _batch_of(sizes):
    return torch.cat([torch.full((n,), g, dtype=torch.long) for g, n in enumerate(sizes)])


@pytest.mark.parametrize("sizes,levels", [([5, 3, 1, 8], 0), ([5041, 5041, 2000, 1], 0), ([700, 300], 4),
                                          ([1], 0), ([4096 + 17], 3)])
@pytest.mark.parametrize("ratio", [0.5, 0.3, 2])
def test_topk_select_matches_oracle(dev, sizes, levels, ratio):
    """perm bit-exact vs oracle topk (stable sorts), incl. heavy ties (scores on a few levels,
    +0.0 / -0.0 equal), one-node graphs, graphs larger than one LDS tile."""
    g = torch.Generator().manual_seed(sum(sizes) + levels)
    batch = _batch_of(sizes)
    score = torch.rand(batch.numel(), generator=g) * 2 - 1
    if levels:
        score = torch.round(score * levels) / levels
        score[score == 0] = torch.where(torch.rand((score == 0).sum(), generator=g) < 0.5, 0.0, -0.0)
    perm, new_id, b_out = P.topk_select(score.to(dev), ratio, batch.to(dev))
    ref = pyg_ref.topk(score, ratio, batch) if ratio < 1 else _topk_int(score, int(ratio), batch)
    np.testing.assert_array_equal(perm.cpu().numpy(), ref.numpy())
    np.testing.assert_array_equal(b_out.cpu().numpy(), batch[ref].numpy())
    nid = torch.full((batch.numel(),), -1, dtype=torch.int32)
    nid[ref] = torch.arange(ref.numel(), dtype=torch.int32)
    np.testing.assert_array_equal(new_id.cpu().numpy(), nid.numpy())


def _topk_int(score, k, batch):
    """ratio >= 1: min(k, n_g) nodes per graph (PyG's integer-ratio form), same order rules."""
    out = []
    for gi in range(int(batch.max()) + 1):
        idx = torch.nonzero(batch == gi).flatten()
        _, o = torch.sort(score[idx], descending=True, stable=True)
        out.append(idx[o[:min(k, idx.numel())]])
    return torch.cat(out)


def test_topk_rejects_unsorted_batch(dev):
    with pytest.raises(ValueError):
        P.topk_select(torch.rand(4, device=dev), 0.5, torch.tensor([0, 1, 0, 1], device=dev))


@pytest.mark.parametrize("n,super_node", [(9, False), (30, True), (71, False)])
def test_filter_edges_matches_oracle(dev, n, super_node):
    """edge_index' and edge_attr' bit-exact vs oracle filter_adj on mesh batches (mesh + virtual
    or super-node edges; 1024-edge blocks, several scan slices at n = 71)."""
    b = Batch.from_data_list([S.make_mesh_graph(n, s, super_node=super_node) for s in range(3)])
    torch.manual_seed(n)
    score = torch.rand(b.num_nodes)
    perm = pyg_ref.topk(score, 0.5, b.batch)
    ei_ref, ea_ref = pyg_ref.filter_adj(b.edge_index, b.edge_attr, perm, b.num_nodes)
    _, new_id, _ = P.topk_select(score.to(dev), 0.5, b.batch.to(dev))
    ei, kept = P.filter_edges(b.edge_index.to(dev), new_id, b.num_nodes)
    np.testing.assert_array_equal(ei.cpu().numpy(), ei_ref.numpy())
    np.testing.assert_array_equal(b.edge_attr[kept.cpu()].numpy(), ea_ref.numpy())
    assert ei.is_contiguous()


def test_filter_edges_empty_and_none_kept(dev):
    new_id = torch.tensor([-1, 0, -1], dtype=torch.int32, device=dev)
    ei, kept = P.filter_edges(torch.tensor([[0, 1, 2], [1, 2, 0]], device=dev), new_id, 3)
    assert ei.shape == (2, 0) and kept.numel() == 0
    ei, kept = P.filter_edges(torch.zeros(2, 0, dtype=torch.long, device=dev), new_id, 3)
    assert ei.shape == (2, 0)


@pytest.mark.parametrize("H", [512, 64, 5])
def test_gather_scale_fwd_bwd(dev, H):
    """x[perm] * score[perm] and its backward vs torch autograd on the CPU: forward and dx
    bit-exact (one product each), dscore to fp32 summation order."""
    torch.manual_seed(H)
    N = 3000
    batch = _batch_of([1000, 1500, 500])
    x = torch.randn(N, H)
    score = torch.rand(N) * 2 - 1
    perm = pyg_ref.topk(score, 0.5, batch)
    xd = x.to(dev).requires_grad_(True)
    sd = score.to(dev).requires_grad_(True)
    perm_d, new_id, _ = P.topk_select(sd.detach(), 0.5, batch.to(dev))
    out = P.gather_scale(xd, sd, perm_d, new_id)
    g = torch.randn(out.shape)
    out.backward(g.to(dev))
    xc = x.clone().requires_grad_(True)
    sc = score.clone().requires_grad_(True)
    oc = xc[perm] * sc[perm].view(-1, 1)
    oc.backward(g)
    np.testing.assert_array_equal(out.detach().cpu().numpy(), oc.detach().numpy())
    np.testing.assert_array_equal(xd.grad.cpu().numpy(), xc.grad.numpy())
    np.testing.assert_allclose(sd.grad.cpu().numpy(), sc.grad.numpy(), rtol=1e-5, atol=1e-5 * np.sqrt(H))


def _pool_pair(h, seed):
    torch.manual_seed(seed)
    ref = pyg_ref.SAGPooling(h, ratio=0.5, GNN=pyg_ref.SAGEConv, aggr="add")
    mine = bgnn.SAGPooling(h, ratio=0.5, GNN=bgnn.SAGEConv, aggr="add")
    mine.load_state_dict(ref.state_dict())
    return ref, mine


@pytest.mark.parametrize("h,super_node", [(64, False), (512, True)])
def test_sag_pooling_module_matches_oracle(dev, h, super_node):
    """bgnn.SAGPooling vs the oracle's SAGPooling on a 4-graph mesh batch: all six outputs
    and the gradients of x and of the scoring GNN's parameters."""
    b = Batch.from_data_list([S.make_mesh_graph(12, s, super_node=super_node) for s in range(4)])
    ref, mine = _pool_pair(h, h)
    mine = mine.to(dev)
    torch.manual_seed(1)
    x = torch.randn(b.num_nodes, h)
    xr = x.clone().requires_grad_(True)
    xm = x.to(dev).requires_grad_(True)
    o_ref = ref(xr, b.edge_index, b.edge_attr, b.batch)
    o = mine(xm, b.edge_index.to(dev), b.edge_attr.to(dev), b.batch.to(dev))
    np.testing.assert_array_equal(o[4].cpu().numpy(), o_ref[4].numpy())            # perm
    np.testing.assert_array_equal(o[1].cpu().numpy(), o_ref[1].numpy())            # edge_index'
    np.testing.assert_array_equal(o[2].cpu().numpy(), o_ref[2].numpy())            # edge_attr'
    np.testing.assert_array_equal(o[3].cpu().numpy(), o_ref[3].numpy())            # batch'
    np.testing.assert_allclose(o[5].detach().cpu().numpy(), o_ref[5].detach().numpy(), rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(o[0].detach().cpu().numpy(), o_ref[0].detach().numpy(), rtol=1e-4, atol=1e-5)
    gy = torch.randn(o_ref[0].shape)
    (o_ref[0] * gy).sum().backward()
    (o[0] * gy.to(dev)).sum().backward()
    np.testing.assert_allclose(xm.grad.cpu().numpy(), xr.grad.numpy(), rtol=1e-4, atol=1e-5)
    # the scorer's weight gradients are sums over all nodes (|g| up to ~2e3 at h = 512) and the
    # GPU scorer is transform-first: elements that cancel are compared at 2e-6 of the tensor's max
    pr = dict(ref.named_parameters())
    for k, p in mine.named_parameters():
        if k == "select.weight":   # d tanh(attn * w / |w|) / dw = 0 exactly: both sides hold rounding noise
            continue
        r = pr[k].grad.numpy()
        np.testing.assert_allclose(p.grad.cpu().numpy(), r, rtol=1e-4, atol=max(1e-5, 2e-6 * np.abs(r).max()),
                                   err_msg=k)


def test_sag_pooling_loads_checkpoint_without_select_weight(dev):
    """Checkpoints of PyG releases whose SAGPooling has no select projection load with w = 1."""
    _, mine = _pool_pair(16, 0)
    sd = {k: v for k, v in mine.state_dict().items() if not k.startswith("select.")}
    mine.load_state_dict(sd)
    assert float(mine.select.weight) == 1.0


@pytest.mark.parametrize("name", ["sag_h64", "sag_super_h64", "sag_single_h64", "eagnn_sag_h64"])
def test_sag_model_selects_reference_nodes(dev, name):
    """The reference model's own pooled node selection (golden pool_perm / pool_score)."""
    z = np.load(os.path.join(GOLDEN, name + ".npz"))
    meta = meta_from_array(z["meta"])
    m = bgnn.BuckGNN(16, 5, hidden_channels=meta["hidden"], num_layers=meta["num_layers"],
                     pooling_layer=meta["pooling"], dropout_rate=0.0, model_name=meta["model_name"])
    sd = m.state_dict()
    w = make_weights({k: tuple(v.shape) for k, v in sd.items()}, meta["weight_seed"])
    m.load_state_dict({k: torch.from_numpy(w[k]) if k in w else sd[k] for k in sd})
    m = m.to(dev).train()
    got = {}
    m.pool.register_forward_hook(lambda mod, inp, o: got.update(perm=o[4], score=o[5], ne=o[1].size(1)))
    batch = None if meta["single_graph"] else torch.from_numpy(z["batch"]).to(dev)
    m(torch.from_numpy(z["x"]).to(dev), torch.from_numpy(z["edge_index"]).to(dev),
      torch.from_numpy(z["edge_attr"]).to(dev), batch)
    np.testing.assert_array_equal(got["perm"].cpu().numpy(), z["pool_perm"])
    np.testing.assert_allclose(got["score"].detach().cpu().numpy(), z["pool_score"], rtol=1e-4, atol=1e-5)
    assert got["ne"] == int(z["pool_edges"])


def test_sag_model_cfg2_sized_matches_oracle(dev, monkeypatch):
    """GraphSAGE_SAG at h = 512 on 4 cfg2 meshes (20,164 nodes, the fused layers with the
    folded encoder): eval prediction vs the oracle within 1e-4; the pooled node set of every
    graph is the oracle's topk of the scores the GPU computed (ordering is checked bit-exact
    on those scores)."""
    b = Batch.from_data_list([S.make_mesh_graph(71, s) for s in range(4)])
    torch.manual_seed(0)
    m = bgnn.BuckGNN(16, 5, hidden_channels=512, num_layers=6, pooling_layer="mean", dropout_rate=0.0,
                     model_name="GraphSAGE_SAG")
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    m = m.to(dev).eval()
    got = {}
    m.pool.register_forward_hook(lambda mod, inp, o: got.update(perm=o[4]))
    scores = {}
    topk_select = P.topk_select

    def spy(score, ratio, batch):
        scores["s"] = score.detach().cpu()
        return topk_select(score, ratio, batch)
    monkeypatch.setattr(P, "topk_select", spy)
    with torch.no_grad():
        pred, _ = m(b.x.to(dev), b.edge_index.to(dev), b.edge_attr.to(dev), b.batch.to(dev))
        ref, ref_perm = R.sag_forward(sd, "GraphSAGE_SAG", b.x, b.edge_index, b.edge_attr, b.batch, False)
    np.testing.assert_allclose(pred.cpu().numpy(), ref.numpy(), rtol=1e-4, atol=1e-4)
    np.testing.assert_array_equal(got["perm"].cpu().numpy(), pyg_ref.topk(scores["s"], 0.5, b.batch).numpy())
    same = np.mean(np.isin(got["perm"].cpu().numpy(), ref_perm.numpy()))
    assert same > 0.999


@pytest.mark.parametrize("name,h,n", [("GraphSAGE_SAG", 512, 71), ("EAGNN_SAG", 64, 30)])
def test_sag_adam_steps_follow_oracle(dev, name, h, n):
    """Three Adam steps (lr 1e-3, dropout 0, BN in train mode) of the whole pooled model on the GPU
    (fused SAGE / GraphNet layers, the folded encoder for GraphSAGE_SAG on 20k nodes, SAGPooling
    forward + backward) follow the oracle's CPU trajectory: same losses to 1e-3 relative, finite
    gradients for every trained parameter, the scorer included."""
    b = Batch.from_data_list([S.make_mesh_graph(n, s) for s in range(4)])
    torch.manual_seed(0)
    m = bgnn.BuckGNN(16, 5, hidden_channels=h, num_layers=6, pooling_layer="mean", dropout_rate=0.0,
                     model_name=name)
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    m = m.to(dev).train()
    bd = b.to(dev)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    crit = bgnn.RelativeErrorLoss()
    ref_p = {k: v.clone().requires_grad_(v.is_floating_point() and "running" not in k) for k, v in sd.items()}
    used = [k for k, v in ref_p.items() if v.requires_grad]
    ref_opt = torch.optim.Adam([ref_p[k] for k in used], lr=1e-3)
    got, ref = [], []
    for _ in range(3):
        pred, _ = m(bd.x, bd.edge_index, bd.edge_attr, bd.batch)
        loss = crit(pred, bd.y)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        for k in ("pool.gnn.lin_l.weight", "pool.gnn.lin_r.weight"):
            gk = dict(m.named_parameters())[k].grad
            assert gk is not None and bool(torch.isfinite(gk).all()), k
        for k, p in m.named_parameters():
            if p.grad is not None:
                assert bool(torch.isfinite(p.grad).all()), k
        opt.step()
        got.append(float(loss))
        rp, _ = R.sag_forward(ref_p, name, b.x, b.edge_index, b.edge_attr, b.batch, True, 0.0)
        rl = R.relative_error_loss(rp, b.y)
        ref_opt.zero_grad(set_to_none=True)
        rl.backward()
        ref_opt.step()
        ref.append(float(rl))
    np.testing.assert_allclose(got, ref, rtol=1e-3, atol=1e-5)


def test_sagpooling_int32_edge_index_and_no_batch(dev):
    """An int32 edge_index with batch=None (one graph): the pooled output equals the int64 call
    (advisor round 2: the top-k kernels read `batch` as int64), and int32 `batch` vectors are
    accepted by topk_select."""
    b = S.make_batch(9, 1)
    torch.manual_seed(5)
    pool = bgnn.nn.SAGPooling(32, ratio=0.5, GNN=bgnn.nn.SAGEConv, aggr="add").to(dev)
    x = torch.randn(b.num_nodes, 32, device=dev)
    ei64 = b.edge_index.to(dev)
    out64 = pool(x, ei64)
    out32 = pool(x, ei64.to(torch.int32))
    for a, c in zip(out64, out32):
        if a is not None:
            torch.testing.assert_close(a.to(c.dtype) if a.dtype != c.dtype else a, c)
    score = torch.rand(b.num_nodes, device=dev)
    p64 = P.topk_select(score, 0.5, torch.zeros(b.num_nodes, dtype=torch.long, device=dev))
    p32 = P.topk_select(score, 0.5, torch.zeros(b.num_nodes, dtype=torch.int32, device=dev))
    for a, c in zip(p64, p32):
        assert torch.equal(a, c)
    with pytest.raises(TypeError):
        P.filter_edges(ei64, p64[1].to(torch.long), b.num_nodes)
