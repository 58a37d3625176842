"""GPU: max aggregation on the hand-written path (GraphSage_maxAggr, Models/BuckGNN.py:165-180,
459-471): the aggregate-first fused layer (bgnn.fused.SageMaxLayerFn: max aggregation with
CSR argmax, one f16x3 GEMM on [agg | x], the SAGE row epilogue, the BN / ReLU / skip / dropout
kernels) and the per-module SAGEConv(aggr='max') against the fp64 oracle, forward and every
gradient at 1e-4; the tie convention (the first maximum in edge_index order takes the gradient,
oracle/pyg_ref._ScatterMaxFirst) on integer-valued features where ties are everywhere."""
import pytest
import torch

import bgnn
from bgnn import fused, nn as bnn
from bgnn import synthetic as S
from bgnn.graph import Graph
from oracle import pyg_ref as P
from test_gpu_fused import make_params, oracle_layer

pytestmark = pytest.mark.gpu
TOL = dict(rtol=1e-4, atol=1e-4)


def _layer(dev, x, b, p, bn, training, skip, drop=0.0, seed=123, chunk=16):
    graph = Graph.build(b.edge_index.to(dev), b.num_nodes, chunk=chunk)
    d = {k: v.to(dev).requires_grad_(k not in ("rm", "rv")) for k, v in p.items()}
    rm, rv = d["rm"].detach().clone(), d["rv"].detach().clone()
    xd = x.to(dev).requires_grad_(True)
    cfg = fused.LayerConfig(2, bn, training, 0.1, 1e-5, skip, drop, seed)
    out, amax = fused.SageMaxLayerFn.apply(xd, None, d["w_l"], d["b_l"], d["w_r"], d["gamma"] if bn else None,
                                           d["beta"] if bn else None, rm if bn else None, rv if bn else None,
                                           graph, cfg)
    return out, amax, xd, d, rm, rv


@pytest.mark.parametrize("bn,training", [(True, True), (True, False), (False, True)])
@pytest.mark.parametrize("skip", [False, True])
@pytest.mark.parametrize("H", [64, 512])
@pytest.mark.parametrize("super_node", [False, True])
def test_fused_max_layer_matches_oracle(dev, bn, training, skip, H, super_node):
    b = S.make_batch(9, 3, super_node=super_node)
    torch.manual_seed(H + 1)
    x = torch.randn(b.num_nodes, H)
    p = make_params(H, 11)
    out, amax, xd, d, rm, rv = _layer(dev, x, b, p, bn, training, skip)
    assert amax.item() == out.detach().abs().max().item()
    up = torch.randn_like(out)
    out.backward(up)
    ro, xc, t = oracle_layer(x, b.edge_index, p, "max", bn, training, skip)
    ro.backward(up.cpu().double())
    torch.testing.assert_close(out.detach().cpu(), ro.float(), **TOL)
    torch.testing.assert_close(xd.grad.cpu(), xc.grad.float(), **TOL)
    for k in ("w_l", "b_l", "w_r") + (("gamma", "beta") if bn else ()):
        torch.testing.assert_close(d[k].grad.cpu(), t[k].grad.float(), **TOL, msg=k)
    if bn and training:
        torch.testing.assert_close(rm.cpu(), t["rm"].detach().float(), rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(rv.cpu(), t["rv"].detach().float(), rtol=1e-5, atol=1e-6)


def test_fused_max_layer_dropout_mask(dev):
    """Skip layer with dropout: the forward mask and the backward's (the drop-add epilogue of the
    lin_r input-gradient GEMM) are the same counter-based mask."""
    H, drop = 512, 0.25
    b = S.make_batch(12, 2)
    torch.manual_seed(0)
    x = torch.randn(b.num_nodes, H)
    p = make_params(H, 3)
    out, _, xd, d, _, _ = _layer(dev, x, b, p, True, True, True, drop=drop, seed=987654321)
    y0, _, _ = oracle_layer(x, b.edge_index, p, "max", True, True, True)
    keep = out.detach().cpu() != 0
    nz = y0.detach().abs() > 1e-6
    assert abs((1 - keep[nz].float().mean().item()) - drop) < 0.01
    up = torch.randn_like(out)
    out.backward(up)
    ro, xc, t = oracle_layer(x, b.edge_index, p, "max", True, True, True, mask=keep, keep_scale=1 / (1 - drop))
    ro.backward(up.cpu().double())
    torch.testing.assert_close(out.detach().cpu(), ro.detach().float(), **TOL)
    torch.testing.assert_close(xd.grad.cpu(), xc.grad.float(), **TOL)
    torch.testing.assert_close(d["w_r"].grad.cpu(), t["w_r"].grad.float(), **TOL)


@pytest.mark.parametrize("H,Cin", [(64, 64), (512, 512), (512, 128)])
@pytest.mark.parametrize("super_node", [False, True])
@pytest.mark.parametrize("ties", [False, True])
def test_sageconv_max_module_fast_path(dev, monkeypatch, H, Cin, super_node, ties):
    """bgnn.nn.SAGEConv(aggr='max') takes the hand-written path (SageConvFn, aggregate-first) and
    matches the fp64 oracle; with ties=True the features are small integers (ReLU-like zeros and
    repeated values: most (target, column) maxima are tied), which pins the tie convention --
    splitting the gradient over the ties would miss by O(1)."""
    calls = []
    real = fused.SageConvFn.apply
    monkeypatch.setattr(fused.SageConvFn, "apply", lambda *a: calls.append(1) or real(*a))
    b = S.make_batch(11, 3, super_node=super_node)
    torch.manual_seed(5)
    conv = bnn.SAGEConv(in_channels=Cin, out_channels=H, normalize=True, aggr="max")
    ref = P.SAGEConv(Cin, H, aggr="max", normalize=True).double()
    ref.load_state_dict({k: v.double() for k, v in conv.state_dict().items()})
    conv = conv.to(dev)
    x = torch.randint(-1, 3, (b.num_nodes, Cin)).clamp_min(0).float() if ties else torch.randn(b.num_nodes, Cin)
    up = torch.randn(b.num_nodes, H)
    xd = x.to(dev).requires_grad_(True)
    out = conv(xd, b.edge_index.to(dev))
    out.backward(up.to(dev))
    xr = x.double().requires_grad_(True)
    ro = ref(xr, b.edge_index)
    ro.backward(up.double())
    assert calls, "SAGEConv(aggr='max') did not take the hand-written path"
    torch.testing.assert_close(out.detach().cpu(), ro.detach().float(), **TOL)
    torch.testing.assert_close(xd.grad.cpu(), xr.grad.float(), **TOL)
    for (k, p), (_, q) in zip(conv.named_parameters(), ref.named_parameters()):
        torch.testing.assert_close(p.grad.cpu(), q.grad.float(), **TOL, msg=k)


def test_max_ties_kernel_first_occurrence(dev):
    """The aggregation kernel's own argmax on the oracle KAT (tests/test_oracle.py): targets
    0 <- {1, 2, 3}, 1 <- {2, 0}; the first edge attaining the maximum gets the whole gradient."""
    from bgnn import ops
    x = torch.tensor([[0.0, 5.0, 0.0, 5.0], [0.0, 1.0, 0.0, 1.0], [0.0, 5.0, 0.0, 5.0], [-1.0, 5.0, -1.0, 5.0]],
                     device=dev, requires_grad=True)
    ei = torch.tensor([[1, 2, 3, 2, 0], [0, 0, 0, 1, 1]], device=dev)
    g = bgnn.graph_for(ei, 4)
    out = ops.aggregate(x, g, "max")
    up = torch.tensor([[1.0, 10.0] * 2, [100.0, 1000.0] * 2, [7.0, 7.0] * 2, [9.0, 9.0] * 2], device=dev)
    out.backward(up)
    exp = torch.tensor([[0.0, 0.0] * 2, [1.0, 0.0] * 2, [100.0, 1010.0] * 2, [0.0, 0.0] * 2])
    assert torch.equal(x.grad.cpu(), exp)


def test_maxaggr_model_runs_fused_layers(dev, monkeypatch):
    """bgnn.BuckGNN('GraphSage_maxAggr') at h = 512 runs its six layers as SageMaxLayerFn (no torch
    Linear / BatchNorm / F.normalize in the layer loop) and matches its own per-op module graph."""
    calls = []
    real = fused.SageMaxLayerFn.apply
    monkeypatch.setattr(fused.SageMaxLayerFn, "apply", lambda *a: calls.append(1) or real(*a))
    b = S.make_batch(20, 3, super_node=True).to(dev)
    res = []
    for use_fused in (True, False):
        torch.manual_seed(0)
        m = bgnn.BuckGNN(16, 5, hidden_channels=512, num_layers=6, dropout_rate=0.0,
                         model_name="GraphSage_maxAggr").to(dev)
        m.use_fused = use_fused
        pred, _ = m(b.x, b.edge_index, b.edge_attr, b.batch)
        pred.sum().backward()
        res.append([pred.detach()] + [p.grad for p in m.sage_blocks_max.parameters()])
    assert len(calls) == 6
    for a, c in zip(*res):
        torch.testing.assert_close(a, c, rtol=1e-3, atol=1e-4)


def test_compact_argmax_rejects_chunk_beyond_byte_range(dev):
    """The compact argmax state keeps a light row's argmax as a byte offset (heavy rows: marker 255),
    so a CSR whose chunk lets a light row have >= 255 edges is rejected loudly instead of wrapping
    the offsets: a 300-chunk CSR with a row of degree 280 fails, the same graph with the
    default chunk (the row is then heavy) runs, and its forward max equals the fp64 oracle."""
    from bgnn import ops
    n = 300
    src = torch.arange(1, 281, dtype=torch.long)
    ei = torch.stack([src, torch.zeros_like(src)])            # row 0: in-degree 280
    ei = torch.cat([ei, torch.stack([torch.arange(n - 1), torch.arange(1, n)])], 1)
    x = torch.randn(n, 64)
    g_big = Graph.build(ei.to(dev), n, chunk=300)
    from bgnn._lib import BgnnError
    with pytest.raises(BgnnError, match="chunk"):
        ops.spmm_fwd(g_big.fwd, x.to(dev), 2, n, want_arg=True)
    g = Graph.build(ei.to(dev), n)
    agg, arg = ops.spmm_fwd(g.fwd, x.to(dev), 2, n, want_arg=True)
    ref = P.sage_aggregate(x.double(), ei, "max")
    torch.testing.assert_close(agg.cpu().double(), ref, rtol=0, atol=0)
