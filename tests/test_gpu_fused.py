"""GPU: the fused SAGE layer (bgnn.fused.SageLayerFn) against the CPU oracle
composition SAGEConv(normalize) -> BatchNorm1d -> ReLU -> skip -> Dropout
(Models/BuckGNN.py:430-444), forward and every gradient."""
import copy
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from bgnn import fused
from bgnn.graph import Graph
from bgnn import synthetic as S
from oracle import pyg_ref as P

pytestmark = pytest.mark.gpu
TOL = dict(rtol=1e-4, atol=1e-4)


def make_params(H, seed):
    g = torch.Generator().manual_seed(seed)
    return dict(
        w_l=torch.randn(H, H, generator=g) / H ** 0.5, b_l=0.1 * torch.randn(H, generator=g),
        w_r=torch.randn(H, H, generator=g) / H ** 0.5, gamma=1 + 0.1 * torch.randn(H, generator=g),
        beta=0.1 * torch.randn(H, generator=g), rm=0.1 * torch.randn(H, generator=g),
        rv=1 + 0.2 * torch.rand(H, generator=g))


def oracle_layer(x, ei, p, aggr, bn, training, skip, mask=None, keep_scale=1.0):
    t = {k: v.double().clone().requires_grad_(k not in ("rm", "rv")) for k, v in p.items()}
    xc = x.double().clone().requires_grad_(True)
    agg = P.sage_aggregate(xc, ei, aggr)
    h = agg @ t["w_l"].t() + t["b_l"] + xc @ t["w_r"].t()
    o = F.normalize(h, p=2.0, dim=-1)
    if bn:
        o = F.batch_norm(o, t["rm"], t["rv"], t["gamma"], t["beta"], training, 0.1, 1e-5)
    y = F.relu(o)
    if skip:
        y = y + xc
    if mask is not None:
        y = y * mask.double() * keep_scale
    return y, xc, t


@pytest.mark.parametrize("aggr,red", [("sum", 0), ("mean", 1)])
@pytest.mark.parametrize("bn,training", [(True, True), (True, False), (False, True)])
@pytest.mark.parametrize("skip", [False, True])
@pytest.mark.parametrize("H", [64, 512])
def test_fused_layer_matches_oracle(dev, aggr, red, bn, training, skip, H):
    b = S.make_batch(9, 3, super_node=True)
    n = b.num_nodes
    torch.manual_seed(H)
    x = torch.randn(n, H)
    p = make_params(H, 7)
    graph = Graph.build(b.edge_index.to(dev), n, chunk=16)
    d = {k: v.to(dev).requires_grad_(k not in ("rm", "rv")) for k, v in p.items()}
    rm, rv = d["rm"].detach().clone(), d["rv"].detach().clone()
    xd = x.to(dev).requires_grad_(True)
    cfg = fused.LayerConfig(red, bn, training, 0.1, 1e-5, skip, 0.0, 123)
    out, amax = fused.SageLayerFn.apply(xd, None, d["w_l"], d["b_l"], d["w_r"], d["gamma"] if bn else None,
                                        d["beta"] if bn else None, rm if bn else None, rv if bn else None, graph,
                                        cfg)
    assert amax.item() == out.detach().abs().max().item()   # next layer's operand scale, exact
    up = torch.randn_like(out)
    out.backward(up)
    ro, xc, t = oracle_layer(x, b.edge_index, p, aggr, bn, training, skip)
    ro.backward(up.cpu().double())
    torch.testing.assert_close(out.detach().cpu(), ro.float(), **TOL)
    torch.testing.assert_close(xd.grad.cpu(), xc.grad.float(), **TOL)
    for k in ("w_l", "b_l", "w_r") + (("gamma", "beta") if bn else ()):
        torch.testing.assert_close(d[k].grad.cpu(), t[k].grad.float(), **TOL, msg=k)
    if bn and training:
        torch.testing.assert_close(rm.cpu(), t["rm"].detach().float(), rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(rv.cpu(), t["rv"].detach().float(), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("z_planes,dz_planes", [(False, False), (True, False), (False, True), (True, True)])
@pytest.mark.parametrize("H", [128, 512])
def test_fused_layer_layouts(dev, monkeypatch, z_planes, dz_planes, H):
    """Every z / dz storage layout (interleaved [N, 2H] or two [N, H] planes) matches the oracle."""
    monkeypatch.setattr(fused, "Z_PLANES", z_planes)
    monkeypatch.setattr(fused, "DZ_PLANES", dz_planes)
    test_fused_layer_matches_oracle(dev, "mean", 1, True, True, True, H)


@pytest.mark.parametrize("mode", [0, 2])
@pytest.mark.parametrize("aggr,red", [("sum", 0), ("mean", 1)])
def test_fused_layer_gemm_modes(dev, mode, aggr, red):
    """The layer matches the oracle with every GEMM family (f32 MFMA / f16x3)."""
    from bgnn import _lib
    _lib.call("bgnn_set_tuning", 5, mode)
    try:
        test_fused_layer_matches_oracle(dev, aggr, red, True, True, True, 512)
    finally:
        _lib.call("bgnn_set_tuning", 5, 2)


def _layer_grads(dev, H, rev):
    from bgnn import _lib
    b = S.make_batch(9, 3, super_node=True)
    torch.manual_seed(3)
    x = torch.randn(b.num_nodes, H)
    p = make_params(H, 7)
    graph = Graph.build(b.edge_index.to(dev), b.num_nodes, chunk=16)
    d = {k: v.to(dev).requires_grad_(k not in ("rm", "rv")) for k, v in p.items()}
    xd = x.to(dev).requires_grad_(True)
    cfg = fused.LayerConfig(0, True, True, 0.1, 1e-5, True, 0.1, 123)
    _lib.call("bgnn_set_tuning", 13, rev)
    try:
        out, amax = fused.SageLayerFn.apply(xd, None, d["w_l"], d["b_l"], d["w_r"], d["gamma"], d["beta"],
                                         d["rm"].detach().clone(), d["rv"].detach().clone(), graph, cfg)
        out.backward(torch.randn(out.shape, generator=torch.Generator().manual_seed(5)).to(dev))
    finally:
        _lib.call("bgnn_set_tuning", 13, 1)
    return {"out": out.detach(), "amax": amax, "x": xd.grad,
            **{k: d[k].grad for k in ("w_l", "b_l", "w_r", "gamma", "beta")}}


@pytest.mark.parametrize("rev", [1, 2, 4, 8, 15])
@pytest.mark.parametrize("H", [64, 512])
def test_rows_rev_walk(dev, H, rev):
    """BGNN_TUNE_ROWS_REV changes only the order rows are visited in. Bits 1 (sage_apply sweeps
    each eighth of the rows from its end) and 3 (the transpose aggregation sweeps each eighth
    downward) leave every result bit-identical; bit 0 (sage_bwd_rows walks each block's rows from
    the last one down) changes only the order of the bias-gradient partial sums: dh, and so every
    other gradient, is bit-identical, b_l agrees to f32 rounding; bit 2 (the SAGE aggregation
    sweeps each eighth downward) changes the summation order of the BatchNorm statistics, so
    everything agrees to f32 rounding. The layer still matches the oracle."""
    a, r = _layer_grads(dev, H, 0), _layer_grads(dev, H, rev)
    keys = ("out", "amax", "x", "w_l", "w_r", "gamma", "beta", "b_l")
    exact = () if rev & 4 else keys[:-1] if rev & 1 else keys
    for k in keys:
        if k in exact:
            assert torch.equal(a[k], r[k]), k
        else:
            torch.testing.assert_close(r[k], a[k], rtol=1e-4, atol=1e-5, msg=k)
    from bgnn import _lib
    _lib.call("bgnn_set_tuning", 13, rev)
    try:
        test_fused_layer_matches_oracle(dev, "sum", 0, True, True, True, H)
    finally:
        _lib.call("bgnn_set_tuning", 13, 1)


def test_dropout_mask_fraction_and_backward_consistency(dev):
    H = 512
    b = S.make_batch(12, 2)
    n = b.num_nodes
    torch.manual_seed(0)
    x = torch.randn(n, H)
    p = make_params(H, 3)
    graph = Graph.build(b.edge_index.to(dev), n)
    d = {k: v.to(dev).requires_grad_(k not in ("rm", "rv")) for k, v in p.items()}
    xd = x.to(dev).requires_grad_(True)
    drop = 0.25
    cfg = fused.LayerConfig(0, True, True, 0.1, 1e-5, True, drop, 987654321)
    out, _ = fused.SageLayerFn.apply(xd, None, d["w_l"], d["b_l"], d["w_r"], d["gamma"], d["beta"],
                                     d["rm"].detach().clone(), d["rv"].detach().clone(), graph, cfg)
    y0, _, _ = oracle_layer(x, b.edge_index, p, "sum", True, True, True)
    keep = out.detach().cpu() != 0
    nz = y0.detach().abs() > 1e-6
    frac = 1 - keep[nz].float().mean().item()
    assert abs(frac - drop) < 0.01, frac
    torch.testing.assert_close(out.detach().cpu()[keep], (y0.detach()[keep] / (1 - drop)).float(), **TOL)
    up = torch.randn_like(out)
    out.backward(up)
    ro, xc, t = oracle_layer(x, b.edge_index, p, "sum", True, True, True, mask=keep, keep_scale=1 / (1 - drop))
    ro.backward(up.cpu().double())
    torch.testing.assert_close(xd.grad.cpu(), xc.grad.float(), **TOL)
    torch.testing.assert_close(d["w_l"].grad.cpu(), t["w_l"].grad.float(), **TOL)


@pytest.mark.parametrize("n,drop", [(71, 0.25), (71, 0.1), (71, 0.0)])
def test_dgrad_dropadd_bit_identical(dev, monkeypatch, n, drop):
    """Skip layers: the dgrad adding drop(g) in its epilogue (bgnn_gemm_f32_dropadd, mask
    recomputed from the layer's seed) gives bit-identical gradients to the path where
    bgnn_sage_bwd_rows writes the skip gradient and the dgrad reads it back as C (10,082 nodes:
    interior and ragged tiles, enough tiles that neither path splits K -- drop-add never does,
    so on small batches the two differ by split-K rounding only, see test_dgrad_dropadd_small)."""
    H = 512
    b = S.make_batch(n, 2)
    N = b.num_nodes
    torch.manual_seed(n)
    x = torch.randn(N, H)
    p = make_params(H, 5)
    graph = Graph.build(b.edge_index.to(dev), N)
    up = torch.randn(N, H).to(dev)
    res = {}
    for flag in (True, False):
        monkeypatch.setattr(fused, "DGRAD_DROPADD", flag)
        d = {k: v.to(dev).requires_grad_(k not in ("rm", "rv")) for k, v in p.items()}
        xd = x.to(dev).requires_grad_(True)
        cfg = fused.LayerConfig(0, True, True, 0.1, 1e-5, True, drop, 4242)
        out, amax = fused.SageLayerFn.apply(xd, None, d["w_l"], d["b_l"], d["w_r"], d["gamma"], d["beta"],
                                         d["rm"].detach().clone(), d["rv"].detach().clone(), graph, cfg)
        out.backward(up)
        res[flag] = [xd.grad] + [d[k].grad for k in ("w_l", "b_l", "w_r", "gamma", "beta")]
    for a, c in zip(res[True], res[False]):
        assert torch.equal(a, c)


def test_dgrad_dropadd_small(dev, monkeypatch):
    """Small batch (288 nodes): the gskip path's dgrad runs split-K, drop-add does not; both
    match the oracle (the dropout test above) and each other to f32 rounding."""
    H = 512
    b = S.make_batch(12, 2)
    N = b.num_nodes
    torch.manual_seed(1)
    x = torch.randn(N, H)
    p = make_params(H, 6)
    graph = Graph.build(b.edge_index.to(dev), N)
    up = torch.randn(N, H).to(dev)
    res = {}
    for flag in (True, False):
        monkeypatch.setattr(fused, "DGRAD_DROPADD", flag)
        d = {k: v.to(dev).requires_grad_(k not in ("rm", "rv")) for k, v in p.items()}
        xd = x.to(dev).requires_grad_(True)
        cfg = fused.LayerConfig(0, True, True, 0.1, 1e-5, True, 0.2, 99)
        out, amax = fused.SageLayerFn.apply(xd, None, d["w_l"], d["b_l"], d["w_r"], d["gamma"], d["beta"],
                                         d["rm"].detach().clone(), d["rv"].detach().clone(), graph, cfg)
        out.backward(up)
        res[flag] = xd.grad
    torch.testing.assert_close(res[True], res[False], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("N", [1, 63, 65, 1000, 80656])
def test_encoder_head_mlp2_matches_fp64(dev, N):
    """bgnn_mlp2 (the encoder's Linear(16,64).ReLU.Linear(64,128).ReLU on the VALU, weights in
    LDS) against an fp64 torch run: output, max|h|, and the four parameter gradients; the
    backward is deterministic (bit-identical on a second run)."""
    from bgnn import fused
    old = fused.FUSED_MLP2
    fused.FUSED_MLP2 = True
    try:
        _check_mlp2(dev, N)
    finally:
        fused.FUSED_MLP2 = old


def _check_mlp2(dev, N):
    from bgnn import fused
    torch.manual_seed(N)
    seq = torch.nn.Sequential(torch.nn.Linear(16, 64), torch.nn.ReLU(), torch.nn.Linear(64, 128), torch.nn.ReLU())
    seq = seq.to(dev)
    x = torch.randn(N, 16, device=dev)
    gy = torch.randn(N, 128, device=dev)
    assert fused._mlp2_prefix(list(seq), x)
    h, amax = fused.mlp(seq, x, return_amax=True)
    (h * gy).sum().backward()
    grads = [p.grad.clone() for p in seq.parameters()]
    for p in seq.parameters():
        p.grad = None
    h2, _ = fused.mlp(seq, x, return_amax=True)
    (h2 * gy).sum().backward()
    for g, p in zip(grads, seq.parameters()):
        assert torch.equal(g, p.grad)
    ref = copy.deepcopy(seq).double().cpu()
    hr = ref(x.double().cpu())
    (hr * gy.double().cpu()).sum().backward()
    torch.testing.assert_close(h.double().cpu(), hr, rtol=1e-5, atol=1e-5)
    assert float(amax) == float(h.abs().max())
    for g, p in zip(grads, ref.parameters()):
        scale = p.grad.abs().max().item() + 1e-30
        assert (g.double().cpu() - p.grad).abs().max().item() <= 1e-5 * scale + 1e-6


@pytest.mark.parametrize("p,with_b", [(0.1, True), (0.25, False), (0.0, True)])
def test_ea_skip_dropout(dev, p, with_b):
    """EA_GNN's skip + dropout in one pass (bgnn_add_dropout): kept elements are exactly
    (a + b) / (1 - p), the keep fraction is 1 - p, and the backward sends the same mask of the
    incoming gradient to both inputs; p = 0 is the plain add."""
    from bgnn.ea import skip_dropout
    torch.manual_seed(3)
    a = torch.randn(20000, 512, device=dev, requires_grad=True)
    b = torch.randn(20000, 512, device=dev, requires_grad=True) if with_b else None
    out = skip_dropout(a, b, p, True, 123456789)
    s = (a + b if with_b else a).detach()
    # the mask itself, from the same seed on a tensor of ones (value-independent)
    keep = skip_dropout(torch.ones_like(s), None, p, True, 123456789) != 0
    if p == 0.0:
        assert torch.equal(out.detach(), s)
    else:
        frac = 1 - keep.float().mean().item()
        assert abs(frac - p) < 0.005, frac
        torch.testing.assert_close(out.detach(), torch.where(keep, s * (1.0 / (1.0 - p)), torch.zeros_like(s)),
                                   rtol=0, atol=0)
    g = torch.randn_like(out)
    out.backward(g)
    want = torch.where(keep, g * (1.0 / (1.0 - p)) if p else g, torch.zeros_like(g))
    torch.testing.assert_close(a.grad, want, rtol=0, atol=0)
    if with_b:
        assert torch.equal(b.grad, a.grad)


@pytest.mark.parametrize("dims", [(512, 128, 64, 1), (1024, 128, 64, 1), (64, 64, 3)])
@pytest.mark.parametrize("rows", [1, 16, 200])
def test_small_mlp_matches_fp64(dev, dims, rows):
    """The decoder on the pooled features (bgnn.fused.small_mlp: bgnn_small_linear_fwd / _bwd,
    Models/BuckGNN.py:94-100): output and every gradient (input, weights, biases) against an fp64
    torch run of the same nn.Sequential, ReLUs included (inputs with many exact zeros)."""
    from bgnn import fused
    torch.manual_seed(rows + dims[0])
    layers = []
    for a, b in zip(dims[:-1], dims[1:]):
        layers += [torch.nn.Linear(a, b), torch.nn.ReLU()]
    seq = torch.nn.Sequential(*layers[:-1]).to(dev)
    x = torch.randn(rows, dims[0], device=dev).clamp_min(0).requires_grad_(True)
    out = fused.small_mlp(seq, x)
    assert out is not None
    gy = torch.randn_like(out)
    grads = torch.autograd.grad(out, [x] + list(seq.parameters()), gy)
    seq64 = copy.deepcopy(seq).double()
    x64 = x.detach().double().requires_grad_(True)
    out64 = seq64(x64)
    grads64 = torch.autograd.grad(out64, [x64] + list(seq64.parameters()), gy.double())
    torch.testing.assert_close(out.double(), out64, rtol=1e-5, atol=1e-5)
    for g, g64 in zip(grads, grads64):
        torch.testing.assert_close(g.double(), g64, rtol=1e-5, atol=1e-5 * (1 + g64.abs().max().item()))
    again = torch.autograd.grad(fused.small_mlp(seq, x), [x] + list(seq.parameters()), gy)
    for g, g2 in zip(grads, again):   # deterministic
        assert torch.equal(g, g2)


@pytest.mark.parametrize("model_name,n,super_node", [("GraphSage_addAggr", 45, False), ("GraphSage_meanAggr", 45, False),
                                                     ("GraphSage_addAggr_Shared", 45, False),
                                                     ("GraphSage_addAggr", 71, True)])
def test_fused_mean_pool_bit_identical(dev, monkeypatch, model_name, n, super_node):
    """Buckling + mean pooling: the last fused layer returning the per-graph mean pool
    (SageLayerFn pool; its backward reads the pooled gradient / count through the batch vector,
    bgnn_sage_bwd_stats / _rows g_rows) gives the same bits as the separate pool + [N, H]
    broadcast: prediction, loss, every parameter gradient and the BatchNorm running statistics
    (train mode, dropout 0.1; 71x71 meshes with super nodes: range rows on the last layer)."""
    import copy as _copy
    import bgnn
    from bgnn import buckgnn
    b = S.make_batch(n, 8 if n == 45 else 16, super_node=super_node).to(dev)
    torch.manual_seed(0)
    model0 = bgnn.BuckGNN(16, 5, hidden_channels=512, num_layers=6, dropout_rate=0.1,
                          model_name=model_name).to(dev).train()
    res = {}
    for flag in (True, False):
        monkeypatch.setattr(buckgnn, "FUSED_POOL", flag)
        m = _copy.deepcopy(model0)
        torch.manual_seed(123)
        out, _ = m(b.x, b.edge_index, b.edge_attr, b.batch)
        loss = (out - torch.linspace(0.5, 1.5, out.numel(), device=dev)).square().mean()
        loss.backward()
        res[flag] = ([out.detach(), loss.detach()] + [p.grad for p in m.parameters()]
                     + [t for k, t in m.state_dict().items() if "running" in k])
    assert len(res[True]) == len(res[False])
    n_grads = 0
    for a, c in zip(res[True], res[False]):
        assert (a is None) == (c is None)   # (modules the model does not use get no gradient)
        if a is not None:
            n_grads += 1
            assert torch.equal(a, c)
    assert n_grads >= 5
