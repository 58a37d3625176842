"""GPU: neighbour aggregation (sum/mean/max, forward + backward), pooling and scatter
against the CPU oracle (oracle.pyg_ref). Tolerance 1e-4 abs/rel in fp32 (BASELINE north star)."""
import numpy as np
import pytest
import torch

import bgnn
from bgnn.graph import Graph, SegmentIndex
from bgnn import synthetic as S
from oracle import pyg_ref as P

pytestmark = pytest.mark.gpu
TOL = dict(rtol=1e-4, atol=1e-4)


def oracle_agg(x, ei, reduce, g):
    xc = x.detach().cpu().double().requires_grad_(True)
    out = P.sage_aggregate(xc, ei.cpu(), reduce)
    out.backward(g.cpu().double())
    return out.float(), xc.grad.float()


def run_agg(x, ei, n, reduce, chunk, dev):
    g = Graph.build(ei.to(dev), n, chunk=chunk)
    xd = x.to(dev).requires_grad_(True)
    out = bgnn.aggregate(xd, g, reduce)
    up = torch.randn_like(out)
    out.backward(up)
    ro, rg = oracle_agg(x, ei, reduce, up)
    torch.testing.assert_close(out.detach().cpu(), ro, **TOL)
    torch.testing.assert_close(xd.grad.cpu(), rg, **TOL)


GRAPHS = {
    "mesh": lambda: S.make_batch(12, 2),
    "super": lambda: S.make_batch(15, 2, super_node=True),
}


@pytest.mark.parametrize("reduce", ["sum", "mean", "max"])
@pytest.mark.parametrize("H", [1, 3, 16, 64, 100, 128, 256, 512, 700, 1024])
def test_aggregate_matches_oracle_random_graph(dev, reduce, H):
    torch.manual_seed(H)
    n, E = 257, 3000
    ei = torch.randint(0, n, (2, E))
    x = torch.randn(n, H)
    run_agg(x, ei, n, reduce, chunk=16, dev=dev)


@pytest.mark.parametrize("reduce", ["sum", "mean", "max"])
@pytest.mark.parametrize("kind", ["mesh", "super"])
@pytest.mark.parametrize("chunk", [4, 64])
def test_aggregate_meshes(dev, reduce, kind, chunk):
    b = GRAPHS[kind]()
    torch.manual_seed(1)
    x = torch.randn(b.num_nodes, 512)
    run_agg(x, b.edge_index, b.num_nodes, reduce, chunk, dev)


def test_aggregate_is_deterministic(dev):
    b = S.make_batch(30, 2, super_node=True)
    g = Graph.build(b.edge_index.to(dev), b.num_nodes, chunk=16)
    x = torch.randn(b.num_nodes, 512, device=dev)
    a1 = bgnn.aggregate(x, g, "sum")
    a2 = bgnn.aggregate(x, g, "sum")
    assert torch.equal(a1, a2)


def test_aggregate_empty_graph_gives_zero(dev):
    g = Graph.build(torch.zeros(2, 0, dtype=torch.long, device=dev), 5)
    for r in ("sum", "mean", "max"):
        assert torch.equal(bgnn.aggregate(torch.randn(5, 8, device=dev), g, r), torch.zeros(5, 8, device=dev))


@pytest.mark.parametrize("reduce", ["mean", "sum", "max"])
def test_global_pool_matches_oracle(dev, reduce):
    torch.manual_seed(0)
    batch = torch.tensor([0] * 40 + [1] * 300 + [3] * 7)     # graph 2 empty
    x = torch.randn(batch.numel(), 512)
    fn = {"mean": bgnn.global_mean_pool, "sum": bgnn.global_add_pool, "max": bgnn.global_max_pool}[reduce]
    rf = {"mean": P.global_mean_pool, "sum": P.global_add_pool, "max": P.global_max_pool}[reduce]
    xd = x.to(dev).requires_grad_(True)
    out = fn(xd, batch.to(dev))
    up = torch.randn_like(out)
    out.backward(up)
    xc = x.double().requires_grad_(True)
    ro = rf(xc, batch)
    ro.backward(up.cpu().double())
    torch.testing.assert_close(out.detach().cpu(), ro.float(), **TOL)
    torch.testing.assert_close(xd.grad.cpu(), xc.grad.float(), **TOL)


def test_scatter_unsorted_index(dev):
    torch.manual_seed(0)
    idx = torch.randint(0, 9, (500,))
    src = torch.randn(500, 33)
    for fn, rf in ((bgnn.scatter_mean, P.scatter_mean), (bgnn.scatter_add, P.scatter_add)):
        out = fn(src.to(dev), idx.to(dev), dim=0, dim_size=12)
        torch.testing.assert_close(out.cpu(), rf(src, idx, dim_size=12), **TOL)


def test_full_size_cfg3_properties(dev):
    """Full cfg3 batch (super nodes of in-degree 5,041): sum aggregation is linear and
    its transpose is the adjoint: <A x, y> == <x, A^T y> (size-independent checks)."""
    b = S.make_config_batch("cfg3")
    g = Graph.build(b.edge_index.to(dev), b.num_nodes)
    assert g.fwd.plan.n_heavy == 16
    torch.manual_seed(0)
    x = torch.randn(b.num_nodes, 512, device=dev, dtype=torch.float32)
    y = torch.randn(b.num_nodes, 512, device=dev, dtype=torch.float32)
    ax = bgnn.aggregate(x, g, "sum")
    ax2 = bgnn.aggregate(2 * x, g, "sum")
    torch.testing.assert_close(ax2, 2 * ax, rtol=0, atol=0)
    xd = x.clone().requires_grad_(True)
    bgnn.aggregate(xd, g, "sum").backward(y)
    lhs = (ax.double() * y.double()).sum()
    rhs = (x.double() * xd.grad.double()).sum()
    assert abs(float(lhs - rhs)) <= 1e-6 * float(ax.double().abs().sum() * y.double().abs().max())
    # super node rows against an independent fp64 torch sum
    s = b.ptr[1:] - 1
    ei = b.edge_index.to(dev)
    for r in s[:2].tolist():
        nb = ei[0][ei[1] == r]
        ref = x.double()[nb].sum(0)
        torch.testing.assert_close(ax[r].double(), ref, rtol=1e-5, atol=1e-4)


def _variant_graph(dev, graph):
    if graph == "mesh_super":
        b = S.make_batch(25, 3, super_node=True)
        return b.edge_index.to(dev), b.num_nodes
    n = 3000
    gen = torch.Generator().manual_seed(11)
    return torch.randint(0, n, (2, 24 * n), generator=gen).to(dev), n


def _run_all_reduces(g, x, gy):
    out = {}
    for r in ("sum", "mean", "max"):
        xx = x.clone().requires_grad_(True)
        y = bgnn.aggregate(xx, g, r)
        y.backward(gy)
        out[r] = (y.detach(), xx.grad)
    return out


@pytest.mark.parametrize("knobs", [(1, 0), (2, 8), (2, 12), (2, 16)],
                         ids=["blocked", "sweep8", "sweep12", "sweep16"])
@pytest.mark.parametrize("graph", ["mesh_super", "random_dense"])
def test_kernel_variants_bit_identical(dev, knobs, graph):
    """The per-row light-row kernels (blocked, XCD sweep with U = 8/12/16 neighbours per batch)
    give bit-identical aggregation results, forward and transpose (backward), on meshes with
    super nodes and on a dense random graph."""
    from bgnn import _lib
    ei, n = _variant_graph(dev, graph)
    g = Graph.build(ei, n)
    torch.manual_seed(3)
    x = torch.randn(n, 512, device=dev)
    gy = torch.randn(n, 512, device=dev)
    old = (_lib.query("bgnn_get_tuning", 1), _lib.query("bgnn_get_tuning", 3))
    try:
        _lib.call("bgnn_set_tuning", 1, 2)
        _lib.call("bgnn_set_tuning", 3, 8)
        ref = _run_all_reduces(g, x, gy)
        _lib.call("bgnn_set_tuning", 1, knobs[0])
        _lib.call("bgnn_set_tuning", 3, knobs[1])
        got = _run_all_reduces(g, x, gy)
        for r in ("sum", "mean", "max"):
            assert torch.equal(got[r][0], ref[r][0]), (r, "fwd")
            assert torch.equal(got[r][1], ref[r][1]), (r, "bwd")
    finally:
        _lib.call("bgnn_set_tuning", 1, old[0])
        _lib.call("bgnn_set_tuning", 3, old[1])


@pytest.mark.parametrize("rows", [4, 8])
@pytest.mark.parametrize("graph", ["mesh_super", "random_dense"])
def test_group_kernel_matches_sweep(dev, rows, graph):
    """The row-group kernel (default for sum/mean with a row-group plan) sums each row's entries
    in plan order: equal to the per-row sweep kernel to fp32 rounding, deterministic run to run,
    and the first row of every group is bit-identical (plan order = CSR order there)."""
    from bgnn import _lib
    from bgnn import graph as Gm
    ei, n = _variant_graph(dev, graph)
    old_rows = Gm.GROUP_ROWS
    Gm.GROUP_ROWS = rows
    try:
        g = Graph.build(ei, n)
    finally:
        Gm.GROUP_ROWS = old_rows
    assert g.fwd.groups is not None and g.bwd.groups is not None
    torch.manual_seed(5)
    x = torch.randn(n, 512, device=dev)
    gy = torch.randn(n, 512, device=dev)
    old = _lib.query("bgnn_get_tuning", 1)
    try:
        _lib.call("bgnn_set_tuning", 1, 2)
        ref = _run_all_reduces(g, x, gy)
        _lib.call("bgnn_set_tuning", 1, 0)
        got = _run_all_reduces(g, x, gy)
        again = _run_all_reduces(g, x, gy)
    finally:
        _lib.call("bgnn_set_tuning", 1, old)
    first = torch.arange(0, n, rows, device=dev)
    for r in ("sum", "mean", "max"):
        for k in (0, 1):
            assert torch.equal(got[r][k], again[r][k]), (r, k)
            torch.testing.assert_close(got[r][k], ref[r][k], rtol=1e-5, atol=1e-5)
        assert torch.equal(got[r][0][first], ref[r][0][first]), r


@pytest.mark.parametrize("kernel", [0, 1, 2], ids=["group", "blocked", "sweep"])
@pytest.mark.parametrize("reduce", [0, 1])
def test_spmm_bwd_folds_max_abs(dev, kernel, reduce):
    """bgnn_spmm_bwd's optional amax output is max |gx| over light rows and the super-node
    (chunked + combined) rows alike, folded into the running value."""
    from bgnn import _lib, ops
    b = S.make_batch(25, 3, super_node=True)
    g = Graph.build(b.edge_index.to(dev), b.num_nodes)
    assert g.bwd.plan.n_heavy > 0
    torch.manual_seed(4)
    gy = torch.randn(b.num_nodes, 512, device=dev)
    gy[b.ptr[1:] - 1] *= 50.0   # make a heavy row hold the maximum in one case
    old = _lib.query("bgnn_get_tuning", 1)
    try:
        _lib.call("bgnn_set_tuning", 1, kernel)
        for scale in (1.0, 1e-3):
            amax = torch.full((1,), 1e-9, device=dev)
            gx = ops.spmm_bwd(g.bwd, g.perm_t, g.fwd.rowptr, gy * scale, reduce, None, b.num_nodes, amax=amax)
            assert amax.item() == gx.abs().max().item()
    finally:
        _lib.call("bgnn_set_tuning", 1, old)


@pytest.mark.parametrize("reduce", [0, 1, 2], ids=["sum", "mean", "max"])
@pytest.mark.parametrize("graph", ["mesh_super", "random_dense"])
def test_spmm_bwd_add_equals_spmm_bwd_plus_addend(dev, reduce, graph):
    """bgnn_spmm_bwd_add (the max-aggregation layer's backward adds dh W_r there) is the transpose
    aggregation plus the addend, bit for bit, on every kernel path (row groups, sweep, heavy-row
    chunks + combine), and folds max|gx| of the sum."""
    from bgnn import _lib, ops
    ei, n = _variant_graph(dev, graph)
    g = Graph.build(ei, n)
    H = 512
    torch.manual_seed(12)
    x = torch.randn(n, H, device=dev)
    gy = torch.randn(n, H, device=dev)
    add = torch.randn(n, H, device=dev)
    arg = None
    if reduce == 2:
        _, arg = ops.spmm_fwd(g.fwd, x, 2, n, want_arg=True)
    ref = ops.spmm_bwd(g.bwd, g.perm_t, g.fwd.rowptr, gy, reduce, arg, n) + add
    gx = torch.empty(n, H, device=dev)
    amax = torch.zeros(1, device=dev)
    part = torch.empty(max(g.bwd.plan.n_chunks, 1) * H, device=dev)
    if reduce == 2:
        _lib.call("bgnn_spmm_bwd_max", g.bwd.ref(), g.perm_t.data_ptr(), g.fwd.rowptr.data_ptr(), n, gy.data_ptr(), H,
                  H, arg.data_ptr(), add.data_ptr(), H, gx.data_ptr(), H, part.data_ptr(), amax.data_ptr(),
                  torch.cuda.current_stream().cuda_stream)
    else:
        _lib.call("bgnn_spmm_bwd_add", g.bwd.ref(), g.perm_t.data_ptr(), g.fwd.rowptr.data_ptr(), gy.data_ptr(), H,
                  H, reduce, add.data_ptr(), H, gx.data_ptr(), H, part.data_ptr(), amax.data_ptr(),
                  torch.cuda.current_stream().cuda_stream)
    assert torch.equal(gx, ref)
    assert amax.item() == gx.abs().max().item()
