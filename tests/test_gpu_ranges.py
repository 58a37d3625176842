"""GPU: range rows (round 6, csrc/ranges.hip, bgnn.fused.RangeRows). A stiffened mesh's super node
(VirtualEdgeCreate.py:81-113) is wired to every real node of its graph in increasing order, and
GraphCreate.py:417-422 emits both directions, so in both CSRs its row is the contiguous run of its
graph's real nodes: its aggregation is a column sum over a row range, which the fused layer takes
from the row passes (bgnn_sage_apply / bgnn_sage_bwd_rows range partials) instead of a chunk pass
over every real row. Checked: the detection (bgnn_heavy_ranges) against a host restatement, with
shuffled super-node edges (chunk path) and overlapping ranges; the row-blocked apply's x_next bit
for bit against the grid form and its range sums against torch; the whole fused model on stiffened
batches -- predictions, loss and every gradient -- against the chunk path (switch off) and against
the fp64 oracle, for sum and mean aggregation, with some super nodes left to the chunk path."""
import numpy as np
import pytest
import torch

import bgnn
from bgnn import _lib, fused
from bgnn import synthetic as S
from bgnn.graph import Graph
from oracle import buckgnn_ref as R

pytestmark = pytest.mark.gpu


def _host_ranges(rowptr, col, chunk):
    """restatement of bgnn_heavy_ranges: (first or -1) per heavy row; a candidate is kept when its
    run starts at or after the end of every earlier candidate's run"""
    deg = np.diff(rowptr)
    heavy = np.nonzero(deg > chunk)[0]
    first = []
    for r in heavy:
        c = col[rowptr[r]:rowptr[r + 1]]
        first.append(int(c[0]) if np.array_equal(c, c[0] + np.arange(c.size)) else -1)
    prev, comp = -(1 << 31), []
    for h, a in enumerate(first):
        if a < 0:
            continue
        e = a + int(deg[heavy[h]])
        if a >= prev:
            comp.append((a, e, h))
        else:
            first[h] = -1
        prev = max(prev, e)
    return first, comp


def _shuffle_super(b, graphs_to_shuffle, seed=0):
    """edge_index with the super-node edges of the given graphs in a random order (their rows stay
    heavy but are no range rows)"""
    ei = b.edge_index.clone()
    rng = np.random.default_rng(seed)
    ptr = b.ptr.numpy()
    for g in graphs_to_shuffle:
        s = int(ptr[g + 1]) - 1                      # the super node: the graph's last node
        idx = torch.nonzero((ei[1] == s) | (ei[0] == s)).flatten().numpy()
        perm = rng.permutation(idx.size)
        ei[:, idx] = ei[:, idx[perm]]
    return ei


@pytest.mark.parametrize("shuffled", [(), (1,)], ids=["all-range", "one-shuffled"])
def test_heavy_ranges_detection(dev, shuffled):
    b = S.make_batch(9, 3, super_node=True)
    ei = _shuffle_super(b, shuffled)
    g = Graph.build(ei.to(dev), b.num_nodes)
    for csr in (g.fwd, g.bwd):
        rg = csr.ensure_ranges().cpu().numpy()
        nh = csr.plan.n_heavy
        assert nh == 3 and rg[1] == nh
        first, comp = _host_ranges(csr.rowptr.cpu().numpy(), csr.col.cpu().numpy(), csr.plan.chunk)
        assert list(rg[2 + 3 * nh:2 + 4 * nh]) == first
        assert rg[0] == len(comp)
        assert [tuple(rg[2 + 3 * k:5 + 3 * k]) for k in range(rg[0])] == comp
        assert csr.ranges_all == int(len(comp) == nh)
    assert g.fwd.ranges_all == (0 if shuffled else 1)


def test_overlapping_ranges_go_to_the_chunk_path(dev):
    """heavy rows over overlapping source ranges [0, 200), [100, 300), [250, 330), [330, 400): the
    second and third start before an earlier run ends and are left to the chunk path"""
    n, chunk = 500, 64
    runs = [(0, 200), (100, 300), (250, 330), (330, 400)]
    src = torch.cat([torch.arange(a, e) for a, e in runs])
    dst = torch.cat([torch.full((e - a,), 496 + i) for i, (a, e) in enumerate(runs)])
    g = Graph.build(torch.stack([src, dst]).to(dev), n, chunk)
    rg = g.fwd.ensure_ranges().cpu().numpy()
    first, comp = _host_ranges(g.fwd.rowptr.cpu().numpy(), g.fwd.col.cpu().numpy(), chunk)
    assert comp == [(0, 200, 0), (330, 400, 3)] and first == [0, -1, -1, 330]
    assert rg[0] == 2 and [tuple(rg[2 + 3 * k:5 + 3 * k]) for k in range(2)] == comp
    assert list(rg[2 + 3 * 4:]) == first
    assert g.fwd.ranges_all == 0


def test_apply_rows_bits_and_range_sums(dev):
    b = S.make_batch(20, 4, super_node=True)
    g = Graph.build(b.edge_index.to(dev), b.num_nodes)
    rg = g.fwd.ensure_ranges()
    N, H = b.num_nodes, 512
    torch.manual_seed(3)
    o = torch.randn(N, H, device=dev)
    xp = torch.randn(N, H, device=dev)
    scale, shift = torch.rand(H, device=dev) + 0.5, torch.randn(H, device=dev) * 0.1
    s = fused._stream()
    outs = []
    for use in (False, True):
        x = torch.empty(N, H, device=dev)
        am = torch.zeros(1, device=dev)
        rp = torch.empty(_lib.query("bgnn_range_partial_bytes", N, H) // 4, device=dev) if use else None
        _lib.call("bgnn_sage_apply", o.data_ptr(), scale.data_ptr(), shift.data_ptr(), xp.data_ptr(), 1, 0.2, 77, N, H,
                  x.data_ptr(), am.data_ptr(), rg.data_ptr() if use else None, rp.data_ptr() if use else None, s)
        outs.append((x, am, rp))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    x = outs[1][0]
    Rn = g.fwd.plan.n_heavy
    sums = torch.empty(Rn, H, device=dev)
    aug = torch.zeros(1, device=dev)
    _lib.call("bgnn_range_sums_finish", outs[1][2].data_ptr(), N, H, g.fwd.ref(), 0, sums.data_ptr(), H,
              outs[1][1].data_ptr(), aug.data_ptr(), s)
    r = rg.cpu().numpy()
    for k in range(r[0]):
        a, e, h = r[2 + 3 * k:5 + 3 * k]
        ref = x[a:e].double().sum(0)
        torch.testing.assert_close(sums[h].double(), ref, rtol=1e-5, atol=1e-4)
    assert aug.item() == max(outs[1][1].item(), sums.abs().max().item())


def _grads(dev, b, ei, model_name, on, monkeypatch):
    monkeypatch.setattr(fused, "RANGE_ROWS", on)
    torch.manual_seed(0)
    m = bgnn.BuckGNN(16, 5, hidden_channels=512, num_layers=6, dropout_rate=0.0, model_name=model_name).to(dev)
    m.train()
    calls = []
    real = _lib.call

    def spy(name, *a):
        calls.append(name)
        return real(name, *a)
    monkeypatch.setattr(_lib, "call", spy)
    pred, _ = m(b.x.to(dev), ei.to(dev), None, b.batch.to(dev))
    loss = bgnn.RelativeErrorLoss()(pred, b.y.to(dev))
    loss.backward()
    monkeypatch.setattr(_lib, "call", real)
    g = {k: p.grad.detach().clone() for k, p in m.named_parameters() if p.grad is not None}
    return pred.detach(), float(loss), g, calls


@pytest.mark.parametrize("model_name", ["GraphSage_addAggr", "GraphSage_meanAggr", "GraphSage_addAggr_Shared"])
@pytest.mark.parametrize("shuffled", [(), (2,)], ids=["all-range", "one-shuffled"])
def test_fused_model_range_rows_match_chunk_path_and_fp64(dev, monkeypatch, model_name, shuffled):
    """stiffened 31x31 meshes (N = 4 x 962, >= 1,024: the folded encoder + the pre-split GEMMs), the
    fused loop with range rows against the chunk path: predictions to 1e-5, every gradient to 1e-4
    relative L2; and against the fp64 oracle as tests/test_gpu_fullsize.py bounds it"""
    b = S.make_batch(31, 4, super_node=True)
    ei = _shuffle_super(b, shuffled)
    p1, l1, g1, c1 = _grads(dev, b, ei, model_name, True, monkeypatch)
    p0, l0, g0, c0 = _grads(dev, b, ei, model_name, False, monkeypatch)
    # the range path ran: 5 of 6 forward layers take their super-node aggregates from the range sums
    # (layer 0 folds the encoder), every backward layer its super-node dz_l rows
    assert c1.count("bgnn_range_sums_finish") == 5 + 6 and c0.count("bgnn_range_sums_finish") == 0
    torch.testing.assert_close(p1, p0, rtol=1e-5, atol=1e-5)
    assert abs(l1 - l0) <= 1e-5 * abs(l0)
    assert g1.keys() == g0.keys()
    # per parameter: L2 distance within 1e-4 of its gradient norm, plus a floor of 1e-6 of the largest
    # per-element RMS gradient (biases feeding a BatchNorm have an exact gradient of 0: rounding noise)
    rms0 = max(float(v.pow(2).mean().sqrt()) for v in g0.values())
    for k in g0:
        err, nrm = float((g1[k] - g0[k]).norm()), float(g0[k].norm())
        assert err <= 1e-4 * nrm + 1e-6 * rms0 * g0[k].numel() ** 0.5, (k, err, nrm)
    # fp64 oracle on the same (shuffled) edge_index
    torch.manual_seed(0)
    sd = bgnn.BuckGNN(16, 5, hidden_channels=512, num_layers=6, dropout_rate=0.0, model_name=model_name).state_dict()
    st = {k: v.double().clone().requires_grad_(v.is_floating_point() and "running" not in k
                                               and "num_batches" not in k) for k, v in sd.items()}
    pred_o = R.forward(st, model_name, b.x.double(), ei, b.batch, True, "mean", 0.0)
    R.relative_error_loss(pred_o, b.y.double()).backward()
    np.testing.assert_allclose(p1.cpu().double().numpy(), pred_o.detach().numpy(), rtol=1e-4, atol=1e-4)
    ref = {k: v.grad for k, v in st.items() if v.grad is not None}
    assert set(ref) == set(g1)
    rms = max(float(v.pow(2).mean().sqrt()) for v in ref.values())
    for k, r in ref.items():
        err = float((g1[k].cpu().double() - r).norm())
        assert err <= 1e-3 * float(r.norm()) + 1e-5 * rms * r.numel() ** 0.5, (k, err, float(r.norm()))
