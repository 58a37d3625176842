"""GPU: bf16 storage of EA_GNN's per-edge activations (BASELINE configs[4], the bf16
configuration): the bf16-operand GEMM with bf16 A / B / C storage (bgnn_gemm_bf16, the gathered
epilogue bgnn_gemm_gather_add_bf16), the bf16 skip + dropout pass and the bf16 segment sums,
each against a torch reference on the same bf16-rounded data. Whole-block error against the f32
block is pinned by tests/test_gpu_model.py::test_ea_gnn_bf16_block_close_to_f32 (within 1.5x of
torch autocast-bf16's) and the training trajectory by tests/test_gpu_ea_train.py."""
import pytest
import torch

from bgnn import _lib, ea, fused
from bgnn import synthetic as S
from bgnn.graph import SegmentIndex
from bgnn.ops import segment_reduce

pytestmark = pytest.mark.gpu


def _ref(a, b, ta, tb, bias=None, relu=False):
    A = a.to(torch.bfloat16).double()
    B = b.to(torch.bfloat16).double()
    c = (A.t() if ta else A) @ (B.t() if tb else B)
    if bias is not None:
        c = c + bias.double()
    return c.clamp_min(0) if relu else c


@pytest.mark.parametrize("ta,tb,storage", [(0, 1, 0), (0, 1, 1), (0, 1, 4), (0, 1, 5), (1, 0, 1), (1, 0, 2),
                                           (1, 0, 3)])
@pytest.mark.parametrize("mnk", [(1000, 256, 128), (4099, 512, 512)])
def test_gemm_bf16_storage(dev, ta, tb, storage, mnk):
    M, N, K = mnk
    torch.manual_seed(storage + M)
    a = torch.randn(*((K, M) if ta else (M, K)), device=dev)
    b = torch.randn(*((N, K) if tb else (K, N)), device=dev) / K ** 0.5
    if storage & 1:
        a = a.to(torch.bfloat16)
    if storage & 2:
        b = b.to(torch.bfloat16)
    bias = torch.randn(N, device=dev) if ta == 0 else None
    out = fused.gemm_bf16(a, b, bool(ta), bool(tb), out_bf16=bool(storage & 4), bias=bias, relu=ta == 0)
    ref = _ref(a.float(), b.float(), ta, tb, bias, ta == 0)
    assert out.dtype == (torch.bfloat16 if storage & 4 else torch.float32)
    scale = (a.float().abs().max() * b.float().abs().max() * K).item()
    if storage & 4:   # the result is one bf16 rounding of the f32-accumulated product
        torch.testing.assert_close(out.float(), ref.float().to(torch.bfloat16).float(), rtol=1e-2, atol=1e-6 * scale)
    else:
        assert (out.double() - ref).abs().max().item() <= 2e-6 * scale


def test_gather_add_bf16_storage_matches_f32_storage(dev):
    """bf16 A and C storage in the gathered epilogue: C = one bf16 rounding of the f32-stored
    result (same bf16 operands, same accumulation)."""
    b = S.make_batch(20, 3).to(dev)
    N, E, H = b.num_nodes, b.num_edges, 256
    torch.manual_seed(1)
    e = torch.randn(E, H, device=dev).to(torch.bfloat16)
    W = torch.randn(H, H, device=dev) / H ** 0.5
    bias = torch.randn(H, device=dev)
    P1 = torch.randn(N, H, device=dev)
    seg_row, seg_col = ea.edge_segments(b.edge_index, N)
    ref = ea._LinearGatherReLU.apply(e.float(), W, bias, P1, seg_row, None, None, True, False)
    out = ea._LinearGatherReLU.apply(e, W, bias, P1, seg_row, None, None, True, True)
    assert out.dtype == torch.bfloat16
    assert torch.equal(out, ref.to(torch.bfloat16))


def test_add_dropout_bf16_same_mask(dev):
    n = 4096 * 8
    ones = torch.ones(n, device=dev)
    f = ea._add_dropout(ones, None, 0.3, 1234)
    h = ea._add_dropout(ones.to(torch.bfloat16), None, 0.3, 1234)
    assert torch.equal(f != 0, h != 0)                                   # the same counter-based mask
    a = torch.randn(n, device=dev).to(torch.bfloat16)
    c = torch.randn(n, device=dev).to(torch.bfloat16)
    out = ea._add_dropout(a, c, 0.3, 99)
    ref = ea._add_dropout(a.float(), c.float(), 0.3, 99).to(torch.bfloat16)
    assert torch.equal(out, ref)


@pytest.mark.parametrize("reduce", ["sum", "mean"])
def test_segment_reduce_bf16(dev, reduce):
    b = S.make_batch(15, 3).to(dev)
    N, E, H = b.num_nodes, b.num_edges, 512
    seg = SegmentIndex.build(b.edge_index[0], N)
    torch.manual_seed(2)
    x = torch.randn(E, H, device=dev).to(torch.bfloat16).requires_grad_(True)
    out = segment_reduce(x, seg, reduce)
    xr = x.detach().double().requires_grad_(True)
    ref = torch.zeros(N, H, dtype=torch.float64, device=dev).index_add_(0, b.edge_index[0], xr)
    if reduce == "mean":
        ref = ref / torch.bincount(b.edge_index[0], minlength=N).clamp_min(1).double().unsqueeze(1)
    torch.testing.assert_close(out.double(), ref, rtol=1e-5, atol=1e-5)
    g = torch.randn(N, H, device=dev)
    out.backward(g)
    ref.backward(g.double())
    assert x.grad.dtype == torch.bfloat16
    torch.testing.assert_close(x.grad.float(), xr.grad.float().to(torch.bfloat16).float(), rtol=1e-2, atol=1e-6)
    # the backward kernel (bgnn_segment_bcast_bf16) is torch's (g / cnt).to(bfloat16).index_select,
    # bit for bit (f32 division, one round-to-nearest-even)
    gg = g / seg.fwd.degree().clamp_min(1).to(g.dtype).unsqueeze(1) if reduce == "mean" else g
    assert torch.equal(x.grad, gg.to(torch.bfloat16).index_select(0, seg.index))


@pytest.fixture
def b16_variant():
    """set bgnn_gemm_b16_variant for one test; restore the default (0) afterwards"""
    def set_(v):
        _lib.call("bgnn_gemm_b16_variant", v)
    yield set_
    _lib.call("bgnn_gemm_b16_variant", 0)


@pytest.mark.parametrize("mnk", [(1000, 256, 128), (4099, 512, 512), (300, 200, 64), (70001, 512, 512)])
@pytest.mark.parametrize("c16", [False, True], ids=["f32C", "bf16C"])
@pytest.mark.parametrize("gather", [False, True], ids=["plain", "gather"])
def test_b16_kernel_bit_identical_to_register_staged(dev, b16_variant, mnk, c16, gather):
    """bf16-stored A and B (storage 3 / 7, the EA_GNN edge products): the LDS-DMA kernel
    (gemm_b16.hip: 256 x 256 tiles, whole-line bf16 C stores, gather indices in LDS) equals the
    register-staged k_gemm_x6 bit for bit -- bias, gathered node rows, ReLU, f32 or bf16 C, ragged
    M and N -- and the register-staged result is the bf16-operand product (fp64 reference on the
    same bf16 operands)."""
    M, N, K = mnk
    torch.manual_seed(M + N)
    a = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16)
    bias = torch.randn(N, device=dev)
    nn_ = 997
    p1, p2 = torch.randn(nn_, N, device=dev), torch.randn(nn_, N, device=dev)
    i1 = torch.sort(torch.randint(0, nn_, (M,), device=dev))[0]
    i2 = torch.randint(0, nn_, (M,), device=dev)
    st = 3 | (4 if c16 else 0)

    def run():
        # NaN-filled: a variant that leaves part of C unwritten cannot pass on stale bytes
        out = torch.full((M, N), float("nan"), dtype=torch.bfloat16 if c16 else torch.float32, device=dev)
        if gather:
            _lib.call("bgnn_gemm_gather_add_bf16", M, N, K, a.data_ptr(), K, w.data_ptr(), K, out.data_ptr(), N,
                      bias.data_ptr(), 1, p1.data_ptr(), i1.data_ptr(), N, p2.data_ptr(), i2.data_ptr(), N, st, None, 0,
                      torch.cuda.current_stream().cuda_stream)
        else:
            fused.gemm_bf16(a, w, False, True, out=out, bias=bias, relu=True)
        return out

    b16_variant(-1)
    ref = run()
    b16_variant(0)
    assert torch.equal(run(), ref)
    exact = a.double() @ w.double().t() + bias.double()
    if gather:
        exact = exact + p1.double()[i1] + p2.double()[i2]
    exact = exact.clamp_min(0)
    scale = float(a.float().abs().max() * w.float().abs().max() * K) + 10.0
    if c16:
        torch.testing.assert_close(ref.float(), exact.float().to(torch.bfloat16).float(), rtol=1e-2, atol=1e-6 * scale)
    else:
        assert (ref.double() - exact).abs().max().item() <= 2e-6 * scale


def test_b16_weight_rounding_matches_in_tile_rounding(dev, b16_variant):
    """fused.gemm_bf16 rounds an f32 weight to bf16 once for a bf16-stored A (so the LDS-DMA
    kernel runs): the result equals the register-staged kernel rounding the f32 weight in-tile."""
    torch.manual_seed(5)
    a = torch.randn(5000, 512, device=dev).to(torch.bfloat16)
    w = torch.randn(384, 512, device=dev) / 512 ** 0.5
    got = fused.gemm_bf16(a, w, False, True, out_bf16=True)
    fused.B16_WEIGHTS = False
    try:
        b16_variant(-1)
        ref = fused.gemm_bf16(a, w, False, True, out_bf16=True)
    finally:
        fused.B16_WEIGHTS = True
    assert torch.equal(got, ref)


@pytest.mark.parametrize("relu", [True, False])
@pytest.mark.parametrize("shape", [(3001, 512), (777, 64), (5, 2048)])
def test_linear_bwd_prep_bf16_matches_torch(dev, relu, shape):
    """bgnn_linear_bwd_prep_bf16 (fused.relu_bias_grad_bf16): the ReLU-masked gradient is
    bit-identical to torch's threshold_backward on the same bf16 data (zeros, negative zeros and
    exact-zero outputs included) and the f32 bias-gradient sums match an fp64 sum of it."""
    torch.manual_seed(21)
    N, C = shape
    g = torch.randn(N, C, device=dev).to(torch.bfloat16)
    y = torch.randn(N, C, device=dev).clamp_min(0).to(torch.bfloat16)   # a ReLU output: many exact zeros
    y[::7, ::3] = -0.0
    ref_g = torch.ops.aten.threshold_backward(g, y, 0.0) if relu else g
    got_g, db = fused.relu_bias_grad_bf16(g, y if relu else None, True)
    assert got_g.dtype == torch.bfloat16
    assert torch.equal(got_g, ref_g)
    ref_db = ref_g.double().sum(0)
    torch.testing.assert_close(db.double(), ref_db, rtol=1e-5, atol=1e-4 * (1 + ref_db.abs().max().item()) * 1e-2)
    g2, none = fused.relu_bias_grad_bf16(g, y if relu else None, False)
    assert none is None and torch.equal(g2, ref_g)


def test_absmax_items_matches_per_item(dev):
    """bgnn_absmax_items_f32 (all layers' max|[W_l;W_r]| of a SAGE loop in one launch) folds the
    same maxima into the strided slots as one bgnn_absmax per item."""
    torch.manual_seed(22)
    L, H = 6, 512
    W = torch.randn(L, 2 * H, H, device=dev) * torch.logspace(-3, 3, L, device=dev).view(L, 1, 1)
    bufs = torch.zeros(L, 3, device=dev)
    bufs[2, 0] = 1e9   # accumulate: an existing larger value stays
    _lib.call("bgnn_absmax_items_f32", W.data_ptr(), L, 2 * H * H, 2 * H, H, H, bufs.data_ptr(), 3,
              torch.cuda.current_stream().cuda_stream)
    want = W.abs().amax(dim=(1, 2))
    want[2] = 1e9
    assert torch.equal(bufs[:, 0], want)
    assert torch.equal(bufs[:, 1:], torch.zeros(L, 2, device=dev))


@pytest.mark.parametrize("p", [0.0, 0.1, 0.5])
def test_add_dropped_bf16_matches_dropout_then_add(dev, p):
    """bgnn_add_dropped_bf16 (a + drop(b), EA_GNN's edge-gradient hand-off): drop(b) uses the same
    mask as bgnn_add_dropout_bf16 for (p, seed); one f32 sum, one bf16 rounding; in place on a."""
    torch.manual_seed(31)
    n = 4096 * 8 + 64
    a = torch.randn(n, device=dev).to(torch.bfloat16)
    b = torch.randn(n, device=dev).to(torch.bfloat16)
    s = torch.cuda.current_stream().cuda_stream
    db = torch.empty_like(b)
    _lib.call("bgnn_add_dropout_bf16", b.data_ptr(), None, n, float(p), 1234, db.data_ptr(), s)
    ref = (a.float() + db.float()).to(torch.bfloat16)
    out = a.clone()
    _lib.call("bgnn_add_dropped_bf16", out.data_ptr(), b.data_ptr(), n, float(p), 1234, out.data_ptr(), s)
    # drop(b) rounded to bf16 first in the reference: equal up to that one rounding
    torch.testing.assert_close(out.float(), ref.float(), rtol=1e-2, atol=1e-2)
    dropped = db == 0   # dropped (or zero) elements of b leave a unchanged, exactly
    assert torch.equal(out[dropped], a[dropped])
    if p > 0:
        assert 0.5 * p < dropped.float().mean().item() < 1.5 * p
    if p == 0.0:
        assert torch.equal(out, ref)


def test_rel_error_loss_kernel_matches_torch(dev):
    """bgnn_rel_error_loss (train_step's fused RelativeErrorLoss on EigenvalueScaler-denormalised
    values, Utils/Losses.py:755-761): loss and d loss / d pred equal torch autograd's on the same
    denormalisation, to f32 rounding."""
    from bgnn import train as T
    torch.manual_seed(32)
    pred = torch.randn(16, 1, device=dev, requires_grad=True)
    y = torch.randn(16, 1, device=dev)
    y[3] = -0.5 / 2.0   # a target whose denormalised value is 0 (eps in the denominator)
    crit, norm = T.RelativeErrorLoss(), T.EigenvalueScaler(center=0.5, scale=2.0)
    ref = crit(norm.denormalize_eigenvalue(pred), norm.denormalize_eigenvalue(y))
    (gref,) = torch.autograd.grad(ref, pred)
    p2 = pred.detach().clone().requires_grad_(True)
    got = T._fused_loss(crit, norm, p2, y)
    assert got is not None
    (ggot,) = torch.autograd.grad(got * 3.0, p2)
    torch.testing.assert_close(got, ref, rtol=1e-6, atol=0)
    torch.testing.assert_close(ggot, 3.0 * gref, rtol=1e-6, atol=0)
    assert T._fused_loss(crit, norm, p2, y.view(-1)) is None   # broadcasting shapes: torch path


def test_rel_error_loss_kernel_nan_like_torch(dev):
    """A NaN prediction: the fused loss is NaN (the divergence signal) and its gradient is what
    torch's autograd of the reference loss gives -- 0 in the NaN position (torch.abs backward
    multiplies by sgn(x), and sgn(NaN) = 0), the other positions unchanged."""
    from bgnn import train as T
    pred = torch.tensor([0.3, float("nan"), -0.7, 1.1], device=dev, requires_grad=True)
    y = torch.tensor([0.5, 0.4, -0.2, 1.0], device=dev)
    crit, norm = T.RelativeErrorLoss(), T.EigenvalueScaler(center=0.5, scale=2.0)
    got = T._fused_loss(crit, norm, pred, y)
    (g,) = torch.autograd.grad(got, pred)
    ref = crit(norm.denormalize_eigenvalue(pred), norm.denormalize_eigenvalue(y))
    (gref,) = torch.autograd.grad(ref, pred)
    assert torch.isnan(got) and torch.isnan(ref)
    assert g[1].item() == gref[1].item() == 0.0
    torch.testing.assert_close(g[[0, 2, 3]], gref[[0, 2, 3]], rtol=1e-6, atol=0)


@pytest.mark.parametrize("mnk", [(1000, 512, 512), (70001, 512, 512), (4099, 256, 128), (300, 256, 96)])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_gemm_bf16_dropadd_bit_identical_to_two_steps(dev, b16_variant, mnk, p):
    """bgnn_gemm_bf16_dropadd (EA_GNN's edge Linear dgrad + the skip + dropout's gradient of the same
    activation, ea.GradSlot.gemm_dropadd): the drop-add in the LDS-DMA kernel's epilogue equals
    bgnn_gemm_bf16 (bf16 C) followed by bgnn_add_dropped_bf16 on the stored C, bit for bit -- ragged
    M (the last row tile), N = 256 / 512, K % 64 != 0 (the two-step fallback), with the LDS-DMA
    kernel (the fused add) and with the register-staged kernel (the two steps)."""
    M, N, K = mnk
    torch.manual_seed(M + K)
    a = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16)
    src = torch.randn(M, N, device=dev).to(torch.bfloat16)
    s = torch.cuda.current_stream().cuda_stream

    def fused_():
        out = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device=dev)
        _lib.call("bgnn_gemm_bf16_dropadd", M, N, K, a.data_ptr(), K, w.data_ptr(), K, out.data_ptr(), N,
                  src.data_ptr(), N, float(p), 77, s)
        return out

    ref = fused.gemm_bf16(a, w, False, True, out_bf16=True)
    _lib.call("bgnn_add_dropped_bf16", ref.data_ptr(), src.data_ptr(), M * N, float(p), 77, ref.data_ptr(), s)
    for v in (0, -1):
        b16_variant(v)
        assert torch.equal(fused_(), ref), v
