"""GPU: bgnn_gemm_f32 (f32 MFMA and f16x3 kernel families) against an fp64 torch
reference, all transposes, ragged shapes, split-K, beta accumulation, operand scaling."""
import pytest
import torch

from bgnn import _lib, fused

pytestmark = pytest.mark.gpu


DEFAULT_MODE = 2


@pytest.fixture(params=[0, 2], ids=["f32", "h3"])
def mode(request):
    """GEMM kernel family: 0 = f32 MFMA, 2 = f16x3 (BGNN_TUNE_GEMM_MODE)."""
    _lib.call("bgnn_set_tuning", 5, request.param)
    yield request.param
    _lib.call("bgnn_set_tuning", 5, DEFAULT_MODE)


def test_default_mode_is_f16x3():
    assert _lib.query("bgnn_get_tuning", 5) == DEFAULT_MODE


def ref(a, b, ta, tb):
    A = a.double().cpu()
    B = b.double().cpu()
    return (A.t() if ta else A) @ (B.t() if tb else B)


@pytest.mark.parametrize("ta", [False, True])
@pytest.mark.parametrize("tb", [False, True])
@pytest.mark.parametrize("mnk", [(1, 1, 1), (37, 129, 15), (300, 200, 64), (128, 128, 128), (513, 1024, 512),
                                 (1024, 512, 9000)])
def test_gemm_matches_fp64(dev, mode, ta, tb, mnk):
    M, N, K = mnk
    torch.manual_seed(M + N + K)
    a = torch.randn((K, M) if ta else (M, K), device=dev)
    b = torch.randn((N, K) if tb else (K, N), device=dev)
    c = fused.gemm(a, b, ta, tb)
    r = ref(a, b, ta, tb)
    err = (c.double().cpu() - r).abs().max().item()
    scale = (a.abs().double().cpu().max() * b.abs().double().cpu().max() * K).item()
    assert err <= 2e-6 * scale + 1e-6, (err, scale)


def test_gemm_beta_accumulates_and_strided_views(dev, mode):
    torch.manual_seed(0)
    big = torch.randn(200, 64, device=dev)
    a = big[:, 32:]            # strided rows (ld = 64)
    w = torch.randn(48, 32, device=dev)
    c0 = torch.randn(200, 48, device=dev)
    c = c0.clone()
    fused.gemm(a, w, False, True, out=c, beta=1.0)
    r = c0.double().cpu() + a.double().cpu() @ w.double().cpu().t()
    torch.testing.assert_close(c.double().cpu(), r, rtol=1e-5, atol=1e-4)


def test_gemm_is_deterministic(dev, mode):
    a = torch.randn(4000, 1024, device=dev)
    b = torch.randn(4000, 512, device=dev)
    c1 = fused.gemm(a, b, True, False)
    c2 = fused.gemm(a, b, True, False)
    assert torch.equal(c1, c2)


@pytest.mark.parametrize("blk", [128, 256, 512])
@pytest.mark.parametrize("N", [64, 1000, 20000])
def test_gemm_planes_layouts(dev, mode, blk, N):
    """Plane-split operands (fused.Planes) give bit-identical results to the dense layout:
    C planes (forward), A planes split along K (dgrad) and along M (wgrad, split-K)."""
    torch.manual_seed(blk + N)
    H = blk
    x = torch.randn(N, H, device=dev)
    w = torch.randn(2 * H, H, device=dev)
    # forward: z = x w^T into planes
    zp = torch.empty(2, N, H, device=dev)
    fused.gemm(x, w, False, True, out=fused.Planes(zp))
    zd = fused.gemm(x, w, False, True)
    r = x.double().cpu() @ w.double().cpu().t()
    assert (zd.double().cpu() - r).abs().max().item() <= 2e-6 * 16 * H + 1e-6
    torch.testing.assert_close(fused.Planes(zp).dense(), zd, rtol=0, atol=0)
    # dgrad: dx = dz w with dz in planes
    dzp = torch.randn(2, N, H, device=dev)
    dzd = fused.Planes(dzp).dense().contiguous()
    g0 = torch.randn(N, H, device=dev)
    a1, a2 = g0.clone(), g0.clone()
    fused.gemm(fused.Planes(dzp), w, False, False, out=a1, beta=1.0)
    fused.gemm(dzd, w, False, False, out=a2, beta=1.0)
    torch.testing.assert_close(a1, a2, rtol=0, atol=0)
    # wgrad: dw = dz^T x with dz in planes (planes split M)
    w1 = fused.gemm(fused.Planes(dzp), x, True, False)
    w2 = fused.gemm(dzd, x, True, False)
    torch.testing.assert_close(w1, w2, rtol=0, atol=0)
    rw = dzd.double().cpu().t() @ x.double().cpu()
    assert (w1.double().cpu() - rw).abs().max().item() <= 2e-6 * 16 * N + 1e-5


def _err_class(a, b, ta, tb, modes):
    A = a.double().t() if ta else a.double()
    B = b.double().t() if tb else b.double()
    c64, mag = A @ B, A.abs() @ B.abs()
    errs = []
    for m in modes:
        _lib.call("bgnn_set_tuning", 5, m)
        try:
            c = fused.gemm(a, b, ta, tb)
        finally:
            _lib.call("bgnn_set_tuning", 5, DEFAULT_MODE)
        errs.append(((c.double() - c64).abs() / mag.clamp_min(1e-300)).max().item())
    return errs


@pytest.mark.parametrize("ta,tb", [(False, True), (False, False), (True, False)])
def test_gemm_error_class_per_element(dev, ta, tb):
    """Per-element error bound max |c - c64| / (|A||B|) of the two kernel families on a
    SAGE-like shape: the f16x3 split is in the f32 MFMA's error class (f32 unit roundoff 6e-8
    times a small factor: the f32 accumulation dominates), far below the 1e-4 parity tolerance."""
    torch.manual_seed(5)
    M, N, K = 3000, 512, 1024
    a = torch.randn((K, M) if ta else (M, K), device=dev)
    b = torch.randn((N, K) if tb else (K, N), device=dev) * 0.03
    errs = _err_class(a, b, ta, tb, (0, 2))
    assert max(errs) < 1e-6, errs
    assert errs[1] < 4 * errs[0] + 1e-7, errs


@pytest.mark.parametrize("ta,tb", [(False, True), (True, False)])
def test_gemm_f16x3_row_magnitudes_spread(dev, ta, tb):
    """f16x3 scales per tensor: rows spanning six decades (and relu zeros) keep f32-class
    per-element error relative to |A||B|."""
    torch.manual_seed(6)
    M, N, K = 2000, 256, 512
    a = torch.randn(M, K, device=dev) * torch.pow(10.0, -6 * torch.rand(M, 1, device=dev))
    a = a.clamp_min(0) if ta else a
    a = a.t().contiguous() if ta else a
    b = torch.randn((N, K) if tb else (K, N), device=dev)
    errs = _err_class(a, b, ta, tb, (0, 2))
    assert errs[1] < 2e-6, errs


@pytest.mark.parametrize("scale", [1e-30, 1e-12, 1.0, 1e12, 1e30])
def test_gemm_f16x3_extreme_magnitudes(dev, scale):
    """Operand scales are powers of two chosen from max|A|, max|B|: tensors far outside the
    f16 range (both ways) multiply at f32-class accuracy; zero operands give exact zeros."""
    torch.manual_seed(7)
    a = torch.randn(300, 200, device=dev) * scale
    b = torch.randn(100, 200, device=dev) / scale ** 0.5
    errs = _err_class(a, b, False, True, (2,))
    assert errs[0] < 2e-6, errs
    z = fused.gemm(torch.zeros(64, 32, device=dev), b[:, :32].contiguous(), False, True)
    assert bool((z == 0).all())


def test_absmax_and_supplied_maxima(dev):
    """bgnn_absmax_f32 matches torch; bgnn_gemm_f32_scaled with supplied maxima equals the
    self-scaled call bit for bit (maxima computed inside from the same data)."""
    torch.manual_seed(8)
    x = torch.randn(1000, 96, device=dev)
    x[123, 45] = -77.5
    out = torch.full((1,), 3.0, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    _lib.call("bgnn_absmax_f32", x.data_ptr(), 1000, 96, 96, out.data_ptr(), 0, s)
    assert out.item() == 77.5
    _lib.call("bgnn_absmax_f32", x[:, :50].data_ptr(), 1000, 50, 96, out.data_ptr(), 1, s)
    assert out.item() == 77.5
    w = torch.randn(64, 96, device=dev)
    amax = torch.stack([x.abs().max(), w.abs().max()]).contiguous()
    c1 = fused.gemm(x, w, False, True)
    c2 = torch.empty_like(c1)
    ws_bytes = _lib.query("bgnn_gemm_ws_bytes", 1000, 64, 96, 0, 1)
    ws = torch.empty(max(ws_bytes, 256), dtype=torch.uint8, device=dev)
    _lib.call("bgnn_gemm_f32_scaled", 0, 1, 1000, 64, 96, 1.0, x.data_ptr(), 96, 0, 0, w.data_ptr(), 96, 0.0,
              c2.data_ptr(), 64, 0, 0, None, 0, amax[0:].data_ptr(), amax[1:].data_ptr(), None, 0, ws.data_ptr(),
              ws.numel(), s)
    torch.testing.assert_close(c1, c2, rtol=0, atol=0)


@pytest.mark.parametrize("shape", [(1000, 64, 96, 0, 1), (1000, 37, 96, 0, 1), (512, 256, 9000, 1, 0)])
def test_gemm_c_amax(dev, mode, shape):
    """c_amax = max |C| of the result, fused into the epilogue (split kernels, no split-K) or one
    extra pass (f32 kernel, split-K); folds into the running value; bias/ReLU applied first."""
    M, N, K, ta, tb = shape
    torch.manual_seed(9)
    a = torch.randn((K, M) if ta else (M, K), device=dev)
    b = torch.randn((N, K) if tb else (K, N), device=dev)
    bias = torch.randn(N, device=dev)
    c = torch.empty(M, N, device=dev)
    cm = torch.full((1,), 0.5, device=dev)
    ws_bytes = _lib.query("bgnn_gemm_ws_bytes", M, N, K, ta, tb)
    ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    _lib.call("bgnn_gemm_f32_scaled", ta, tb, M, N, K, 1.0, a.data_ptr(), a.stride(0), 0, 0, b.data_ptr(), b.stride(0),
              0.0, c.data_ptr(), N, 0, 0, bias.data_ptr(), 1, None, None, cm.data_ptr(), 0, ws.data_ptr(), ws_bytes, s)
    assert cm.item() == c.abs().max().item()
    assert bool((c >= 0).all())


@pytest.mark.parametrize("ta,tb,mnk", [(False, True, (1500, 384, 2000)), (False, False, (1500, 384, 2000)),
                                       (True, False, (1500, 384, 2000)),
                                       # shapes whose plan picks the 256x256 tiles (cfg 3/4): the EA_GNN
                                       # node-block GEMM (N >= 1024) and a split-K weight gradient
                                       (False, True, (4500, 1536, 512)), (True, False, (512, 256, 20000))])
def test_gemm_bf16_precision(dev, ta, tb, mnk):
    """precision = 1: operands rounded to bf16, f32 accumulation -- equal to an fp64 product of the
    bf16-rounded operands up to the f32 accumulation error, over EVERY output element (the output
    is pre-filled with NaN: an element the kernel never writes fails)."""
    torch.manual_seed(10)
    M, N, K = mnk
    a = torch.randn((K, M) if ta else (M, K), device=dev)
    b = torch.randn((N, K) if tb else (K, N), device=dev)
    c = torch.full((M, N), float("nan"), device=dev)
    fused.gemm(a, b, ta, tb, out=c, bf16=True)
    assert bool(torch.isfinite(c).all())
    A = a.bfloat16().double().cpu()
    B = b.bfloat16().double().cpu()
    A = A.t() if ta else A
    B = B.t() if tb else B
    r, mag = A @ B, A.abs() @ B.abs()
    assert ((c.double().cpu() - r).abs() / mag).max().item() < 2e-6


def _wsplit(w, w_amax, M):
    """Pre-split image of the weight operand W [N, K] for the C = A W^T shape (M, N, K)."""
    N, K = w.shape
    bn = _lib.query("bgnn_gemm_w_tile", M, N, K)
    assert bn in (128, 256), (M, N, K, bn)
    img = torch.empty(_lib.query("bgnn_gemm_wsplit_bytes", N, K), dtype=torch.uint8, device=w.device)
    _lib.call("bgnn_gemm_wsplit", w.data_ptr(), 1, 0, N, K, w.stride(0), w_amax.data_ptr(), 0, img.data_ptr(),
              img.numel(), bn, fused._stream())
    return img, bn


# the SAGE layer shapes (forward, input gradient, the folded layer's K = 128 / N = 128 forms) with a
# ragged last row tile (M % BM != 0), and a small M
@pytest.mark.parametrize("M,N,K", [(80656, 1024, 512), (80656, 512, 1024), (80656, 1024, 128), (80656, 128, 1024),
                                   (1000, 512, 1024), (4097, 1024, 512)])
@pytest.mark.parametrize("dropadd", [False, True])
@pytest.mark.parametrize("cfg", [-1, 1, 2])
@pytest.mark.parametrize("bdma", [0, 2, 3])
def test_gemm_presplit_weights_bit_identical(dev, M, N, K, dropadd, cfg, bdma):
    """bgnn_gemm_wsplit + bgnn_gemm_f32_w (the weight operand pre-split once, its image copied into
    LDS) produce exactly the bits of bgnn_gemm_f32_scaled / bgnn_gemm_f32_dropadd on the same
    operands and maxima (the LDS image is the one the register-staged kernel writes), with bias,
    ReLU and max|C| in the plain epilogue and the masked beta source in the drop-add epilogue; on
    the planned tile (cfg -1) and forced 256 x 128 / 128 x 256 tiles; for every B staging of knob 16
    (register copy, and the pipelined kernel gemm_h3p.hip with 3 / 4 slots, which the 128 x 256 tile
    runs: ragged last row tiles, K = 128's four slices)."""
    torch.manual_seed(M + N + K)
    a = torch.randn(M, K, device=dev)
    w = torch.randn(N, K, device=dev) * 0.03
    am = torch.stack([a.abs().max(), w.abs().max()]).contiguous()
    default_bdma = _lib.query("bgnn_get_tuning", 16)
    _lib.call("bgnn_gemm_set_cfg", cfg)
    _lib.call("bgnn_set_tuning", 16, bdma)
    try:
        if _lib.query("bgnn_gemm_w_tile", M, N, K) == 0:
            pytest.skip("no pre-split path for this shape and tile")
        img, bn = _wsplit(w, am[1:2], M)
    finally:
        _lib.call("bgnn_gemm_set_cfg", -1)
        _lib.call("bgnn_set_tuning", 16, default_bdma)

    def run_w(*args):
        _lib.call("bgnn_gemm_set_cfg", cfg)
        _lib.call("bgnn_set_tuning", 16, bdma)
        try:
            _lib.call("bgnn_gemm_f32_w", *args)
        finally:
            _lib.call("bgnn_gemm_set_cfg", -1)
            _lib.call("bgnn_set_tuning", 16, default_bdma)
    if dropadd:
        src = torch.randn(M, N, device=dev)
        ref = torch.empty(M, N, device=dev)
        ws_bytes = _lib.query("bgnn_gemm_ws_bytes_ex", M, N, K, 0, 1, 0)
        ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
        _lib.call("bgnn_gemm_f32_dropadd", 0, 1, M, N, K, a.data_ptr(), K, w.data_ptr(), K, ref.data_ptr(), N,
                  am[0:1].data_ptr(), am[1:2].data_ptr(), src.data_ptr(), N, 0.1, 1234, ws.data_ptr(), ws_bytes,
                  fused._stream())
        out = torch.full((M, N), float("nan"), device=dev)
        run_w(M, N, K, a.data_ptr(), K, img.data_ptr(), bn, out.data_ptr(), N, None, 0,
              am[0:1].data_ptr(), am[1:2].data_ptr(), None, src.data_ptr(), N, 0.1, 1234, fused._stream())
        assert torch.equal(out, ref)
        return
    bias = torch.randn(N, device=dev)
    ca_ref = torch.zeros(1, device=dev)
    ref = fused.gemm(a, w, False, True, bias=bias, relu=True, a_amax=am[0:1], b_amax=am[1:2], c_amax=ca_ref)
    out = torch.full((M, N), float("nan"), device=dev)
    ca = torch.zeros(1, device=dev)
    run_w(M, N, K, a.data_ptr(), K, img.data_ptr(), bn, out.data_ptr(), N, bias.data_ptr(), 1,
          am[0:1].data_ptr(), am[1:2].data_ptr(), ca.data_ptr(), None, 0, 0.0, 0, fused._stream())
    assert torch.equal(out, ref)
    assert torch.equal(ca, ca_ref)


def test_gemm_presplit_rejects_mismatched_tile(dev):
    """An image split with the wrong column tile is refused (no silent misread)."""
    M, N, K = 80656, 512, 1024
    w = torch.randn(N, K, device=dev)
    am = w.abs().max().view(1)
    bn = _lib.query("bgnn_gemm_w_tile", M, N, K)
    wrong = 128 if bn == 256 else 256
    img = torch.empty(_lib.query("bgnn_gemm_wsplit_bytes", N, K), dtype=torch.uint8, device=dev)
    a = torch.randn(M, K, device=dev)
    out = torch.empty(M, N, device=dev)
    with pytest.raises(_lib.BgnnError):
        _lib.call("bgnn_gemm_f32_w", M, N, K, a.data_ptr(), K, img.data_ptr(), wrong, out.data_ptr(), N, None, 0,
                  am.data_ptr(), am.data_ptr(), None, None, 0, 0.0, 0, fused._stream())


@pytest.mark.parametrize("M", [80656, 1000])
def test_gemm_dropadd_cols_bit_identical(dev, M):
    """bgnn_gemm_f32_dropadd_cols (the max layer's merged input gradient [dh W_l | dh W_r + drop(g)]):
    the columns left of src_col0 are exactly the plain product and the rest exactly
    bgnn_gemm_f32_dropadd of the right block with src (its own mask indices)."""
    torch.manual_seed(M)
    C, H = 512, 512
    a = torch.randn(M, H, device=dev)
    w = torch.randn(2 * C, H, device=dev) * 0.03
    src = torch.randn(M, C, device=dev)
    am = torch.stack([a.abs().max(), w.abs().max()]).contiguous()
    out = torch.full((M, 2 * C), float("nan"), device=dev)
    ws_bytes = _lib.query("bgnn_gemm_ws_bytes_ex", M, 2 * C, H, 0, 1, 0)
    ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
    _lib.call("bgnn_gemm_f32_dropadd_cols", M, 2 * C, H, a.data_ptr(), H, w.data_ptr(), H, out.data_ptr(), 2 * C,
              am[0:1].data_ptr(), am[1:2].data_ptr(), src.data_ptr(), C, C, 0.1, 77, ws.data_ptr(), ws_bytes,
              fused._stream())
    left = fused.gemm(a, w[:C].contiguous(), False, True, a_amax=am[0:1], b_amax=am[1:2])
    right = torch.empty(M, C, device=dev)
    ws2_bytes = _lib.query("bgnn_gemm_ws_bytes_ex", M, C, H, 0, 1, 0)
    ws2 = torch.empty(max(ws2_bytes, 1), dtype=torch.uint8, device=dev)
    wr = w[C:].contiguous()
    _lib.call("bgnn_gemm_f32_dropadd", 0, 1, M, C, H, a.data_ptr(), H, wr.data_ptr(), H, right.data_ptr(), C,
              am[0:1].data_ptr(), am[1:2].data_ptr(), src.data_ptr(), C, 0.1, 77, ws2.data_ptr(), ws2_bytes,
              fused._stream())
    assert torch.equal(out[:, :C], left)
    assert torch.equal(out[:, C:], right)
    with pytest.raises(_lib.BgnnError):   # the addend must start on a column tile
        _lib.call("bgnn_gemm_f32_dropadd_cols", M, 2 * C, H, a.data_ptr(), H, w.data_ptr(), H, out.data_ptr(),
                  2 * C, am[0:1].data_ptr(), am[1:2].data_ptr(), src.data_ptr(), C, 100, 0.1, 77, ws.data_ptr(),
                  ws_bytes, fused._stream())


# tall N = 128 products (the folded layer's input gradient dh = dz Wf, 80656 x 128 x 1024; the
# encoder's last Linear) plan the 8-wave 128 x 128 tile (cfg 5): the same 16x16x32 MFMAs per
# element in the same k order as the 256 x 128 tile, so the same bits, with the plain epilogue's
# bias / ReLU / max|C| and the drop-add epilogue; ragged last row tiles included
@pytest.mark.parametrize("M,K", [(80656, 1024), (80656, 64), (4100, 256)])
@pytest.mark.parametrize("dropadd", [False, True])
def test_gemm_tall_n128_tile_bit_identical(dev, M, K, dropadd):
    N = 128
    torch.manual_seed(M + K)
    a = torch.randn(M, K, device=dev)
    w = torch.randn(N, K, device=dev) * 0.05
    am = torch.stack([a.abs().max(), w.abs().max()]).contiguous()
    outs = []
    for cfg in (-1, 1):   # automatic (cfg 5) against the forced 256 x 128 tile
        _lib.call("bgnn_gemm_set_cfg", cfg)
        try:
            if dropadd:
                src = torch.randn(M, N, device=dev, generator=torch.Generator(device=dev).manual_seed(7))
                out = torch.full((M, N), float("nan"), device=dev)
                ws_bytes = _lib.query("bgnn_gemm_ws_bytes_ex", M, N, K, 0, 1, 0)
                ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
                _lib.call("bgnn_gemm_f32_dropadd", 0, 1, M, N, K, a.data_ptr(), K, w.data_ptr(), K, out.data_ptr(), N,
                          am[0:1].data_ptr(), am[1:2].data_ptr(), src.data_ptr(), N, 0.1, 99, ws.data_ptr(),
                          ws_bytes, fused._stream())
                outs.append((out, None))
            else:
                bias = torch.randn(N, device=dev, generator=torch.Generator(device=dev).manual_seed(3))
                ca = torch.zeros(1, device=dev)
                out = fused.gemm(a, w, False, True, bias=bias, relu=True, a_amax=am[0:1], b_amax=am[1:2], c_amax=ca)
                outs.append((out, ca))
        finally:
            _lib.call("bgnn_gemm_set_cfg", -1)
    assert not torch.isnan(outs[0][0]).any()
    assert torch.equal(outs[0][0], outs[1][0])
    if not dropadd:
        assert torch.equal(outs[0][1], outs[1][1])
