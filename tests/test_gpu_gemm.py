"""GPU: bgnn_gemm_f32 (f32 MFMA) against an fp64 torch reference, all transposes,
ragged shapes, split-K and beta accumulation."""
import pytest
import torch

from bgnn import _lib, fused

pytestmark = pytest.mark.gpu


@pytest.fixture(params=[0, 1], ids=["f32", "x6"])
def mode(request):
    """GEMM kernel family: 0 = f32 MFMA, 1 = bf16x6 (BGNN_TUNE_GEMM_MODE)."""
    _lib.call("bgnn_set_tuning", 5, request.param)
    yield request.param
    _lib.call("bgnn_set_tuning", 5, 0)


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


@pytest.mark.parametrize("ta,tb", [(False, True), (False, False), (True, False)])
def test_gemm_error_class_per_element(dev, ta, tb):
    """Per-element error bound max |c - c64| / (|A||B|) of both kernel families on a SAGE-like
    shape: the bf16x6 split is in the f32 MFMA's error class (f32 unit roundoff 6e-8 times a
    small factor), far below the 1e-4 parity tolerance."""
    torch.manual_seed(5)
    M, N, K = 3000, 512, 1024
    a = torch.randn((K, M) if ta else (M, K), device=dev)
    b = torch.randn((N, K) if tb else (K, N), device=dev) * 0.03
    A = a.double().t() if ta else a.double()
    B = b.double().t() if tb else b.double()
    c64, mag = A @ B, A.abs() @ B.abs()
    errs = []
    for m in (0, 1):
        _lib.call("bgnn_set_tuning", 5, m)
        try:
            c = fused.gemm(a, b, ta, tb)
        finally:
            _lib.call("bgnn_set_tuning", 5, 0)
        errs.append(((c.double() - c64).abs() / mag).max().item())
    assert errs[0] < 1e-6 and errs[1] < 1e-6, errs
    assert errs[1] < 4 * errs[0] + 1e-7, errs
