"""GPU: bgnn_gemm_f32 (f32 MFMA) against an fp64 torch reference, all transposes,
ragged shapes, split-K and beta accumulation."""
import pytest
import torch

from bgnn import fused

pytestmark = pytest.mark.gpu


def ref(a, b, ta, tb):
    A = a.double().cpu()
    B = b.double().cpu()
    return (A.t() if ta else A) @ (B.t() if tb else B)


@pytest.mark.parametrize("ta", [False, True])
@pytest.mark.parametrize("tb", [False, True])
@pytest.mark.parametrize("mnk", [(1, 1, 1), (37, 129, 15), (300, 200, 64), (128, 128, 128), (513, 1024, 512),
                                 (1024, 512, 9000)])
def test_gemm_matches_fp64(dev, ta, tb, mnk):
    M, N, K = mnk
    torch.manual_seed(M + N + K)
    a = torch.randn((K, M) if ta else (M, K), device=dev)
    b = torch.randn((N, K) if tb else (K, N), device=dev)
    c = fused.gemm(a, b, ta, tb)
    r = ref(a, b, ta, tb)
    err = (c.double().cpu() - r).abs().max().item()
    scale = (a.abs().double().cpu().max() * b.abs().double().cpu().max() * K).item()
    assert err <= 2e-6 * scale + 1e-6, (err, scale)


def test_gemm_beta_accumulates_and_strided_views(dev):
    torch.manual_seed(0)
    big = torch.randn(200, 64, device=dev)
    a = big[:, 32:]            # strided rows (ld = 64)
    w = torch.randn(48, 32, device=dev)
    c0 = torch.randn(200, 48, device=dev)
    c = c0.clone()
    fused.gemm(a, w, False, True, out=c, beta=1.0)
    r = c0.double().cpu() + a.double().cpu() @ w.double().cpu().t()
    torch.testing.assert_close(c.double().cpu(), r, rtol=1e-5, atol=1e-4)


def test_gemm_is_deterministic(dev):
    a = torch.randn(4000, 1024, device=dev)
    b = torch.randn(4000, 512, device=dev)
    c1 = fused.gemm(a, b, True, False)
    c2 = fused.gemm(a, b, True, False)
    assert torch.equal(c1, c2)
