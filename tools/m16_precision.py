#!/usr/bin/env python
"""f16x3 error class of the 16x16x32 MFMA main loop (the default since round 5) against the
32x32x16 form (BGNN_TUNE_GEMM_PP = 6, pre-split path): max |c - c64| / (|A||B|) and the mean
signed error relative to |c64| (a truncating accumulator shows as a bias growing with K), on
positive and on signed operands.

    python tools/m16_precision.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "buck-gnn_amd"))
import torch  # noqa: E402

from bgnn import _lib, fused  # noqa: E402


def run_w(a, w, pp):
    M, K = a.shape
    N = w.size(0)
    am = torch.stack([a.abs().max(), w.abs().max()]).contiguous()
    _lib.call("bgnn_set_tuning", 14, pp)
    try:
        bn = _lib.query("bgnn_gemm_w_tile", M, N, K)
        if bn == 0:
            return None
        img = torch.empty(_lib.query("bgnn_gemm_wsplit_bytes", N, K), dtype=torch.uint8, device=a.device)
        _lib.call("bgnn_gemm_wsplit", w.data_ptr(), 1, 0, N, K, K, am[1:2].data_ptr(), 0, img.data_ptr(), img.numel(),
                  bn, fused._stream())
        out = torch.empty(M, N, device=a.device)
        _lib.call("bgnn_gemm_f32_w", M, N, K, a.data_ptr(), K, img.data_ptr(), bn, out.data_ptr(), N, None, 0,
                  am[0:1].data_ptr(), am[1:2].data_ptr(), None, None, 0, 0.0, 0, fused._stream())
        return out
    finally:
        _lib.call("bgnn_set_tuning", 14, 0)


def stats(c, a, w):
    r = a.double() @ w.double().t()
    mag = a.abs().double() @ w.abs().double().t()
    e = (c.double() - r)
    return (e.abs() / mag).max().item(), (e / r.abs().clamp_min(1e-300)).mean().item()


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    # the folded encoder's weight products (fused.sage_layer): Wf = Wcat W_in, bf = Wcat b_in, and
    # the backward's dW_in = Wcat^T dWf, db_in = Wcat^T sum(dz), dW = dWf W_in^T
    for (M, N, K, ta, tb) in [(1024, 128, 512, False, False), (1024, 1, 512, False, False),
                              (512, 128, 1024, True, False), (512, 1, 1024, True, False),
                              (1024, 512, 128, False, True)]:
        a = torch.randn((K, M) if ta else (M, K), device=dev) * 0.05
        b = torch.randn((N, K) if tb else (K, N), device=dev) * 0.05
        c = fused.gemm(a, b, ta, tb)
        A = (a.t() if ta else a).double()
        B = (b.t() if tb else b).double()
        r, mag = A @ B, A.abs() @ B.abs()
        e = c.double() - r
        print(f"fold {M}x{N}x{K} ta={int(ta)} tb={int(tb)}: max {(e.abs() / mag).max().item():.2e} "
              f"mean|rel| {(e.abs() / r.abs().clamp_min(1e-30)).median().item():.2e}", flush=True)
    for M, N, K in [(80656, 1024, 512), (4096, 512, 1024)]:
        for kind in ("signed", "positive"):
            a = torch.randn(M, K, device=dev)
            w = torch.randn(N, K, device=dev) * 0.03
            if kind == "positive":
                a, w = a.abs(), w.abs()
            a = a[: min(M, 8192)].contiguous()
            Mr = a.size(0)
            c16 = run_w(a, w, 0)
            c32 = run_w(a, w, 6)
            if c16 is None or c32 is None:
                continue
            tm = fused.gemm(a, w, False, True)
            s16, s32, sg = stats(c16, a, w), stats(c32, a, w), stats(tm, a, w)
            print(f"{Mr}x{N}x{K} {kind:8s}: 16x16x32 max {s16[0]:.2e} bias {s16[1]:+.2e} | 32x32x16 max {s32[0]:.2e} "
                  f"bias {s32[1]:+.2e} | fused.gemm max {sg[0]:.2e} bias {sg[1]:+.2e}", flush=True)


if __name__ == "__main__":
    main()
