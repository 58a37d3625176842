#!/usr/bin/env python
"""f16x3 error class by MFMA shape: the 4-wave 128x128 tile (bgnn_gemm_set_cfg 0) runs
v_mfma_f32_32x32x16_f16, the 8-wave tiles (cfg 1-4) v_mfma_f32_16x16x32_f16, on the same operands
(register-staged path, fused.gemm): max |c - c64| / (|A||B|), the mean signed error relative to
sum |a b| (the bias a truncating accumulator leaves, growing with K), and the RMS of that relative
error -- on positive and on signed operands, over K, and on the folded encoder's weight products
(fused.sage_layer: Wf = Wcat W_in, bf = Wcat b_in, dW = dWf W_in^T, dW_in = Wcat^T dWf,
db_in = Wcat^T sum(dz)), both shapes.

    python tools/m16_precision.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "buck-gnn_amd"))
import torch  # noqa: E402

from bgnn import _lib, fused  # noqa: E402


def gemm_cfg(a, b, ta, tb, cfg):
    _lib.call("bgnn_gemm_set_cfg", cfg)
    try:
        return fused.gemm(a, b, ta, tb)
    finally:
        _lib.call("bgnn_gemm_set_cfg", -1)


def stats(c, a, b, ta, tb):
    A = (a.t() if ta else a).double()
    B = (b.t() if tb else b).double()
    r, mag = A @ B, A.abs() @ B.abs()
    e = c.double() - r
    rel = e / mag.clamp_min(1e-300)
    return rel.abs().max().item(), rel.mean().item(), rel.pow(2).mean().sqrt().item()


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    print("shape                      operands  | 32x32x16 (cfg 0): max      bias       rms  | "
          "16x16x32 (cfg 1): max      bias       rms")
    cases = [(1024, 128, 512, False, False), (1024, 1, 512, False, False), (512, 128, 1024, True, False),
             (512, 1, 1024, True, False), (1024, 512, 128, False, True)]
    for M, N, K in [(4096, 512, 512), (4096, 512, 1024), (4096, 512, 4096), (4096, 512, 16384)]:
        cases.append((M, N, K, False, True))
    for (M, N, K, ta, tb) in cases:
        for kind in ("positive", "signed"):
            a = torch.randn((K, M) if ta else (M, K), device=dev) * 0.05
            b = torch.randn((N, K) if tb else (K, N), device=dev) * 0.05
            if kind == "positive":
                a, b = a.abs(), b.abs()
            s0 = stats(gemm_cfg(a, b, ta, tb, 0), a, b, ta, tb)
            s1 = stats(gemm_cfg(a, b, ta, tb, 1), a, b, ta, tb)
            print(f"{M}x{N}x{K} ta={int(ta)} tb={int(tb)}  {kind:8s} | {s0[0]:.2e} {s0[1]:+.2e} {s0[2]:.2e} | "
                  f"{s1[0]:.2e} {s1[1]:+.2e} {s1[2]:.2e}", flush=True)


if __name__ == "__main__":
    main()


def epilogue_check():
    """Run under BGNN_LIBRARY=<libbgnn_m16.so> (make -C buck-gnn_amd m16): every tile config on
    16x16x32 MFMAs, so the 4-wave 128x128 tile (cfg 0) and the 8-wave 256x128 tile (cfg 1) must give
    the same bits wherever their split-K factors agree. The folded layer's calls (N = 2304 rows,
    H = 512, K_in = 128), with the epilogue features they use: bias (fwd_fold), c_amax (wgrad_fold,
    the weight products' maxima), split-K (wgrad_fold, dw_in). Prints bit-identity and the max
    error against fp64 relative to |A||B| for both tiles."""
    dev = torch.device("cuda", 0)
    torch.manual_seed(1)
    N, H, K = 2304, 512, 128
    calls = {"fwd_fold+bias": (N, 2 * H, K, False, True, True, False),
             "dgrad_fold": (N, K, 2 * H, False, True, False, False),
             "wgrad_fold+c_amax": (2 * H, K, N, True, False, False, True),
             "wf": (2 * H, K, H, False, False, False, False), "bf": (2 * H, 1, H, False, False, False, False),
             "dw": (2 * H, H, K, False, True, False, False), "dw_in": (H, K, 2 * H, True, False, False, False),
             "db_in": (H, 1, 2 * H, True, False, False, False)}
    for name, (M, Nn, Kd, ta, tb, bias, camax) in calls.items():
        a = torch.randn((Kd, M) if ta else (M, Kd), device=dev) * 0.05
        b = torch.randn((Nn, Kd) if tb else (Kd, Nn), device=dev) * 0.05
        bv = torch.randn(Nn, device=dev) if bias else None
        outs = []
        for cfg in (0, 1):
            ca = torch.zeros(1, device=dev) if camax else None
            _lib.call("bgnn_gemm_set_cfg", cfg)
            try:
                c = fused.gemm(a, b, ta, tb, bias=bv, c_amax=ca) if camax else fused.gemm(a, b, ta, tb, bias=bv)
            finally:
                _lib.call("bgnn_gemm_set_cfg", -1)
            torch.cuda.synchronize()
            outs.append((c, ca))
        A = (a.t() if ta else a).double()
        B = (b.t() if tb else b).double()
        r = A @ B + (bv.double() if bias else 0)
        mag = A.abs() @ B.abs() + (bv.double().abs() if bias else 0)
        errs = [((c.double() - r).abs() / mag).max().item() for c, _ in outs]
        same = torch.equal(outs[0][0], outs[1][0])
        extra = ""
        if camax:
            extra = (f" c_amax cfg0 {outs[0][1].item():.6e} cfg1 {outs[1][1].item():.6e} "
                     f"true {outs[0][0].abs().max().item():.6e}")
        print(f"{name:18s} {M}x{Nn}x{Kd} ta={int(ta)} tb={int(tb)}: cfg0 {errs[0]:.2e} cfg1 {errs[1]:.2e} "
              f"bit-identical {same}{extra}", flush=True)


if __name__ == "__main__" and os.environ.get("M16_EPILOGUE"):
    epilogue_check()
