#!/usr/bin/env python
"""Diagnostic for the persistent pipelined GEMM (knob 16 = 5): compares it with k_gemm_x6 (knob 0) on
small shapes and prints where the outputs differ (tile, row / column inside the 128 x 256 tile)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "buck-gnn_amd"))
import torch  # noqa: E402

from bgnn import _lib, fused  # noqa: E402


def run(M, N, K, knob, a, w, am, img, bn, src=None):
    _lib.call("bgnn_gemm_set_cfg", 2)
    _lib.call("bgnn_set_tuning", 16, knob)
    out = torch.full((M, N), float("nan"), device=a.device)
    _lib.call("bgnn_gemm_f32_w", M, N, K, a.data_ptr(), K, img.data_ptr(), bn, out.data_ptr(), N, None, 0,
              am[0:1].data_ptr(), am[1:2].data_ptr(), None, src.data_ptr() if src is not None else None, N,
              0.1 if src is not None else 0.0, 1234, fused._stream())
    torch.cuda.synchronize()
    _lib.call("bgnn_gemm_set_cfg", -1)
    _lib.call("bgnn_set_tuning", 16, 3)
    return out


def main():
    dev = torch.device("cuda", 0)
    for (M, N, K) in [(25600, 256, 1024)]:
        torch.manual_seed(0)
        a = torch.randn(M, K, device=dev)
        w = torch.randn(N, K, device=dev) * 0.03
        am = torch.stack([a.abs().max(), w.abs().max()]).contiguous()
        _lib.call("bgnn_gemm_set_cfg", 2)
        bn = _lib.query("bgnn_gemm_w_tile", M, N, K)
        if bn == 0:
            print(f"M={M} N={N} K={K}: no pre-split plan", flush=True)
            continue
        img = torch.empty(_lib.query("bgnn_gemm_wsplit_bytes", N, K), dtype=torch.uint8, device=dev)
        _lib.call("bgnn_gemm_wsplit", w.data_ptr(), 1, 0, N, K, K, am[1:2].data_ptr(), 0, img.data_ptr(), img.numel(),
                  bn, fused._stream())
        _lib.call("bgnn_gemm_set_cfg", -1)
        ref = run(M, N, K, 0, a, w, am, img, bn)
        out = run(M, N, K, 5, a, w, am, img, bn)
        bad = (out != ref) & ~(out.isnan() & ref.isnan())
        print(f"M={M} N={N} K={K} bn={bn}: {int(bad.sum())} of {M * N} differ", flush=True)
        if bad.any():
            r, c = bad.nonzero(as_tuple=True)
            print("  rows in tile (r % 128) histogram by 16:", torch.bincount((r % 128) // 16, minlength=8).tolist())
            print("  cols in tile (c % 256) histogram by 16:", torch.bincount((c % 256) // 16, minlength=16).tolist())
            print("  tiles (r // 128):", torch.unique(r // 128)[:20].tolist())
            i = 0
            print(f"  first: row {int(r[i])} col {int(c[i])} out {float(out[r[i], c[i]]):.6g} ref {float(ref[r[i], c[i]]):.6g}")
            print("  out[0:4, 8:16]:", out[0:4, 8:16].tolist())
            print("  ref[0:4, 8:16]:", ref[0:4, 8:16].tolist())
            sc = float(am[0]) * float(am[1])
            for k in range(min(6, len(r))):
                v = float(out[r[k], c[k]])
                hit = (ref[:128, :256] == v).nonzero().tolist()
                print(f"  bad ({int(r[k])},{int(c[k])}) = {v:.7g}; equal ref at {hit[:3]}; /ref {v / float(ref[r[k], c[k]]):.5g}")
            # lanes: which (row % 16, col % 16) positions are bad
            pos = torch.zeros(16, 16, dtype=torch.long, device=out.device)
            pos.index_put_(((r % 16), (c % 16)), torch.ones_like(r), accumulate=True)
            print("  bad count by (row % 16, col % 16):")
            for rr in range(16):
                print("   ", pos[rr].tolist())
            # is the output a permutation of the reference inside 4x4 blocks?
            o4 = out[: (M // 4) * 4].reshape(M // 4, 4, N // 4, 4)
            r4 = ref[: (M // 4) * 4].reshape(M // 4, 4, N // 4, 4)
            print("  equals transposed 4x4 blocks:", bool(torch.equal(o4, r4.transpose(1, 3))))


if __name__ == "__main__":
    main()
