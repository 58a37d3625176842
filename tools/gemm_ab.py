#!/usr/bin/env python
"""A/B of f16x3 GEMM variants on the SAGE layer shapes, in one process, each timed over REPS
launches with HIP events with operand maxima supplied (as inside the layer: no absmax passes),
with a 1 GiB cache flush between launches (cold L2 / Infinity Cache, as inside a training step).

    python tools/gemm_ab.py [--reps 20] [--variants=x-1,x2,x102] [--shapes fwd,dgrad]

A variant "xC" runs tile config C % 100 with timing ablation C // 100 (bgnn_gemm_set_cfg; x-1 =
the automatic plan); "pC" the same with the ping-pong main loop (BGNN_TUNE_GEMM_PP = 1), "lC" with
line-major staging loads (2), "qC" with both (3); "w" the pre-split weight path (bgnn_gemm_wsplit +
bgnn_gemm_f32_w, the weight image copied into LDS), "d" the same with the drop-add epilogue (src = a
[M, N] gradient, p = 0.1: the skip layers' dgrad); "r" / "s" as "w" / "d" with B's MFMA fragments
loaded from the image into registers (BGNN_TUNE_GEMM_PP = 4); "i" / "j" as "w" / "d" with the interleaved
steady-state schedule (BGNN_TUNE_GEMM_PP = 5); "m" / "n" with 16x16x32 MFMAs (BGNN_TUNE_GEMM_PP = 6).
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "buck-gnn_amd"))
import torch  # noqa: E402

from bgnn import _lib, fused  # noqa: E402

SHAPES = {"fwd": (80656, 1024, 512), "dgrad": (80656, 512, 1024), "ea": (715872, 512, 512),
          "fwd_small": (10082, 1024, 512), "fwd_fold": (80656, 1024, 128), "dgrad_fold": (80656, 128, 1024)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--variants", default="x-1")
    ap.add_argument("--shapes", default="fwd,dgrad")
    ap.add_argument("--no-flush", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    flush = None if args.no_flush else torch.empty(1 << 28, device=dev)
    for name in args.shapes.split(","):
        M, N, K = SHAPES[name]
        torch.manual_seed(0)
        a = torch.randn(M, K, device=dev)
        b = torch.randn(N, K, device=dev) * 0.05
        am = torch.stack([a.abs().max(), b.abs().max()]).contiguous()
        out = torch.empty(M, N, device=dev)
        src = torch.randn(M, N, device=dev)
        ref = None
        for vs in args.variants.split(","):
            wimg = None
            if vs[0] in "wdrsijmn":   # pre-split weight image + bgnn_gemm_f32_w ("wC": tile config C)
                _lib.call("bgnn_gemm_set_cfg", int(vs[1:]) if len(vs) > 1 else -1)
                _lib.call("bgnn_set_tuning", 14, {"r": 4, "s": 4, "i": 5, "j": 5, "m": 6, "n": 6}.get(vs[0], 0))
                bn = _lib.query("bgnn_gemm_w_tile", M, N, K)
                wimg = torch.empty(_lib.query("bgnn_gemm_wsplit_bytes", N, K), dtype=torch.uint8, device=dev)
                _lib.call("bgnn_gemm_wsplit", b.data_ptr(), 1, 0, N, K, K, am[1:2].data_ptr(), 0, wimg.data_ptr(),
                          wimg.numel(), bn | (0x10000 if vs[0] in "rs" else 0), fused._stream())
            else:
                _lib.call("bgnn_gemm_set_cfg", int(vs[1:]))
                _lib.call("bgnn_set_tuning", 14, {"x": 0, "p": 1, "l": 2, "q": 3}[vs[0]])   # BGNN_TUNE_GEMM_PP
            ts = []
            for i in range(args.reps + 3):
                if flush is not None:
                    flush.fill_(float(i))
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                if wimg is not None:
                    _lib.call("bgnn_gemm_f32_w", M, N, K, a.data_ptr(), K, wimg.data_ptr(), bn, out.data_ptr(), N,
                              None, 0, am[0:1].data_ptr(), am[1:2].data_ptr(), None,
                              src.data_ptr() if vs[0] in "dsjn" else None, N, 0.1, 1234, fused._stream())
                else:
                    fused.gemm(a, b, False, True, out=out, a_amax=am[0:1], b_amax=am[1:2])
                e1.record()
                ts.append((e0, e1))
            torch.cuda.synchronize()
            us = sorted(e0.elapsed_time(e1) * 1e3 for e0, e1 in ts[3:])
            med = us[len(us) // 2]
            same = "" if ref is None else ("bit-identical" if torch.equal(out, ref) else
                                           f"DIFFERS max {(out - ref).abs().max().item():.3g}")
            if ref is None:
                ref = out.clone()
            print(f"{name:9s} {M}x{N}x{K} staging {vs:>3s}: median {med:7.1f} us  min {us[0]:7.1f}  "
                  f"{2 * M * N * K / med / 1e6:6.1f} TF  {same}", flush=True)
        _lib.call("bgnn_gemm_set_cfg", -1)
        _lib.call("bgnn_set_tuning", 14, 0)


if __name__ == "__main__":
    main()
