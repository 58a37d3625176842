#!/usr/bin/env python
"""Interleaved A/B of f16x3 GEMM variants on the SAGE layer shapes, in one process: every round
times each variant once (HIP events, operand maxima supplied as inside the layer, a 1 GiB cache
flush before each launch: cold L2 / Infinity Cache, as inside a training step); medians over the
rounds. Results are checked bit-identical to the first variant.

    python tools/gemm_ab.py [--reps 20] [--variants=w,d,w.2] [--shapes fwd,dgrad]

(Round 6 measured a "+e" variant here, the ragged last row tile scheduled first: no gain beyond
the first-variant order bias, profiles/r06_gemm_edge_first_l.txt; not kept.) Variants: "xC" the register-staged kernel (bgnn_gemm_f32_scaled) on tile config C (-1 = the
automatic plan); "w" the pre-split weight path (bgnn_gemm_wsplit + bgnn_gemm_f32_w); "d" the same
with the drop-add epilogue (src = an [M, N] gradient, p = 0.1: the skip layers' dgrad), "n" that epilogue
with p = 0 (no dropout mask); "w.C" /
"d.C" on tile config C; "W", "D" (and "W.C", "D.C") the same with B staged by LDS-DMA (knob 16 = 1); a suffix "@V" sets
knob 16 (BGNN_TUNE_GEMM_BDMA) to V for that variant ("w@2": the pipelined kernel gemm_h3p.hip). (Round 6 measured the main-loop variants "wP" of the then knob 14 here,
profiles/r06_gemm_ab_b.txt.)
"""
import argparse
import random
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "buck-gnn_amd"))
import torch  # noqa: E402

from bgnn import _lib, fused  # noqa: E402

SHAPES = {"wgrad": (1024, 512, 80656), "fwd": (80656, 1024, 512), "dgrad": (80656, 512, 1024), "ea": (715872, 512, 512),
          "fwd_small": (10082, 1024, 512), "fwd3": (80672, 1024, 512), "fwd3r": (80688, 1024, 512), "fwd0": (80640, 1024, 512), "fwd_fold": (80656, 1024, 128), "dgrad_fold": (80656, 128, 1024)}


def parse(vs):
    """-> (kind, knob-16 value, tile cfg)"""
    vs, _, kv = vs.partition("@")
    kind = vs[0]
    if kind in "WD":   # the w / d variants with B staged by LDS-DMA (knob 16 = 1)
        kind, kv = kind.lower(), kv or "1"
    knob = int(kv) if kv else 0
    if kind == "x":
        return kind, knob, int(vs[1:])
    if kind == "t":   # the TN weight-gradient product on its automatic plan
        return kind, knob, -1
    _, _, cfg = vs[1:].partition(".")
    return kind, knob, int(cfg) if cfg else -1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--variants", default="w,d")
    ap.add_argument("--shapes", default="fwd,dgrad")
    ap.add_argument("--no-flush", action="store_true")
    ap.add_argument("--fixed-order", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    flush = None if args.no_flush else torch.empty(1 << 28, device=dev)
    variants = args.variants.split(",")
    for name in args.shapes.split(","):
        M, N, K = SHAPES[name]
        torch.manual_seed(0)
        # ("t" variants: the TN product C = a^T b of the weight gradient, a [K, M], b [K, N])
        a = torch.randn(K, M, device=dev) if name == "wgrad" else torch.randn(M, K, device=dev)
        b = torch.randn(K, N, device=dev) * 0.05 if name == "wgrad" else torch.randn(N, K, device=dev) * 0.05
        am = torch.stack([a.abs().max(), b.abs().max()]).contiguous()
        src = torch.randn(M, N, device=dev)
        outs = {v: torch.empty(M, N, device=dev) for v in variants}
        imgs = {}
        for vs in variants:
            kind, pp, cfg = parse(vs)
            if kind[0] in "wdn":
                _lib.call("bgnn_gemm_set_cfg", cfg)
                _lib.call("bgnn_set_tuning", 16, pp)   # (knob 16 = 4 plans 128-column images)
                bn = _lib.query("bgnn_gemm_w_tile", M, N, K)
                img = torch.empty(_lib.query("bgnn_gemm_wsplit_bytes", N, K), dtype=torch.uint8, device=dev)
                _lib.call("bgnn_gemm_wsplit", b.data_ptr(), 1, 0, N, K, K, am[1:2].data_ptr(), 0, img.data_ptr(),
                          img.numel(), bn, fused._stream())
                imgs[vs] = (img, bn)
        _lib.call("bgnn_gemm_set_cfg", -1)
        times = {v: [] for v in variants}
        rng = random.Random(0)
        for i in range(args.reps + 2):
            order = list(variants)
            if not args.fixed_order:   # (a fixed order favours or penalises the first variant by up to ~10 %)
                rng.shuffle(order)
            for vs in order:
                kind, pp, cfg = parse(vs)
                _lib.call("bgnn_gemm_set_cfg", cfg)
                _lib.call("bgnn_set_tuning", 16, pp)
                if flush is not None:
                    flush.fill_(float(i))
                out = outs[vs]
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                if kind[0] in "wdn":
                    img, bn = imgs[vs]
                    _lib.call("bgnn_gemm_f32_w", M, N, K, a.data_ptr(), K, img.data_ptr(), bn, out.data_ptr(), N,
                              None, 0, am[0:1].data_ptr(), am[1:2].data_ptr(), None,
                              src.data_ptr() if kind[0] in "dn" else None, N,
                              0.0 if kind[0] == "n" else 0.1, 1234, fused._stream())
                elif kind[0] == "t":
                    fused.gemm(a, b, True, False, out=out, a_amax=am[0:1], b_amax=am[1:2])
                else:
                    fused.gemm(a, b, False, True, out=out, a_amax=am[0:1], b_amax=am[1:2])
                e1.record()
                if i >= 2:
                    times[vs].append((e0, e1))
        _lib.call("bgnn_gemm_set_cfg", -1)
        _lib.call("bgnn_set_tuning", 16, 3)
        torch.cuda.synchronize()
        ref = {}
        for vs in variants:
            us = sorted(e0.elapsed_time(e1) * 1e3 for e0, e1 in times[vs])
            med = us[len(us) // 2]
            kind = vs[0].lower()
            r = ref.setdefault(kind, outs[vs])
            same = "ref" if r is outs[vs] else ("bit-identical" if torch.equal(outs[vs], r) else
                                                f"DIFFERS max {(outs[vs] - r).abs().max().item():.3g}")
            print(f"{name:9s} {M}x{N}x{K} {vs:>6s}: median {med:7.1f} us  min {us[0]:7.1f}  "
                  f"{2 * M * N * K / med / 1e6:6.1f} TF  {same}", flush=True)


if __name__ == "__main__":
    main()
