#!/usr/bin/env python
"""Interleaved A/B of f16x3 GEMM tile configs (bgnn_gemm_set_cfg) on the SAGE layer shapes as the
training step runs them: fwd z = x [W_l;W_r]^T, dgrad dx = dz Wcat (B = Wcat^T, K-contiguous), the
drop-add dgrad of skip layers (bgnn_gemm_f32_dropadd), wgrad dW = dz^T x. Operand maxima supplied
(as in the layer), 1 GiB cache flush between launches, median of R rounds; bit-identity against
the default plan.   python tools/gemm_cfg_ab.py [--cfgs -1,1,2,3,4] [--rounds 15] [--shapes ...]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "buck-gnn_amd"))
import torch  # noqa: E402

from bgnn import _lib, fused  # noqa: E402

H = 512


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfgs", default="-1,1,2,3,4")
    ap.add_argument("--rounds", type=int, default=15)
    ap.add_argument("--shapes", default="fwd,dgrad,dropadd,wgrad")
    ap.add_argument("--rows", type=int, default=80656, help="M (node rows; cfg2 = 80656)")
    ap.add_argument("--knob", type=int, default=-1, help="a bgnn_set_tuning knob crossed with --cfgs")
    ap.add_argument("--values", default="", help="comma list of values for --knob")
    args = ap.parse_args()
    M = args.rows
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    x = torch.randn(M, H, device=dev)
    W = torch.randn(2 * H, H, device=dev) * 0.05
    Wt = W.t().contiguous()
    dz = torch.randn(M, 2 * H, device=dev) * 1e-3
    g = torch.randn(M, H, device=dev) * 1e-3
    am = torch.stack([x.abs().max(), W.abs().max(), dz.abs().max()]).contiguous()
    flush = torch.empty(1 << 28, device=dev)
    s = torch.cuda.current_stream().cuda_stream

    def dropadd(out):
        ws_bytes = _lib.query("bgnn_gemm_ws_bytes_ex", M, H, 2 * H, 0, 1, 0)
        ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
        _lib.call("bgnn_gemm_f32_dropadd", 0, 1, M, H, 2 * H, dz.data_ptr(), 2 * H, Wt.data_ptr(), 2 * H,
                  out.data_ptr(), H, am[2:3].data_ptr(), am[1:2].data_ptr(), g.data_ptr(), H, 0.1, 1234,
                  ws.data_ptr(), ws_bytes, s)

    shapes = {
        "fwd": (torch.empty(M, 2 * H, device=dev),
                lambda o: fused.gemm(x, W, False, True, out=o, a_amax=am[0:1], b_amax=am[1:2]), 2.0 * M * 2 * H * H),
        "dgrad": (torch.empty(M, H, device=dev),
                  lambda o: fused.gemm(dz, Wt, False, True, out=o, a_amax=am[2:3], b_amax=am[1:2]), 2.0 * M * 2 * H * H),
        "dropadd": (torch.empty(M, H, device=dev), dropadd, 2.0 * M * 2 * H * H),
        "wgrad": (torch.empty(2 * H, H, device=dev),
                  lambda o: fused.gemm(dz, x, True, False, out=o, a_amax=am[2:3], b_amax=am[0:1]), 2.0 * M * 2 * H * H),
    }
    vals = [int(v) for v in args.values.split(",")] if args.knob >= 0 and args.values else [None]
    cfgs = [(int(c), v) for c in args.cfgs.split(",") for v in vals]
    knob0 = _lib.query("bgnn_get_tuning", args.knob) if args.knob >= 0 else None
    names = args.shapes.split(",")
    times = {(n, c): [] for n in names for c in cfgs}
    outs = {}
    for rnd in range(args.rounds + 2):
        for n in names:
            out, fn, _ = shapes[n]
            for c in cfgs:
                _lib.call("bgnn_gemm_set_cfg", c[0])
                if c[1] is not None:
                    _lib.call("bgnn_set_tuning", args.knob, c[1])
                flush.fill_(float(rnd))
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn(out)
                e1.record()
                torch.cuda.synchronize()
                if rnd >= 2:
                    times[(n, c)].append(e0.elapsed_time(e1) * 1e3)
                if rnd == 1:
                    outs[(n, c)] = out.clone()
    _lib.call("bgnn_gemm_set_cfg", -1)
    if args.knob >= 0:
        _lib.call("bgnn_set_tuning", args.knob, knob0)
    for n in names:
        flop = shapes[n][2]
        for c in cfgs:
            ts = sorted(times[(n, c)])
            med = ts[len(ts) // 2]
            same = "ref" if c == cfgs[0] else ("bit-identical" if torch.equal(outs[(n, c)], outs[(n, cfgs[0])])
                                               else f"differs {(outs[(n, c)] - outs[(n, cfgs[0])]).abs().max().item():.2e}")
            print(f"{n:8s} cfg {c[0]:3d} {'' if c[1] is None else f'k{args.knob}={c[1]:<3d}'}: median {med:7.1f} us  min {ts[0]:7.1f}  {flop / med / 1e6:6.1f} TF  "
                  f"({flop / med / 1e6 / 833.3:.3f} of 833 TF)  {same}", flush=True)


if __name__ == "__main__":
    main()
