#!/usr/bin/env python
"""A/B of the pre-split f16x3 GEMM (bgnn_gemm_p16, LDS-DMA staging of f16 pieces) against the
register-staged split GEMM (bgnn_gemm_f32_scaled, f16x3) on the cfg2 SAGE shapes: bit identity
and per-launch time (HIP events, median of R launches, L2/MALL flushed by a 512 MB write before
each). Also times the stand-alone split pass (bgnn_split_f16x2).

    python tools/p16_ab.py [R]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "buck-gnn_amd"))
from bgnn import _lib, fused  # noqa: E402
from bgnn.graph import _stream  # noqa: E402

R = int(sys.argv[1]) if len(sys.argv) > 1 else 15
dev = torch.device("cuda", 0)
flush = torch.empty(128 * 1024 * 1024, dtype=torch.float32, device=dev)


def timed(fn):
    ts = []
    for _ in range(R):
        flush.fill_(1.0)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def pieces(x, amax):
    p = torch.empty(x.size(0), 2 * x.size(1), dtype=torch.float16, device=dev)
    _lib.call("bgnn_split_f16x2", x.data_ptr(), x.size(0), x.size(1), x.stride(0), amax.data_ptr(), p.data_ptr(),
              2 * x.size(1), _stream())
    return p


def p16(ap, bp, M, N, K, a_amax, b_amax, C, variant, bsrc=None, p=0.0, seed=0):
    _lib.call("bgnn_gemm_p16", M, N, K, ap.data_ptr(), 2 * K, a_amax.data_ptr(), bp.data_ptr(), 2 * K,
              b_amax.data_ptr(), 1.0, 1.0 if bsrc is not None else 0.0, C.data_ptr(), N, None, 0, None,
              None if bsrc is None else bsrc.data_ptr(), N, float(p), seed, variant, _stream())


def run(name, M, N, K):
    torch.manual_seed(0)
    A = torch.randn(M, K, device=dev)
    B = torch.randn(N, K, device=dev) / K ** 0.5
    a_amax, b_amax = fused.absmax(A), fused.absmax(B)
    ref = fused.gemm(A, B, trans_a=False, trans_b=True, a_amax=a_amax, b_amax=b_amax)
    ap, bp = pieces(A, a_amax), pieces(B, b_amax)
    t_ref = timed(lambda: fused.gemm(A, B, trans_a=False, trans_b=True, a_amax=a_amax, b_amax=b_amax, out=ref))
    _lib.call("bgnn_gemm_set_cfg", 900 + (4 if N == 1024 else 2))   # x6 with s_setprio around the MFMA block
    out9 = torch.empty_like(ref)
    t_prio = timed(lambda: fused.gemm(A, B, trans_a=False, trans_b=True, a_amax=a_amax, b_amax=b_amax, out=out9))
    _lib.call("bgnn_gemm_set_cfg", -1)
    print(f"   x6 + s_setprio: {t_prio:7.1f} us, bit-identical: {bool(torch.equal(out9, ref))}")
    t_split = timed(lambda: pieces(A, a_amax))
    fl = 2.0 * M * N * K
    print(f"{name} {M}x{N}x{K}: x6 {t_ref:7.1f} us ({fl / t_ref / 1e6:6.1f} TF)   split pass of A {t_split:6.1f} us")
    for v in (1, 4, 15):
        C = torch.full((M, N), float("nan"), device=dev)
        p16(ap, bp, M, N, K, a_amax, b_amax, C, v)
        torch.cuda.synchronize()
        same = bool(torch.equal(C, ref)) if (v < 10 or v == 16) else None
        t = timed(lambda: p16(ap, bp, M, N, K, a_amax, b_amax, C, v))
        print(f"   p16 v{v:<2d} {t:7.1f} us ({fl / t / 1e6:6.1f} TF)  bit-identical: {same}")
    if N == 512:   # dgrad drop-add epilogue against bgnn_gemm_f32_dropadd
        g = torch.randn(M, N, device=dev)
        C1 = torch.empty(M, N, device=dev)
        ws_bytes = _lib.query("bgnn_gemm_ws_bytes_ex", M, N, K, 0, 1, 0)
        ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
        _lib.call("bgnn_gemm_f32_dropadd", 0, 1, M, N, K, A.data_ptr(), K, B.data_ptr(), K, C1.data_ptr(), N,
                  a_amax.data_ptr(), b_amax.data_ptr(), g.data_ptr(), N, 0.1, 77, ws.data_ptr(), ws_bytes, _stream())
        C2 = torch.empty(M, N, device=dev)
        p16(ap, bp, M, N, K, a_amax, b_amax, C2, 0, bsrc=g, p=0.1, seed=77)
        torch.cuda.synchronize()
        t1 = timed(lambda: _lib.call("bgnn_gemm_f32_dropadd", 0, 1, M, N, K, A.data_ptr(), K, B.data_ptr(), K,
                                     C1.data_ptr(), N, a_amax.data_ptr(), b_amax.data_ptr(), g.data_ptr(), N, 0.1,
                                     77, ws.data_ptr(), ws_bytes, _stream()))
        t2 = timed(lambda: p16(ap, bp, M, N, K, a_amax, b_amax, C2, 0, bsrc=g, p=0.1, seed=77))
        print(f"   drop-add: x6 {t1:7.1f} us, p16 {t2:7.1f} us, bit-identical: {bool(torch.equal(C1, C2))}")
        C3 = torch.empty(M, N, device=dev)
        p16(ap, bp, M, N, K, a_amax, b_amax, C3, 4, bsrc=g, p=0.1, seed=77)
        torch.cuda.synchronize()
        t3 = timed(lambda: p16(ap, bp, M, N, K, a_amax, b_amax, C3, 4, bsrc=g, p=0.1, seed=77))
        print(f"   drop-add persistent p16 {t3:7.1f} us, bit-identical: {bool(torch.equal(C1, C3))}")


run("fwd  ", 80656, 1024, 512)
run("dgrad", 80656, 512, 1024)
run("fold ", 80656, 1024, 128)
