#!/usr/bin/env python
"""Time bgnn_mlp2_fwd / _bwd (the encoder head) at cfg2 size and print a digest of their outputs,
so two builds of the library can be compared bit for bit: run once per build, diff the digests.
    python tools/mlp2_ab.py [--rows 80656] [--reps 50]"""
import argparse
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "buck-gnn_amd"))
import torch  # noqa: E402

from bgnn import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=80656)
    ap.add_argument("--reps", type=int, default=50)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    N, F, D1, D2 = args.rows, 16, 64, 128
    g = torch.Generator(device="cpu").manual_seed(0)
    x = torch.randn(N, F, generator=g).to(dev)
    W1 = (torch.randn(D1, F, generator=g) * 0.25).to(dev)
    b1 = (torch.randn(D1, generator=g) * 0.1).to(dev)
    W2 = (torch.randn(D2, D1, generator=g) * 0.125).to(dev)
    b2 = (torch.randn(D2, generator=g) * 0.1).to(dev)
    dh = torch.randn(N, D2, generator=g).to(dev)
    h = torch.empty(N, D2, device=dev)
    amax = torch.zeros(1, device=dev)
    dW1, db1, dW2, db2 = torch.empty_like(W1), torch.empty_like(b1), torch.empty_like(W2), torch.empty_like(b2)
    ws_bytes = _lib.query("bgnn_mlp2_bwd_ws_bytes", N)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream().cuda_stream

    def fwd():
        _lib.call("bgnn_mlp2_fwd", x.data_ptr(), N, F, D1, D2, W1.data_ptr(), b1.data_ptr(), W2.data_ptr(),
                  b2.data_ptr(), h.data_ptr(), amax.data_ptr(), s)

    def bwd():
        _lib.call("bgnn_mlp2_bwd", x.data_ptr(), N, F, D1, D2, W1.data_ptr(), b1.data_ptr(), W2.data_ptr(),
                  h.data_ptr(), dh.data_ptr(), dW1.data_ptr(), db1.data_ptr(), dW2.data_ptr(), db2.data_ptr(),
                  ws.data_ptr(), ws_bytes, s)

    for name, fn in (("fwd", fwd), ("bwd", bwd)):
        for _ in range(5):
            fn()
        ts = []
        for _ in range(args.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        ts.sort()
        print(f"mlp2 {name}: median {ts[len(ts) // 2]:7.1f} us  min {ts[0]:7.1f} us", flush=True)
    torch.cuda.synchronize()
    d = hashlib.sha256()
    for t in (h, amax, dW1, db1, dW2, db2):
        d.update(t.cpu().numpy().tobytes())
    print("digest", d.hexdigest()[:32])


if __name__ == "__main__":
    main()
