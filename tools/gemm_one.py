#!/usr/bin/env python
"""Run one GEMM (SAGE layer shape) repeatedly with a fixed kernel family / tile config, for
rocprofv3 counter passes. Usage: tools/gemm_one.py MODE CFG SHAPE [REPS]
MODE 0 = f32 MFMA, 2 = f16x3 (the bf16x6 mode 1 was removed in ABI 9); CFG as bgnn_gemm_set_cfg (-1 = the plan, 0..4 the tiles);
SHAPE in fwd, dgrad, wgrad. Env GEMM_FLUSH=1 overwrites a 1 GiB buffer between launches
(cold L2 / Infinity Cache, as inside a training step); GEMM_RELU=1 makes A non-negative with
~half zeros (post-ReLU activations)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "buck-gnn_amd"))
import torch  # noqa: E402

from bgnn import _lib, fused  # noqa: E402

SHAPES = {"fwd": (80656, 1024, 512, False, True), "dgrad": (80656, 512, 1024, False, True),
          "wgrad": (1024, 512, 80656, True, False),
          # the folded first layer (encoder Linear folded into [W_l;W_r]: K_in = 128)
          "fold_fwd": (80656, 1024, 128, False, True), "fold_dgrad": (80656, 128, 1024, False, True),
          "fold_wgrad": (1024, 128, 80656, True, False)}


def main():
    mode, cfg, shape = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 20
    M, N, K, ta, tb = SHAPES[shape]
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    a = torch.randn((K, M) if ta else (M, K), device=dev)
    b = torch.randn((N, K) if tb else (K, N), device=dev)
    _lib.call("bgnn_set_tuning", 5, mode)
    _lib.call("bgnn_gemm_set_cfg", cfg)
    if os.environ.get("GEMM_RELU") == "1":
        a.clamp_(min=0)
    out = torch.empty(M, N, device=dev)
    flush = torch.empty(1 << 28, device=dev) if os.environ.get("GEMM_FLUSH") == "1" else None
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(reps + 3):
        if i == 3:
            e0.record()
        if flush is not None:
            flush.fill_(float(i))
        fused.gemm(a, b, ta, tb, out=out)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    print(f"mode {mode} cfg {cfg} {shape}: {ms * 1e3:.1f} us/launch, {2 * M * N * K / ms / 1e9:.1f} TF")


if __name__ == "__main__":
    main()
