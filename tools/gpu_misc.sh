#!/bin/bash
# Round-2 A/B inside the train step: the fused encoder head (bgnn_mlp2) against the GEMM path.
mkdir -p gpurun_out
timeout -k 10 300 python tools/ab_step.py "bgnn.fused.FUSED_MLP2=True" "bgnn.fused.FUSED_MLP2=False" > gpurun_out/ab_mlp2.txt 2>&1
