#!/bin/bash
# round 6 record w: order-shuffled A/B of the pre-split GEMM forms (measurement build: 0 x6 register copy,
# 1 x6 + B by LDS-DMA, 2 / 3 pipelined with 3 / 4 slots, 1024 pipelined 4 slots without the stagger),
# then the cfg2 step with knob 16 = 0 against 3 (product build), alternating order
set -o pipefail
O=gpurun_out
BGNN_LIBRARY=$PWD/buck-gnn_amd/bgnn/_lib/libbgnn_abl.so timeout -k 10 400 python -u tools/gemm_ab.py --shapes dgrad \
  --variants w,W,w@2,w@3,w@1024,d,d@3,d@1024 --reps 25 > $O/r06w_gemm_ab.txt 2>&1 &&
AB_ROUNDS=8 timeout -k 10 500 python -u tools/ab_step.py "knob:16=0" "knob:16=3" > $O/r06w_ab_step.txt 2>&1
