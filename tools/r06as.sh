#!/bin/bash
# round 6 record as: the folded first layer's forward (80656 x 1024 x 128, K = 128) on each tile config
set -o pipefail
O=gpurun_out
timeout -k 10 300 python -u tools/gemm_ab.py --shapes fwd_fold --variants x-1,x0,x1,x2,x3,x4,x5 --reps 30 > $O/r06as_fold_tiles.txt 2>&1
