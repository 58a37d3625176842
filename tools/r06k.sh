#!/bin/bash
# round 6 record k: fwd GEMM at M = N vs N + R (range rows), and the fold precision across seeds
# with every GEMM on its planned tile vs forced onto the 8-wave 16x16x32 tile
set -o pipefail
O=gpurun_out
timeout -k 10 300 python -u tools/gemm_ab.py --shapes fwd3,fwd3r,fwd3,fwd3r --variants w --reps 30 > $O/r06k_gemm_m.txt 2>&1 &&
FOLD_GLOBAL_CFG=1 timeout -k 10 600 python -u tools/fold_ab.py > $O/r06k_fold_global_cfg.txt 2>&1
