#!/bin/bash
# round 6 record ac: the weight-gradient GEMM (k_gemm_x6 TN 256 x 256, split-K) with the staggered
# staging (measurement build, knob 16 = 5) and the pipelined dgrad with a scalar wave index; shuffled
set -o pipefail
O=gpurun_out
BGNN_LIBRARY=$PWD/buck-gnn_amd/bgnn/_lib/libbgnn_abl.so timeout -k 10 300 python -u tools/gemm_ab.py --shapes wgrad \
  --variants t,t@5 --reps 30 > $O/r06ac_gemm_wgrad_stagger.txt 2>&1 &&
timeout -k 10 300 python -u tools/gemm_ab.py --shapes dgrad --variants w,w@3,d,d@3 --reps 25 >> $O/r06ac_gemm_wgrad_stagger.txt 2>&1
