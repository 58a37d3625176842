#!/bin/bash
# round 6 record p: timing ablations of the pipelined GEMM (measurement build libbgnn_abl.so)
set -o pipefail
O=gpurun_out
BGNN_LIBRARY=$PWD/buck-gnn_amd/bgnn/_lib/libbgnn_abl.so timeout -k 10 300 python -u tools/gemm_ab.py --shapes dgrad \
  --variants w,w@3,w@16,w@32,w@48,w@64,w@112,w@128,w@256,w@240,w@496,w@512,w@1008 --reps 15 > $O/r06p_gemm_abl.txt 2>&1
