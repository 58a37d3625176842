#!/bin/bash
# round 6 record z: the forward on the pipelined kernel with 256 x 128 tiles (measurement build,
# cfg 1 forced) against k_gemm_x6 256 x 256 (its plan) and 256 x 128; order-shuffled
set -o pipefail
O=gpurun_out
BGNN_LIBRARY=$PWD/buck-gnn_amd/bgnn/_lib/libbgnn_abl.so timeout -k 10 300 python -u tools/gemm_ab.py --shapes fwd,fwd_fold \
  --variants w,w.1,w.1@3,w.2@3 --reps 25 > $O/r06z_gemm_fwd.txt 2>&1
