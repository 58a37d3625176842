#!/bin/bash
# round 6 record aa: the forward GEMM (k_gemm_x6 256 x 256, pre-split B) with the staging of waves 4-7
# moved between the two halves of their MFMA block (measurement build, knob 16 = 5); order-shuffled
set -o pipefail
O=gpurun_out
BGNN_LIBRARY=$PWD/buck-gnn_amd/bgnn/_lib/libbgnn_abl.so timeout -k 10 300 python -u tools/gemm_ab.py --shapes fwd,fwd_fold \
  --variants w,w@5 --reps 30 > $O/r06aa_gemm_fwd_stagger.txt 2>&1
