#!/bin/bash
# round 6 record u: staggered staging of the pipelined GEMM (measurement build, X = 64 -> knob 1024)
set -o pipefail
O=gpurun_out
BGNN_LIBRARY=$PWD/buck-gnn_amd/bgnn/_lib/libbgnn_abl.so timeout -k 10 300 python -u tools/gemm_ab.py --shapes dgrad \
  --variants w@3,w@1024,w@3,w@1024,d@3,d@1024 --reps 20 > $O/r06u_gemm_stagger.txt 2>&1
