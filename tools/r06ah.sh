#!/bin/bash
# round 6 record ah: the pipelined GEMM's wave index through readfirstlane (product) against the plain
# threadIdx shift (measurement build, knob 16 = 2048); order-shuffled, drop-add dgrad and plain shapes
set -o pipefail
O=gpurun_out
BGNN_LIBRARY=$PWD/buck-gnn_amd/bgnn/_lib/libbgnn_abl.so timeout -k 10 300 python -u tools/gemm_ab.py --shapes dgrad \
  --variants d@3,d@2048,w@3,w@2048 --reps 30 > $O/r06ah_gemm_rfl.txt 2>&1
