#!/bin/bash
# round 6 record aj: half of each XCD's first-round workgroups of the pipelined dgrad start late
# (s_sleep, ~7 / 14 / 20 us; measurement build, knob 16 = 4096 / 8192 / 12288) so that later rounds'
# epilogues (C stores) of the two halves do not coincide; order-shuffled
set -o pipefail
O=gpurun_out
BGNN_LIBRARY=$PWD/buck-gnn_amd/bgnn/_lib/libbgnn_abl.so timeout -k 10 300 python -u tools/gemm_ab.py --shapes dgrad \
  --variants w@3,w@4096,w@8192,w@12288,d@3,d@4096,d@8192,d@12288 --reps 30 > $O/r06aj_gemm_delay.txt 2>&1
