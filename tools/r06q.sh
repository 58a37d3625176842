#!/bin/bash
# round 6 record q: the pipelined pre-split GEMM, 8-wave 128 x 256 (knob 16 = 3) and 4-wave 128 x 128
# with two workgroups per CU (knob 16 = 4), against k_gemm_x6 (knob 16 = 0); then the cfg2 step
set -o pipefail
O=gpurun_out
timeout -k 10 300 python -u tools/gemm_ab.py --shapes dgrad,fwd,fwd_fold,dgrad_fold --variants w,w@3,w@4,d,d@3,d@4 --reps 20 > $O/r06q_gemm_ab.txt 2>&1 &&
timeout -k 10 400 python -u tools/ab_step.py "knob:16=0" "knob:16=3" "knob:16=4" > $O/r06q_ab_step.txt 2>&1
