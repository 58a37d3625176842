#!/bin/bash
# round 6 record n: B staged by LDS-DMA (knob 16) against the register copy -- isolated GEMM A/B
# (bit identity checked), then the whole cfg2 step A/B
set -o pipefail
O=gpurun_out
timeout -k 10 300 python -u tools/gemm_ab.py --shapes dgrad,fwd,fwd_fold,dgrad_fold --variants w,W,d,D --reps 20 > $O/r06n_gemm_ab.txt 2>&1 &&
timeout -k 10 400 python -u tools/ab_step.py "knob:16=0" "knob:16=1" > $O/r06n_ab_step.txt 2>&1
