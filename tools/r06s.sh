#!/bin/bash
# round 6 record s: the persistent pipelined GEMM (knob 16 = 5) against the pipelined (3) and x6 (0)
set -o pipefail
O=gpurun_out
timeout -k 10 300 python -u tools/gemm_ab.py --shapes dgrad,fwd --variants w.2@3,w.2@5,w,d.2@3,d.2@5,d --reps 20 > $O/r06s_gemm_ab.txt 2>&1 &&
timeout -k 10 400 python -u tools/ab_step.py "knob:16=3" "knob:16=5" > $O/r06s_ab_step.txt 2>&1
