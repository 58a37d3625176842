#!/bin/bash
# round 6 record o: the pipelined pre-split GEMM (gemm_h3p.hip, knob 16 = 2 / 3) against k_gemm_x6
set -o pipefail
O=gpurun_out
timeout -k 10 200 python -u tools/gemm_ab.py --shapes dgrad --variants w,w@2,w@3,d,d@2,d@3 --reps 20 > $O/r06o_gemm_ab.txt 2>&1 &&
timeout -k 10 200 python -u tools/gemm_ab.py --shapes fwd --variants w,w.2,w.2@2,w.2@3 --reps 20 >> $O/r06o_gemm_ab.txt 2>&1 &&
timeout -k 10 400 python -u tools/ab_step.py "knob:16=0" "knob:16=2" "knob:16=3" > $O/r06o_ab_step.txt 2>&1
