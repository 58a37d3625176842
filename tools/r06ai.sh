#!/bin/bash
# round 6 record ai: the drop-add dgrad with and without its dropout mask (p = 0.1 / p = 0) against the
# plain product: the epilogue's counter-hash cost; order-shuffled
set -o pipefail
O=gpurun_out
timeout -k 10 300 python -u tools/gemm_ab.py --shapes dgrad,dgrad_fold --variants w,d,n --reps 30 > $O/r06ai_gemm_mask.txt 2>&1
