#!/bin/bash
# round 6 record aq: the 32-bit dropout hash (common.h keep_bits4): every GPU test, the drop-add
# dgrad with / without mask against the plain product, and the cfg2 bench
set -o pipefail
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/r06aq_tests.txt 2>&1 &&
timeout -k 10 300 python -u tools/gemm_ab.py --shapes dgrad --variants w,d,n --reps 30 > $O/r06aq_gemm_mask.txt 2>&1 &&
timeout -k 10 200 python bench.py --no-cpu-baseline --no-cfg3 --steps 40 > $O/r06aq_bench.json 2> $O/r06aq_bench.err
