#!/bin/bash
# round 6 record ad: tall N = 128 products on the 8-wave 128 x 128 tile (cfg 5) -- bit identity and
# an order-shuffled A/B against the 256 x 128 tile (cfg 1)
set -o pipefail
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -m gpu -x -q --timeout 300 -k tall_n128 > $O/r06ad_tests.txt 2>&1 &&
timeout -k 10 300 python -u tools/gemm_ab.py --shapes dgrad_fold --variants x1,x5,x0 --reps 30 > $O/r06ad_gemm_ab.txt 2>&1
