#!/bin/bash
# round 6 record v: the bf16 edge GEMM's 128 x 256 two-workgroups-per-CU form (b16 variant 1) at cfg5's
# E = 2,863,488, then the pre-split GEMM tests with the staggered staging default
set -o pipefail
O=gpurun_out
timeout -k 10 400 python -u tools/bf16_storage_ab.py 2863488 7 > $O/r06v_b16_ab.txt 2>&1 &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm.py -m gpu -x -q --timeout 300 -k presplit > $O/r06v_gemm_tests.txt 2>&1
