#!/bin/bash
# round 6 record y: the drop-add source staged through LDS by the last steps' DMA (pipelined GEMM):
# the pre-split GEMM tests, an order-shuffled A/B against k_gemm_x6, the cfg2 step
set -o pipefail
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm.py -m gpu -x -q --timeout 300 -k presplit > $O/r06y_gemm_tests.txt 2>&1 &&
timeout -k 10 300 python -u tools/gemm_ab.py --shapes dgrad --variants w,w@3,d,d@3 --reps 25 > $O/r06y_gemm_ab.txt 2>&1 &&
AB_ROUNDS=8 timeout -k 10 500 python -u tools/ab_step.py "knob:16=0" "knob:16=3" > $O/r06y_ab_step.txt 2>&1
