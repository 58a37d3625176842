#!/bin/bash
# round 6 record am: the mean pool from the last fused layer (buckgnn.FUSED_POOL, ABI 13 g_rows):
# bit identity against the separate pool, the fused / model / full-size GPU tests, a same-process
# step A/B (cfg2 and cfg3)
set -o pipefail
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -x -q --timeout 120 --timeout-method thread -k mean_pool > $O/r06am_pool_test.txt 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_model.py tests/test_gpu_fullsize.py tests/test_gpu_ranges.py tests/test_gpu_max.py -x -q --timeout 300 --timeout-method thread > $O/r06am_tests.txt 2>&1 &&
timeout -k 10 300 python -u tools/ab_step.py "bgnn.buckgnn.FUSED_POOL=True" "bgnn.buckgnn.FUSED_POOL=False" > $O/r06am_ab_cfg2.txt 2>&1 &&
AB_CONFIG=cfg3 timeout -k 10 300 python -u tools/ab_step.py "bgnn.buckgnn.FUSED_POOL=True" "bgnn.buckgnn.FUSED_POOL=False" > $O/r06am_ab_cfg3.txt 2>&1
