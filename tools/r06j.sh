#!/bin/bash
# round 6 record j: range rows after the LDS range sums / parallel finish -- tests, cfg3 A/B, profile
set -o pipefail
O=gpurun_out
T="python -u -m pytest -m gpu -x -v --timeout 400 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_ranges.py tests/test_gpu_spmm.py tests/test_gpu_fused.py > $O/r06j_tests.txt 2>&1 &&
timeout -k 10 900 $T tests/test_gpu_fullsize.py -k cfg3 > $O/r06j_fullsize.txt 2>&1 &&
timeout -k 10 600 python -u bench.py --config cfg3 --no-cpu-baseline --py-set bgnn.fused.RANGE_ROWS=False > $O/r06j_bench_cfg3_norange.txt 2>&1 &&
timeout -k 10 600 python -u bench.py --config cfg3 --no-cpu-baseline > $O/r06j_bench_cfg3_range.txt 2>&1 &&
bash tools/gpu_check.sh r06j profcfg3
