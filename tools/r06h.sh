#!/bin/bash
# round 6 record h: range rows (csrc/ranges.hip) -- GPU tests, full-size cfg3 parity, bench A/B
set -o pipefail
O=gpurun_out
T="python -u -m pytest -m gpu -x -v --timeout 400 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_ranges.py tests/test_gpu_spmm.py tests/test_gpu_fused.py > $O/r06h_tests.txt 2>&1 &&
timeout -k 10 900 $T tests/test_gpu_fullsize.py -k cfg3 > $O/r06h_fullsize.txt 2>&1 &&
timeout -k 10 600 python -u bench.py > $O/r06h_bench.txt 2>&1 &&
timeout -k 10 600 python -u bench.py --config cfg3 --no-cpu-baseline --py-set bgnn.fused.RANGE_ROWS=False > $O/r06h_bench_cfg3_norange.txt 2>&1 &&
timeout -k 10 600 python -u bench.py --config cfg3 --no-cpu-baseline > $O/r06h_bench_cfg3_range.txt 2>&1
