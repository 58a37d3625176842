#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fold.py tests/test_gpu_fused.py -q --timeout 120 --timeout-method thread > gpurun_out/fold_tests.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 240 python bench.py --no-cpu-baseline > gpurun_out/bench_g.json 2> gpurun_out/bench_g.err
