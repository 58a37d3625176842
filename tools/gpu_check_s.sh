#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fold.py tests/test_gpu_fullsize.py tests/test_gpu_model.py tests/test_gpu_fused.py tests/test_gpu_sag.py tests/test_gpu_inference.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_s.log 2>&1
tail -1 gpurun_out/gpu_tests_s.log
timeout -k 10 240 python bench.py --no-cpu-baseline > gpurun_out/bench_s.json 2> gpurun_out/bench_s.err
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_s" -o run -- python "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline > "$ROOT/gpurun_out/prof_bench_s.json" 2>&1
