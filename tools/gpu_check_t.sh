#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_t.log 2>&1 || true
tail -1 gpurun_out/gpu_tests_t.log
timeout -k 10 240 python bench.py --no-cpu-baseline > gpurun_out/bench_t.json 2> gpurun_out/bench_t.err
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_t" -o run -- python "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline > "$ROOT/gpurun_out/prof_bench_t.json" 2>&1
