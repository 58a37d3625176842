#!/bin/bash
# full GPU check: every GPU test, smoke, bench, kernel-trace profile of the bench
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_x.log 2>&1
tail -1 gpurun_out/gpu_tests_x.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_x.log 2>&1
tail -1 gpurun_out/smoke_x.log
timeout -k 10 300 python bench.py > gpurun_out/bench_x.json 2> gpurun_out/bench_x.err
tail -1 gpurun_out/bench_x.json
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_x" -o run -- python "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline > "$ROOT/gpurun_out/prof_bench_x.json" 2>&1
