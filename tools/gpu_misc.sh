#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_model.py tests/test_gpu_fold.py -q --timeout 120 --timeout-method thread > gpurun_out/rows_tests.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_rows" -o run -- python "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline > "$ROOT/gpurun_out/prof_rows_bench.json" 2>&1
