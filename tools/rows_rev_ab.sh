#!/bin/bash
# BGNN_TUNE_ROWS_REV A/B (include/bgnn.h): bit 0 bwd_rows, bit 2 SAGE aggregation, bit 3 transpose aggregation walk downward
set -e
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_fused.py -q -x --timeout 120 --timeout-method thread -k "rows_rev" > gpurun_out/rows_rev_tests.log 2>&1
tail -1 gpurun_out/rows_rev_tests.log
AB_ROUNDS=7 timeout -k 10 240 python tools/ab_step.py "knob:13=0" "knob:13=1" "knob:13=5" "knob:13=9" "knob:13=13" > gpurun_out/rows_rev_ab.txt 2>&1
cat gpurun_out/rows_rev_ab.txt
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
for v in 1 13; do
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_rev$v" -o run -- python "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --tune 13=$v > "$ROOT/gpurun_out/prof_rev$v.json" 2>&1
done
