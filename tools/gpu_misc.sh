#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_fused.py -q --timeout 120 --timeout-method thread -k mlp2 > gpurun_out/mlp2_tests.log 2>&1 || exit $?
timeout -k 10 300 python tools/ab_step.py "bgnn.fused.FUSED_MLP2=True" "bgnn.fused.FUSED_MLP2=False" > gpurun_out/ab_mlp2.txt 2>&1 || exit $?
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_mlp2" -o run -- python "$ROOT/tools/ab_step.py" "bgnn.fused.FUSED_MLP2=True" > /dev/null 2>&1
