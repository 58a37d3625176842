#!/bin/bash
# round 4: new GPU tests, per-op benches (torch / bgnn BatchNorm, Shared), NT knob step A/B
set -e
TAG=${1:-b}
mkdir -p gpurun_out
rc=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_bn.py tests/test_gpu_model.py tests/test_gpu_bf16.py tests/test_gpu_max.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || rc=$?
tail -3 gpurun_out/gpu_tests_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "gpu tests ended with rc=$rc"; exit $rc; fi
for v in "addAggr torch" "addAggr bgnn" "addAggr_Shared torch"; do
  set -- $v
  timeout -k 10 300 python bench.py --path per_op --model GraphSage_$1 --bn $2 --no-cpu-baseline > gpurun_out/bench_perop_$1_$2_$TAG.json 2> gpurun_out/bench_perop_$1_$2_$TAG.err
  python -c "import json; d=json.load(open('gpurun_out/bench_perop_$1_$2_$TAG.json')); print('$1 $2', d['value'], d['ms_per_step'])"
done
AB_CLEAR=0 AB_ROUNDS=7 timeout -k 10 300 python tools/ab_step.py "knob:4=1" "knob:4=0" "knob:4=1;knob:6=1" > gpurun_out/ab_nt_$TAG.txt 2>&1
cat gpurun_out/ab_nt_$TAG.txt
