#!/bin/bash
# Round-4 validation: every GPU test, smoke, and the bench lines (cfg2 with cpu_baseline, cfg3,
# GraphSage_maxAggr, inference mode, per-op route with torch / bgnn BatchNorm and the BN-free
# Shared variant, EA_GNN cfg5 bf16). Usage (GPU box, repo root): bash tools/gpu_r4c.sh TAG
set -e
TAG=${1:-c}
mkdir -p gpurun_out
rc=0
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || rc=$?
tail -3 gpurun_out/gpu_tests_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "gpu tests ended with rc=$rc"; exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
tail -1 gpurun_out/smoke_$TAG.log
B() { local name=$1; shift; timeout -k 10 200 python bench.py "$@" > gpurun_out/bench_${name}_$TAG.json 2> gpurun_out/bench_${name}_$TAG.err; }
B cfg2
B cfg3 --config cfg3 --no-cpu-baseline
B max --model GraphSage_maxAggr --no-cpu-baseline
B infer --mode infer --steps 10 --warmup 2
B perop_torchbn --path per_op --no-cpu-baseline
B perop_bgnnbn --path per_op --bn bgnn --no-cpu-baseline
B perop_shared --path per_op --model GraphSage_addAggr_Shared --no-cpu-baseline
B shared --model GraphSage_addAggr_Shared --no-cpu-baseline
B ea5 --model EA_GNN --bf16 --config cfg5 --steps 5 --warmup 2 --no-cpu-baseline
for f in gpurun_out/bench_*_$TAG.json; do echo "$f"; python -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d.get('roofline',{}).get('frac'), d.get('roofline_hbm',{}).get('frac'), d.get('roofline_agg_bwd',{}).get('frac'))"; done
