#!/bin/bash
# Round-4 GPU check: every GPU test, smoke, benches (cfg2, cfg3, GraphSage_maxAggr), kernel-trace
# profile of the cfg2 bench. Usage (GPU box, repo root): bash tools/gpu_r4.sh TAG [pytest args]
set -e
TAG=${1:-run}
shift || true
mkdir -p gpurun_out
rc=0
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread "$@" > gpurun_out/gpu_tests_$TAG.log 2>&1 || rc=$?
tail -3 gpurun_out/gpu_tests_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "gpu tests ended with rc=$rc"; exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
timeout -k 10 300 python bench.py --config cfg3 --no-cpu-baseline > gpurun_out/bench_cfg3_$TAG.json 2> gpurun_out/bench_cfg3_$TAG.err
timeout -k 10 300 python bench.py --model GraphSage_maxAggr --no-cpu-baseline > gpurun_out/bench_max_$TAG.json 2> gpurun_out/bench_max_$TAG.err
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_$TAG" -o run -- python "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline > "$ROOT/gpurun_out/prof_bench_$TAG.json" 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_max_$TAG" -o run -- python "$ROOT/bench.py" --model GraphSage_maxAggr --steps 5 --warmup 2 --no-cpu-baseline > "$ROOT/gpurun_out/prof_bench_max_$TAG.json" 2>&1
echo done
