#!/bin/bash
# bench (cfg2, cfg3) + kernel-trace profile of the cfg2 bench; TAG = $1
set -e
TAG=${1:-base}
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
timeout -k 10 300 python bench.py --config cfg3 --no-cpu-baseline > gpurun_out/bench_cfg3_$TAG.json 2> gpurun_out/bench_cfg3_$TAG.err
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_$TAG" -o run -- python "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline > "$ROOT/gpurun_out/prof_bench_$TAG.json" 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_cfg3_$TAG" -o run -- python "$ROOT/bench.py" --config cfg3 --steps 10 --warmup 3 --no-cpu-baseline > "$ROOT/gpurun_out/prof_bench_cfg3_$TAG.json" 2>&1
