#!/bin/bash
# Bench lines of the other BASELINE configs at HEAD: cfg3 (super nodes) and cfg5 (EA_GNN, bf16 and
# f32-accurate GEMM operands, 64 graphs per GPU), plus kernel stats of the cfg5 bf16 step.
mkdir -p gpurun_out
timeout -k 10 240 python bench.py --config cfg3 --no-cpu-baseline > gpurun_out/bench_cfg3.json 2> gpurun_out/bench_cfg3.err || exit $?
timeout -k 10 300 python bench.py --model EA_GNN --bf16 --config cfg5 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/bench_ea_cfg5_bf16.json 2> gpurun_out/bench_ea_cfg5_bf16.err || exit $?
timeout -k 10 300 python bench.py --model EA_GNN --config cfg5 --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/bench_ea_cfg5_f32.json 2> gpurun_out/bench_ea_cfg5_f32.err || exit $?
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_ea" -o run -- python "$ROOT/bench.py" --model EA_GNN --bf16 --config cfg5 --steps 3 --warmup 1 --no-cpu-baseline > "$ROOT/gpurun_out/prof_ea_bench.json" 2>&1
