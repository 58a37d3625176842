#!/bin/bash
# cfg3 (super nodes) and cfg5 (EA_GNN, bf16) bench lines on the current code
set -e
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --config cfg3 --no-cpu-baseline > gpurun_out/bench_cfg3_y.json 2> gpurun_out/bench_cfg3_y.err
tail -1 gpurun_out/bench_cfg3_y.json | cut -c1-300
timeout -k 10 400 python bench.py --model EA_GNN --bf16 --config cfg5 --no-cpu-baseline > gpurun_out/bench_ea_y.json 2> gpurun_out/bench_ea_y.err
tail -1 gpurun_out/bench_ea_y.json | cut -c1-300
