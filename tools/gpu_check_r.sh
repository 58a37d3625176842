#!/bin/bash
# bwd_rows norm-prefetch check + 2-rank gloo rehearsal of bench.py's N > 1 path (both ranks on one GPU)
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_fullsize.py tests/test_gpu_model.py tests/test_gpu_sageconv.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_r.log 2>&1
tail -1 gpurun_out/gpu_tests_r.log
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_r" -o run -- python "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline > "$ROOT/gpurun_out/prof_bench_r.json" 2>&1
cd "$ROOT"
BGNN_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_n2_gloo_r.json 2> gpurun_out/bench_n2_gloo_r.err
