set -e
# EA_GNN bf16 check: bf16 GEMM / training tests, the cfg5 bench line and its kernel trace
TAG=${1:-m}
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_bf16.py tests/test_gpu_ea_train.py tests/test_gpu_gemm.py > gpurun_out/ea_tests_$TAG.txt 2>&1 || (tail -30 gpurun_out/ea_tests_$TAG.txt; exit 1)
tail -2 gpurun_out/ea_tests_$TAG.txt
timeout -k 10 300 python bench.py --model EA_GNN --bf16 --config cfg5 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_ea5_$TAG.json 2> gpurun_out/bench_ea5_$TAG.err
python -c "import json; d=json.loads(open('gpurun_out/bench_ea5_$TAG.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])"
ROOT=$(pwd); cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_ea5_$TAG" -o run -- python "$ROOT/bench.py" --model EA_GNN --bf16 --config cfg5 --steps 3 --warmup 1 --no-cpu-baseline > "$ROOT/gpurun_out/prof_ea5_$TAG.json" 2>&1
cd $ROOT; python tools/kstep.py gpurun_out/prof_ea5_$TAG/run_kernel_stats.csv 4 8
