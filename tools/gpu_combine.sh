set -e
TAG=${1:-j}
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_spmm.py tests/test_gpu_fullsize.py tests/test_gpu_model.py tests/test_gpu_sag.py tests/test_gpu_max.py > gpurun_out/combine_tests_$TAG.txt 2>&1 || (tail -30 gpurun_out/combine_tests_$TAG.txt; exit 1)
tail -2 gpurun_out/combine_tests_$TAG.txt
timeout -k 10 200 python bench.py --config cfg3 --no-cpu-baseline > gpurun_out/bench_cfg3_$TAG.json 2> gpurun_out/bench_cfg3_$TAG.err
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/bench_cfg2_$TAG.json 2> gpurun_out/bench_cfg2_$TAG.err
ROOT=$(pwd); cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_cfg3_$TAG" -o run -- python "$ROOT/bench.py" --config cfg3 --steps 10 --warmup 3 --no-cpu-baseline > "$ROOT/gpurun_out/prof_cfg3_$TAG.json" 2>&1
cd $ROOT
python -c "import json; [print(f, json.loads(open(f).read().strip().splitlines()[-1])['value']) for f in ['gpurun_out/bench_cfg3_$TAG.json','gpurun_out/bench_cfg2_$TAG.json']]"
python tools/kstep.py gpurun_out/prof_cfg3_$TAG/run_kernel_stats.csv 13 16
