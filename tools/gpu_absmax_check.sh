set -e
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py tests/test_gpu_fused.py tests/test_gpu_fold.py tests/test_gpu_model.py > gpurun_out/absx_tests.txt 2>&1 || (tail -20 gpurun_out/absx_tests.txt; exit 1)
tail -1 gpurun_out/absx_tests.txt
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/bench_w.json 2>/dev/null
ROOT=$(pwd); cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_cfg2_w" -o run -- python "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline > /dev/null 2>&1
cd $ROOT; python -c "import json; d=json.loads(open('gpurun_out/bench_w.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])"
grep -h "absmax" gpurun_out/prof_cfg2_w/run_kernel_stats.csv | cut -d, -f1-4
