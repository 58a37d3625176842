set -e
TAG=${1:-s}
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_fold.py tests/test_gpu_model.py tests/test_gpu_fullsize.py tests/test_gpu_fused.py tests/test_gpu_wpack.py > gpurun_out/fold_tests_$TAG.txt 2>&1 || (tail -30 gpurun_out/fold_tests_$TAG.txt; exit 1)
tail -2 gpurun_out/fold_tests_$TAG.txt
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/bench_cfg2_$TAG.json 2> gpurun_out/bench_cfg2_$TAG.err
timeout -k 10 400 python tools/ab_step.py "bgnn.fused.FOLD_WEIGHTS_TORCH=False" > gpurun_out/ab_step_$TAG.txt 2>&1 || true
python -c "import json; d=json.loads(open('gpurun_out/bench_cfg2_$TAG.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])"
