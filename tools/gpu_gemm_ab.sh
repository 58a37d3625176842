set -e
# GEMM shapes of the SAGE layers, interleaved A/B (tools/gemm_cfg_ab.py) at the cfg2 node count and
# at a multiple of 32 (K of the weight gradient), GEMM tests, one cfg2 bench
TAG=${1:-e}
timeout -k 10 250 python tools/gemm_cfg_ab.py --cfgs=-1 --rounds 8 > gpurun_out/gemm_ab_$TAG.txt 2>&1
timeout -k 10 250 python tools/gemm_cfg_ab.py --cfgs=-1 --rounds 8 --rows 80640 >> gpurun_out/gemm_ab_$TAG.txt 2>&1
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py tests/test_gpu_fused.py tests/test_gpu_fullsize.py > gpurun_out/gemm_tests_$TAG.txt 2>&1
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/bench_gemm_$TAG.json 2> gpurun_out/bench_gemm_$TAG.err
grep -v amdgpu.ids gpurun_out/gemm_ab_$TAG.txt; tail -2 gpurun_out/gemm_tests_$TAG.txt; cat gpurun_out/bench_gemm_$TAG.json
