set -e
timeout -k 10 200 python tools/agg_knob_ab.py --rounds 12 "" "14=1" "15=1280" "14=1;15=1280" > gpurun_out/agg_ab_a.txt 2>&1
timeout -k 10 200 python tools/agg_knob_ab.py --rounds 12 --group-rows 8 "" >> gpurun_out/agg_ab_a.txt 2>&1
timeout -k 10 200 python tools/agg_knob_ab.py --rounds 12 --group-rows 8 --reorder "" >> gpurun_out/agg_ab_a.txt 2>&1
timeout -k 10 200 python tools/agg_knob_ab.py --rounds 12 --group-rows 4 --reorder "" >> gpurun_out/agg_ab_a.txt 2>&1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_store.py > gpurun_out/store_tests_a.txt 2>&1
timeout -k 10 200 python bench.py --reorder 0 --no-cpu-baseline > gpurun_out/bench_reorder0_a.json 2> gpurun_out/bench_reorder0_a.err
timeout -k 10 200 python bench.py --reorder 1 --no-cpu-baseline > gpurun_out/bench_reorder1_a.json 2> gpurun_out/bench_reorder1_a.err
timeout -k 10 200 python bench.py --mode infer --steps 10 --warmup 2 > gpurun_out/bench_infer_a.json 2> gpurun_out/bench_infer_a.err
tail -3 gpurun_out/store_tests_a.txt; cat gpurun_out/bench_reorder*_a.json gpurun_out/bench_infer_a.json
cat gpurun_out/agg_ab_a.txt
