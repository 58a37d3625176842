#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_ea_train.py tests/test_gpu_model.py -q --timeout 120 --timeout-method thread > gpurun_out/ea_tests.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --model EA_GNN --bf16 --config cfg5 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/bench_ea_cfg5_bf16_c.json 2> gpurun_out/bench_ea_c.err || exit $?
timeout -k 10 300 python -c "import sys, runpy; sys.argv=['bench.py','--model','EA_GNN','--bf16','--config','cfg5','--steps','6','--warmup','2','--no-cpu-baseline']; sys.path.insert(0,'buck-gnn_amd'); import bgnn.ea as E; E.FUSED_SKIP_DROPOUT=False; runpy.run_path('bench.py', run_name='__main__')" > gpurun_out/bench_ea_cfg5_bf16_noskipdrop.json 2>> gpurun_out/bench_ea_c.err
