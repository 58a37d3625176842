#!/bin/bash
# Round-2 experiments: SAG tests, an N=2 rehearsal of the distributed bench on one GPU (gloo),
# row-group kernel knobs (isolated with cache flushes, then inside the train step).
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_sag.py tests/test_gpu_spmm.py tests/test_gpu_store.py -q --timeout 120 --timeout-method thread > gpurun_out/misc_tests.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
BGNN_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline \
  > gpurun_out/bench_n2_gloo.json 2> gpurun_out/bench_n2_gloo.err || exit $?
timeout -k 10 200 python tools/tune_agg.py --flush --rounds 10 \
  --variants group4_b1024,group4_b1024_u16,group4_b1024_ze,group4_b1024_u16_ze > gpurun_out/tune_agg_knobs.txt 2>&1 || exit $?
timeout -k 10 300 python tools/ab_step.py "knob:10=8;knob:11=0" "knob:10=16;knob:11=0" "knob:10=8;knob:11=1" "knob:10=16;knob:11=1" > gpurun_out/ab_group.txt 2>&1
