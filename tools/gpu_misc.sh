#!/bin/bash
# SAG tests, an N=2 rehearsal of the distributed bench on one GPU (gloo), aggregation grid sweep.
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_sag.py -q --timeout 120 --timeout-method thread > gpurun_out/sag_tests.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
BGNN_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline \
  > gpurun_out/bench_n2_gloo.json 2> gpurun_out/bench_n2_gloo.err || exit $?
timeout -k 10 200 python tools/tune_agg.py --flush --rounds 10 \
  --variants group4_b512,group4_b768,group4_b1024,group4_b2048,group8_b1024,sweep12 > gpurun_out/tune_agg_flush.txt 2>&1
