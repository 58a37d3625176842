#!/bin/bash
# round 6 record ap: slot reductions (k_reduce_slots) with 32 slot loads in flight per thread: the
# BN / bias-gradient GPU tests, then a cfg2 bench and its kernel trace
set -o pipefail
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_bn.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > $O/r06ap_tests.txt 2>&1 &&
timeout -k 10 200 python bench.py --no-cpu-baseline --no-cfg3 --steps 40 > $O/r06ap_bench.json 2> $O/r06ap_bench.err &&
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$O/prof_r06ap -o run -- python bench.py --no-cpu-baseline --no-cfg3 --steps 10 --warmup 3 > $O/r06ap_prof.json 2> $O/r06ap_prof.err
