#!/bin/bash
# One GPU call: parity tests, smoke, bench (JSON), rocprofv3 kernel stats of a short bench.
# Usage (on the GPU box, from the repo root): bash tools/gpu_round.sh TAG
set -e
TAG=${1:-run}
mkdir -p gpurun_out
# assertion failures (pytest rc 1) do not stop the measurement; a crash, fault or timeout does
rc=0
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/gpu_tests_$TAG.log 2>&1 || rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "gpu tests ended with rc=$rc"; exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
timeout -k 10 240 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
timeout -k 10 240 python bench.py --path per_op --no-cpu-baseline > gpurun_out/bench_perop_$TAG.json 2> gpurun_out/bench_perop_$TAG.err
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_$TAG" -o run -- python "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline > "$ROOT/gpurun_out/prof_bench_$TAG.json" 2>&1
cd "$ROOT" && python tools/gemm_launches.py "$(find gpurun_out/prof_$TAG -name '*kernel_trace.csv' | head -1)" 80656 gpurun_out/gemm_launches_$TAG.json > /dev/null
cd /tmp
# PMC traffic of the bench's roofline kernels (separate counter-only passes)
if [ "${PMC:-1}" = "1" ]; then
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$ROOT/gpurun_out/pmc_$TAG/fetch" -o run -- python "$ROOT/bench.py" --steps 3 --warmup 2 --no-cpu-baseline > /dev/null 2>&1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$ROOT/gpurun_out/pmc_$TAG/write" -o run -- python "$ROOT/bench.py" --steps 3 --warmup 2 --no-cpu-baseline > /dev/null 2>&1
  cd "$ROOT" && python tools/traffic.py "gpurun_out/pmc_$TAG" "gpurun_out/traffic_$TAG.json" > /dev/null
fi
