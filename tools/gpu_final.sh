set -e
# end-of-round check of the committed tree: every GPU test, smoke, the cfg2 bench line
TAG=${1:-z}
rc=0
timeout -k 10 500 python -u -m pytest tests -m gpu -q -s --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || rc=$?
tail -3 gpurun_out/gpu_tests_$TAG.log; grep "largest gradient error" gpurun_out/gpu_tests_$TAG.log || true
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
python -c "import json; d=json.loads(open('gpurun_out/bench_$TAG.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline']['value'])"
exit $rc
