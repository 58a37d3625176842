#!/bin/bash
# The one GPU-box check script (replaces the per-round one-offs): runs the named steps in order,
# each under its own time limit, and stops at the first crash, fault or time-out.
#
#   bash tools/gpu_check.sh TAG [STEP ...]        (on the GPU box, from the repo root)
#
# Steps (default: tests smoke bench prof):
#   tests      pytest -m gpu over ${TESTS:-tests} (PYTEST_ARGS adds arguments); assertion failures
#              (rc 1) are reported and do not stop the later measurements
#   smoke      __graft_entry__.smoke()
#   bench      python bench.py (the driver's line; BENCH_ARGS adds arguments)
#   cfg3       bench.py --config cfg3
#   max        bench.py --model GraphSage_maxAggr
#   shared     bench.py --model GraphSage_addAggr_Shared
#   mean       bench.py --model GraphSage_meanAggr
#   perop      bench.py --path per_op (the reference's Models/BuckGNN.py module graph under the shim)
#   ea5        bench.py --model EA_GNN --bf16 --config cfg5
#   infer      bench.py --mode infer
#   prof       rocprofv3 kernel trace + stats of the cfg2 bench, GEMM launch table
#   profmax    the same for GraphSage_maxAggr
#   profperop  the same for the per-op path
#   profcfg3   the same for cfg3
#   profea5    the same for EA_GNN cfg5 bf16
#   pmc        FETCH_SIZE and WRITE_SIZE passes of the cfg2 bench -> gpurun_out/traffic_TAG.json
#   pmcgemm    SQ counter passes of the SAGE GEMM shapes (tools/pmc_passes.sh, tools/gemm_cfg_ab.py)
# Outputs land in gpurun_out/ named by step and TAG.
set -o pipefail
TAG=${1:-run}
shift || true
STEPS=${*:-tests smoke bench prof}
ROOT=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp

die() { echo "step $1 ended with rc=$2"; exit "$2"; }

bench() {   # bench NAME SECONDS ARGS...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" python bench.py "$@" ${BENCH_ARGS:-} > "gpurun_out/bench_${name}_$TAG.json" \
    2> "gpurun_out/bench_${name}_$TAG.err" || die "$name" $?
  tail -c 400 "gpurun_out/bench_${name}_$TAG.json"; echo
}

prof() {   # prof NAME SECONDS ARGS...
  local name=$1 secs=$2; shift 2
  (cd /tmp && timeout -k 10 "$secs" rocprofv3 --kernel-trace --stats --output-format csv \
     -d "$ROOT/gpurun_out/prof_${name}_$TAG" -o run -- python "$ROOT/bench.py" "$@" ${BENCH_ARGS:-} \
     > "$ROOT/gpurun_out/prof_bench_${name}_$TAG.json" 2>&1) || die "prof_$name" $?
}

for s in $STEPS; do
  echo "== $s ($(date +%T))"
  case $s in
    tests)
      rc=0
      timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -q -rA --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} \
        > "gpurun_out/gpu_tests_$TAG.log" 2>&1 || rc=$?
      tail -3 "gpurun_out/gpu_tests_$TAG.log"
      if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then die tests $rc; fi ;;
    smoke)
      timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "gpurun_out/smoke_$TAG.log" 2>&1 \
        || die smoke $?
      tail -1 "gpurun_out/smoke_$TAG.log" ;;
    bench) bench cfg2 400 ;;
    cfg3) bench cfg3 300 --config cfg3 --no-cpu-baseline ;;
    max) bench max 300 --model GraphSage_maxAggr --no-cpu-baseline ;;
    shared) bench shared 300 --model GraphSage_addAggr_Shared --no-cpu-baseline ;;
    mean) bench mean 300 --model GraphSage_meanAggr --no-cpu-baseline ;;
    perop) bench perop 300 --path per_op --no-cpu-baseline ;;
    ea5) bench ea5 400 --model EA_GNN --bf16 --config cfg5 --steps 6 --warmup 2 --no-cpu-baseline ;;
    infer) bench infer 300 --mode infer --no-cpu-baseline ;;
    prof)
      prof cfg2 300 --steps 10 --warmup 3 --no-cpu-baseline --no-cfg3
      python tools/gemm_launches.py "$(find gpurun_out/prof_cfg2_$TAG -name '*kernel_trace.csv' | head -1)" 80656 \
        "gpurun_out/gemm_launches_$TAG.json" > /dev/null || true ;;
    profmax) prof max 300 --model GraphSage_maxAggr --steps 5 --warmup 2 --no-cpu-baseline ;;
    profperop) prof perop 300 --path per_op --steps 5 --warmup 2 --no-cpu-baseline ;;
    profcfg3) prof cfg3 300 --config cfg3 --steps 10 --warmup 3 --no-cpu-baseline ;;
    profea5) prof ea5 400 --model EA_GNN --bf16 --config cfg5 --steps 3 --warmup 1 --no-cpu-baseline ;;
    pmc)
      (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$ROOT/gpurun_out/pmc_$TAG/fetch" \
         -o run -- python "$ROOT/bench.py" --steps 3 --warmup 2 --no-cpu-baseline --no-cfg3 > /dev/null 2>&1) || die pmc_fetch $?
      (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$ROOT/gpurun_out/pmc_$TAG/write" \
         -o run -- python "$ROOT/bench.py" --steps 3 --warmup 2 --no-cpu-baseline --no-cfg3 > /dev/null 2>&1) || die pmc_write $?
      python tools/traffic.py "gpurun_out/pmc_$TAG" "gpurun_out/traffic_$TAG.json" > /dev/null || true ;;
    pmcgemm)   # SQ counter anatomy of the SAGE GEMM shapes (default plans), two counter passes
      bash tools/pmc_passes.sh "gpurun_out/pmc_gemm_$TAG" "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU" \
        "SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM" \
        -- python tools/gemm_cfg_ab.py --cfgs=-1 --rounds 3 || die pmcgemm $?
      python tools/pmc_summary.py "gpurun_out/pmc_gemm_$TAG" k_gemm_x6 > "gpurun_out/pmc_gemm_$TAG.txt" || true ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "done ($(date +%T))"
