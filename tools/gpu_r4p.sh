#!/bin/bash
# Round-4 profiles: rocprofv3 kernel traces (cfg2, cfg3, per-op Shared, per-op bgnn BN, EA cfg5 bf16)
# and PMC traffic passes (FETCH_SIZE / WRITE_SIZE in separate runs) for cfg2, cfg3 and EA cfg5.
# Usage (GPU box, repo root): bash tools/gpu_r4p.sh TAG {kt|pmc}
set -e
TAG=${1:-c}
PHASE=${2:-kt}
ROOT=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
KT() { local name=$1; shift; timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_${name}_$TAG" -o run -- python "$ROOT/bench.py" "$@" --no-cpu-baseline > "$ROOT/gpurun_out/prof_${name}_$TAG.json" 2>&1; echo "kt $name ok"; }
PMC() { local name=$1; shift; for c in FETCH_SIZE WRITE_SIZE; do d=fetch; [ $c = WRITE_SIZE ] && d=write; timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d "$ROOT/gpurun_out/pmc_${name}_$TAG/$d" -o run -- python "$ROOT/bench.py" "$@" --no-cpu-baseline > "$ROOT/gpurun_out/pmc_${name}_$TAG/$d.log" 2>&1; done; echo "pmc $name ok"; }
if [ "$PHASE" = kt ]; then
KT cfg2 --steps 10 --warmup 3
KT cfg3 --config cfg3 --steps 10 --warmup 3
KT perop_shared --path per_op --model GraphSage_addAggr_Shared --steps 5 --warmup 2
KT perop_bgnnbn --path per_op --bn bgnn --steps 5 --warmup 2
KT ea5 --model EA_GNN --bf16 --config cfg5 --steps 3 --warmup 1
cd "$ROOT"
exit 0
fi
mkdir -p "$ROOT/gpurun_out/pmc_cfg2_$TAG" "$ROOT/gpurun_out/pmc_cfg3_$TAG" "$ROOT/gpurun_out/pmc_ea5_$TAG"
PMC cfg2 --steps 3 --warmup 1
PMC cfg3 --config cfg3 --steps 3 --warmup 1
PMC ea5 --model EA_GNN --bf16 --config cfg5 --steps 2 --warmup 1
cd "$ROOT"
for n in cfg2 cfg3 ea5; do python tools/traffic.py gpurun_out/pmc_${n}_$TAG gpurun_out/traffic_${n}_$TAG.json > /dev/null && echo "traffic $n ok"; done
timeout -k 10 200 python tools/host_profile.py --steps 20 > gpurun_out/host_profile_$TAG.txt 2>&1 && echo "host profile ok"
