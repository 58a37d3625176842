ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_ea5_${TAG:-d}" -o run -- python "$ROOT/bench.py" --model EA_GNN --bf16 --config cfg5 --steps 3 --warmup 1 --no-cpu-baseline > "$ROOT/gpurun_out/prof_ea5_${TAG:-d}.json" 2>&1
