#!/bin/bash
# kernel statistics of the per-op path (the PyG-surface SAGEConv module graph): which kernels run
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_perop_${TAG:-y}" -o run -- python "$ROOT/bench.py" --path per_op --steps 5 --warmup 2 --no-cpu-baseline > "$ROOT/gpurun_out/prof_perop_${TAG:-y}.json" 2>&1
