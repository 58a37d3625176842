#!/bin/bash
# round 6 record ak: bench.py's per-launch timers on fence-free HIP events (default) against
# torch.cuda.Event (--torch-events), alternating, same box; then a kernel trace of the default
set -o pipefail
O=gpurun_out
A="--no-cpu-baseline --no-cfg3 --steps 30 --warmup 5"
timeout -k 10 200 python bench.py $A > $O/r06ak_hip1.json 2> $O/r06ak_hip1.err &&
timeout -k 10 200 python bench.py $A --torch-events > $O/r06ak_torch1.json 2> $O/r06ak_torch1.err &&
timeout -k 10 200 python bench.py $A > $O/r06ak_hip2.json 2> $O/r06ak_hip2.err &&
timeout -k 10 200 python bench.py $A --torch-events > $O/r06ak_torch2.json 2> $O/r06ak_torch2.err &&
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$O/prof_r06ak -o run -- python bench.py --no-cpu-baseline --no-cfg3 --steps 10 --warmup 3 > $O/r06ak_prof.json 2> $O/r06ak_prof.err
