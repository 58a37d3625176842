#!/bin/bash
# Collect PMC counter groups for a command, one rocprofv3 pass per group (counters only,
# with kernel trace for durations; no tracing domains mixed in).
# Usage: tools/pmc_passes.sh OUTDIR "CTR_A CTR_B" "CTR_C" ... -- python script.py args...
set -e
OUT=$1; shift
GRPS=()
while [ "$1" != "--" ]; do GRPS+=("$1"); shift; done
shift
export TMPDIR=/tmp
ROOT=$(pwd)
i=0
for g in "${GRPS[@]}"; do
  i=$((i+1))
  mkdir -p "$OUT/pass$i"
  (timeout -k 10 90 rocprofv3 --kernel-trace --pmc $g --output-format csv -d "$ROOT/$OUT/pass$i" -o run \
      -- "$@" > "$ROOT/$OUT/pass$i/stdout.log" 2>&1)
done
