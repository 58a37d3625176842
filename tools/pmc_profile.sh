#!/bin/bash
# Collect PMC counters for a command in separate rocprofv3 passes (counters only, no
# tracing domains mixed in). Usage: tools/pmc_profile.sh OUTDIR -- python script.py args...
# Each pass writes OUTDIR/passN/*counter_collection.csv; summarise with tools/pmc_summary.py.
set -e
OUT=$(realpath -m "$1"); shift
[ "$1" == "--" ] && shift
export TMPDIR=/tmp
ROOT=$(pwd)
PASSES=(
  "FETCH_SIZE GRBM_GUI_ACTIVE"
  "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
  "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_REQ_sum TCC_READ_sum"
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VALU"
  "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM"
)
i=0
for p in "${PASSES[@]}"; do
  i=$((i+1))
  mkdir -p "$OUT/pass$i"
  (cd /tmp && timeout -k 10 300 rocprofv3 --pmc $p --output-format csv -d "$OUT/pass$i" -o run -- "$@" > "$OUT/pass$i/stdout.log" 2>&1) || true
done
