#!/bin/bash
# PMC comparison of the register-staged f16x3 GEMM (staging -1) and the LDS-DMA variant
# (staging $1, default 0) on the forward SAGE shape, one rocprofv3 pass per counter group.
# Usage (GPU box): bash tools/pmc_h3g.sh [variant] ; tables in gpurun_out/pmc_h3g.txt
set -e
cd $GRAFT_REPO_ROOT
V=${1:-0}
OUT=gpurun_out/pmc_h3g_v$V
bash tools/pmc_passes.sh $OUT \
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS" \
  "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_MFMA GRBM_GUI_ACTIVE" \
  "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" \
  -- python tools/gemm_ab.py --reps 5 --no-flush --shapes fwd --variants=-1,$V
for k in k_gemm_x6 k_gemm_h3g; do
  echo "== $k (variant $V)" >> gpurun_out/pmc_h3g.txt
  python tools/pmc_table.py $OUT $k >> gpurun_out/pmc_h3g.txt
done
