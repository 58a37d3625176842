set -e
cd $GRAFT_REPO_ROOT
for v in "2 1" "2 401" "2 501" "1 1"; do
  set -- $v
  timeout -k 10 60 python tools/gemm_one.py $1 $2 fwd 20 >> gpurun_out/gemm_one.log 2>&1
  bash tools/pmc_passes.sh gpurun_out/pmc_m$1_c$2 "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" -- python tools/gemm_one.py $1 $2 fwd 10
  python tools/pmc_table.py gpurun_out/pmc_m$1_c$2 k_gemm_x6 >> gpurun_out/pmc_gemm.txt
done
