set -e
# PMC anatomy of the four SAGE GEMM shapes (tools/gemm_cfg_ab.py, default plans), two passes
TAG=${1:-p}
bash tools/pmc_passes.sh gpurun_out/pmc_gemm_$TAG "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU" "SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM" -- python tools/gemm_cfg_ab.py --cfgs=-1 --rounds 3
python tools/pmc_summary.py gpurun_out/pmc_gemm_$TAG k_gemm_x6 > gpurun_out/pmc_gemm_$TAG.txt
cat gpurun_out/pmc_gemm_$TAG.txt
