set -o pipefail
M16=$PWD/buck-gnn_amd/bgnn/_lib/libbgnn_m16.so
timeout -k 10 300 python -u tools/fold_ab.py GraphSage_addAggr_Shared > gpurun_out/r06c_fold_default.txt 2>&1 &&
BGNN_LIBRARY=$M16 timeout -k 10 300 python -u tools/fold_ab.py GraphSage_addAggr_Shared > gpurun_out/r06c_fold_m16.txt 2>&1 &&
FOLD_INMODEL=1 timeout -k 10 300 python -u tools/fold_ab.py GraphSage_addAggr_Shared > gpurun_out/r06c_inmodel_default.txt 2>&1 &&
FOLD_INMODEL=1 BGNN_LIBRARY=$M16 timeout -k 10 300 python -u tools/fold_ab.py GraphSage_addAggr_Shared > gpurun_out/r06c_inmodel_m16.txt 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r06c_bench.json 2> gpurun_out/r06c_bench.err &&
bash tools/pmc_passes.sh gpurun_out/r06c_pmc "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA" "SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM" -- python bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-cfg3 &&
python tools/pmc_summary.py gpurun_out/r06c_pmc k_gemm_x6 > gpurun_out/r06c_pmc_gemm.txt
