set -o pipefail
M16=$PWD/buck-gnn_amd/bgnn/_lib/libbgnn_m16.so
BGNN_LIBRARY=$M16 timeout -k 10 200 python -u tools/m16_precision.py > gpurun_out/r06d_m16lib_precision.txt 2>&1 &&
FOLD_INMODEL=1 timeout -k 10 300 python -u tools/fold_ab.py GraphSage_addAggr_Shared > gpurun_out/r06d_inmodel_default.txt 2>&1 &&
FOLD_INMODEL=1 BGNN_LIBRARY=$M16 timeout -k 10 300 python -u tools/fold_ab.py GraphSage_addAggr_Shared > gpurun_out/r06d_inmodel_m16.txt 2>&1
