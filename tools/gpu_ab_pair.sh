set -e
bash tools/gpu_gemm_ab.sh g
bash tools/gpu_agg_ab.sh f
