set -e
timeout -k 10 250 python tools/gemm_cfg_ab.py --cfgs=-1 --l2pf 0,0x11,0x13 --rounds 8 > gpurun_out/gemm_ab_d1.txt 2>&1
timeout -k 10 250 python tools/gemm_cfg_ab.py --cfgs=-1 --l2pf 0,0x11,0x13 --rounds 8 --rows 80640 > gpurun_out/gemm_ab_d2.txt 2>&1
cat gpurun_out/gemm_ab_d1.txt gpurun_out/gemm_ab_d2.txt
