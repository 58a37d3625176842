set -e
timeout -k 10 250 python tools/gemm_cfg_ab.py --cfgs=-1,1,2 --rounds 8 --shapes dgrad,dropadd > gpurun_out/gemm_cfg_i.txt 2>&1
grep -v amdgpu.ids gpurun_out/gemm_cfg_i.txt
bash tools/gpu_r4p.sh i kt
