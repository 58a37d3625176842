#!/bin/bash
# f16x3 tile configs of the folded first-layer GEMMs (K_in = 128), cache flushed between launches
export GEMM_FLUSH=1
for shape in fold_fwd fold_dgrad; do
  for cfg in 0 1 2 4; do
    timeout -k 10 60 python tools/gemm_one.py 2 $cfg $shape 20 || exit $?
  done
done
for cfg in 0 1 4; do timeout -k 10 60 python tools/gemm_one.py 2 $cfg fold_wgrad 20 || exit $?; done
