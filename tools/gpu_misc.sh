#!/bin/bash
# Round-2 A/B inside the train step: the skip gradient added in the dgrad epilogue (drop-add) or
# written by bgnn_sage_bwd_rows and read back.
mkdir -p gpurun_out
timeout -k 10 300 python tools/ab_step.py "bgnn.fused.DGRAD_DROPADD=True" "bgnn.fused.DGRAD_DROPADD=False" > gpurun_out/ab_dropadd.txt 2>&1
