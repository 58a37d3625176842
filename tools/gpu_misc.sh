#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python tools/ab_step.py "bgnn.fused.FUSED_MLP2=True" > gpurun_out/ab_wprep.txt 2>&1
