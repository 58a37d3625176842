#!/bin/bash
# round 6 record an: longer same-process step A/B of buckgnn.FUSED_POOL (15 rounds, cfg2 then cfg3)
set -o pipefail
O=gpurun_out
AB_ROUNDS=15 timeout -k 10 400 python -u tools/ab_step.py "bgnn.buckgnn.FUSED_POOL=True" "bgnn.buckgnn.FUSED_POOL=False" > $O/r06an_ab_cfg2.txt 2>&1 &&
AB_ROUNDS=15 AB_CONFIG=cfg3 timeout -k 10 400 python -u tools/ab_step.py "bgnn.buckgnn.FUSED_POOL=True" "bgnn.buckgnn.FUSED_POOL=False" > $O/r06an_ab_cfg3.txt 2>&1
