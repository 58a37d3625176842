set -e
# aggregation A/B (tools/agg_knob_ab.py): row groups of 4 in dataset order against row groups of 8
# (k_seg_group<.., 8, 4>) in dataset order and in cluster_order; round-4 record profiles/r04_ab_agg_*.txt
TAG=${1:-f}
timeout -k 10 200 python tools/agg_knob_ab.py --rounds 12 "" > gpurun_out/agg_ab_$TAG.txt 2>&1
timeout -k 10 200 python tools/agg_knob_ab.py --rounds 12 --group-rows 8 "" >> gpurun_out/agg_ab_$TAG.txt 2>&1
timeout -k 10 200 python tools/agg_knob_ab.py --rounds 12 --group-rows 8 --reorder "" >> gpurun_out/agg_ab_$TAG.txt 2>&1
grep -v amdgpu.ids gpurun_out/agg_ab_$TAG.txt
