set -e
timeout -k 10 200 python tools/agg_knob_ab.py --rounds 12 "" "14=1" "15=1280" "14=1;15=1280" > gpurun_out/agg_ab_a.txt 2>&1
timeout -k 10 200 python tools/agg_knob_ab.py --rounds 12 --group-rows 8 "" >> gpurun_out/agg_ab_a.txt 2>&1
timeout -k 10 200 python tools/agg_knob_ab.py --rounds 12 --group-rows 8 --reorder "" >> gpurun_out/agg_ab_a.txt 2>&1
timeout -k 10 200 python tools/agg_knob_ab.py --rounds 12 --group-rows 4 --reorder "" >> gpurun_out/agg_ab_a.txt 2>&1
cat gpurun_out/agg_ab_a.txt
