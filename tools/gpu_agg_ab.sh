set -e
# aggregation knob A/B (tools/agg_knob_ab.py); round-4 record: profiles/r04_ab_agg_knobs.txt
timeout -k 10 200 python tools/agg_knob_ab.py --rounds 12 "" "7=2048" > gpurun_out/agg_ab.txt 2>&1
timeout -k 10 200 python tools/agg_knob_ab.py --rounds 12 --group-rows 8 --reorder "" >> gpurun_out/agg_ab.txt 2>&1
cat gpurun_out/agg_ab.txt
