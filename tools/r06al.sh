#!/bin/bash
# round 6 record al: per-launch roofline events on every 4th timed step (default) against every step,
# fence-free HIP events against torch.cuda.Event, alternating, same box
set -o pipefail
O=gpurun_out
A="--no-cpu-baseline --no-cfg3 --steps 40 --warmup 5"
timeout -k 10 200 python bench.py $A > $O/r06al_e4a.json 2> $O/r06al_e4a.err &&
timeout -k 10 200 python bench.py $A --timer-every 1 > $O/r06al_e1a.json 2> $O/r06al_e1a.err &&
timeout -k 10 200 python bench.py $A --timer-every 1 --torch-events > $O/r06al_t1a.json 2> $O/r06al_t1a.err &&
timeout -k 10 200 python bench.py $A --timer-every 1000 > $O/r06al_e0a.json 2> $O/r06al_e0a.err &&
timeout -k 10 200 python bench.py $A > $O/r06al_e4b.json 2> $O/r06al_e4b.err &&
timeout -k 10 200 python bench.py $A --timer-every 1 > $O/r06al_e1b.json 2> $O/r06al_e1b.err &&
timeout -k 10 200 python bench.py $A --timer-every 1 --torch-events > $O/r06al_t1b.json 2> $O/r06al_t1b.err &&
timeout -k 10 200 python bench.py $A --timer-every 1000 > $O/r06al_e0b.json 2> $O/r06al_e0b.err
