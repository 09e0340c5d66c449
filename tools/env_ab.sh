#!/bin/bash
# Runtime-knob A/B of the default decode bench (development): one bench line per setting.
B="python3 bench.py --no-fp16-compare --no-layers --cpu-budget 0 --no-calibrate --steps 50"
run() { echo "== $1"; env $1 timeout -k 10 120 $B 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['per_launch_us'])"; }
for s in "X=0" "HIP_FORCE_DEV_KERNARG=1" "HIP_FORCE_DEV_KERNARG=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1" "X=0"; do run "$s" || exit 1; done
