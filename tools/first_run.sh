# First vs later bench runs in one fresh-box session (development): is the first run slower?
B="python3 -u bench.py --cpu-budget 0 --no-fp16-compare --no-layers --no-extra-configs --no-calibrate"
for i in 1 2 3; do
  timeout -k 10 200 $B 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('run', $i, d['ms_per_step'], d['roofline']['per_launch_us'])" || exit 1
done
