# Headline step per build (development bisection): ms/step and per-launch us, twice each
B="python3 -u bench.py --cpu-budget 0 --no-fp16-compare --no-layers --no-extra-configs --no-calibrate"
for i in 1 2; do
  for L in tools/libflexq_hip_r2.so tools/libflexq_hip_ef08e1a.so tools/libflexq_hip_0a43314.so tools/libflexq_hip_e45a36a.so tools/libflexq_hip_7f0e966.so flexq_amd/libflexq_hip.so; do
    printf "%s " $L; FLEXQ_AMD_LIB=$L timeout -k 10 200 $B 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['per_launch_us'])" || exit 1
  done
done
