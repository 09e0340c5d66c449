# Kernel-argument preloading into SGPRs (development): this build (56-byte list, fully preloaded), HEAD,
# and a packed-argument build with preload; headline step A/B x 3
B="python3 -u bench.py --cpu-budget 0 --no-fp16-compare --no-layers --no-extra-configs --no-calibrate"
for i in 1 2 3; do
  for L in flexq_amd/libflexq_hip.so tools/libflexq_hip_head.so tools/libflexq_hip_pkkp.so; do
    printf "%s " $L; FLEXQ_AMD_LIB=$L timeout -k 10 200 $B 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['per_launch_us'])" || exit 1
  done
done
