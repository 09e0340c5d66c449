# Argument preloading for every kernel (development): this build vs HEAD's, the batch-16 step
# (one quantize launch per linear) and the decoder layers end to end, A/B x 3
B="python3 -u bench.py --cpu-budget 0 --no-fp16-compare --no-extra-configs --no-calibrate"
for i in 1 2 3; do
  for L in flexq_amd/libflexq_hip.so tools/libflexq_hip_head.so; do
    printf "%s " $L; FLEXQ_AMD_LIB=$L timeout -k 10 300 $B --config llama2-7b-m16 --steps 10 --warmup 3 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('m16', d['ms_per_step'], 'e2e', d['decoder_layers_e2e']['M1']['w6_ms_per_step'], d['decoder_layers_e2e']['M16']['w6_ms_per_step'])" || exit 1
  done
done
