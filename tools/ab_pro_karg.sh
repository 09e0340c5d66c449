# Fused producers' kernel argument list (development): this build vs HEAD's build, producer
# microbench and the 32-layer e2e step, A/B x 2
for i in 1 2; do
  for L in flexq_amd/libflexq_hip.so tools/libflexq_hip_head.so; do
    echo "== $L"
    FLEXQ_AMD_LIB=$L timeout -k 10 200 python3 -u tools/fusedpro_bench.py 2>/dev/null | grep -v amdgpu || exit 1
    FLEXQ_AMD_LIB=$L timeout -k 10 300 python3 -u bench.py --cpu-budget 0 --no-fp16-compare --no-extra-configs --no-calibrate --steps 5 --warmup 2 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('step', d['ms_per_step'], 'e2e', d['decoder_layers_e2e']['M1']['w6_ms_per_step'], d['decoder_layers_e2e']['M16']['w6_ms_per_step'])" || exit 1
  done
done
