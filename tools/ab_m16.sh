# M = 16 decode GEMM (pre-quantized, the C3 launch) under ring-budget variants (development A/B)
set -e
S="4096 4096 12288 4096 22016 4096 4096 11008"
for i in 1 2; do
  for L in flexq_amd/libflexq_hip.so tools/libflexq_hip_rb9k.so tools/libflexq_hip_rb18k4.so; do
    FQ_SWEEP=gemm FQ_LIB=$L timeout -k 10 120 python3 -u tools/shape_sweep.py 16 $S | grep -v amdgpu.ids
  done
done
