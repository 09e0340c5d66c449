# Fused quantizer: lazy chunks (default) vs every chunk before the stream (FQ_LAZY_ABL=1), A/B x 3
set -e
S="4096 11008 8192 8192 10240 8192 4096 4096 12288 4096"
for i in 1 2 3; do
  for L in flexq_amd/libflexq_hip.so tools/libflexq_hip_nolazy.so; do
    FQ_LIB=$L timeout -k 10 150 python3 -u tools/shape_sweep.py 1 $S | grep -v amdgpu.ids
  done
done
