# M = 1 decode: dequantize only the stored accumulator vs all four (FQ_M1_ABL=1 build), A/B/A/B
set -e
S="4096 4096 12288 4096 22016 4096 4096 11008"
for i in 1 2 3; do
  for L in flexq_amd/libflexq_hip.so tools/libflexq_hip_m1old.so; do
    FQ_LIB=$L timeout -k 10 120 python3 -u tools/shape_sweep.py 1 $S | grep -v amdgpu.ids
  done
done
