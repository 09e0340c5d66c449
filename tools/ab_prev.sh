set -e
S="4096 4096 12288 4096 22016 4096 4096 11008"
for i in 1 2; do
  timeout -k 10 120 python -u tools/shape_sweep.py 1 $S
  FQ_LIB=tools/libflexq_hip_prev.so timeout -k 10 120 python -u tools/shape_sweep.py 1 $S
done
