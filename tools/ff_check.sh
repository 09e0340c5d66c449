# development: fp16 fused quantizer forced at M <= 8 (variant) vs the cost model's choice
set -o pipefail
mkdir -p gpurun_out
PB_M=2,4,8 timeout -k 10 200 python tools/planes_bench.py > gpurun_out/ff_default.txt 2>&1 && \
PB_M=2,4,8 FLEXQ_AMD_LIB=tools/libflexq_hip_ff.so timeout -k 10 200 python tools/planes_bench.py > gpurun_out/ff_forced.txt 2>&1
