# development: parity of the 32x32x32 prefill core variants, then an A/B against the default build
set -o pipefail
mkdir -p gpurun_out
FLEXQ_AMD_LIB=tools/libflexq_hip_pb32.so timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "prefill" --timeout 300 --timeout-method thread > gpurun_out/pb32_tests.log 2>&1 && \
FLEXQ_AMD_LIB=tools/libflexq_hip_pb32s.so timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "prefill" --timeout 300 --timeout-method thread > gpurun_out/pb32s_tests.log 2>&1 && \
timeout -k 10 700 bash tools/ab_prefill.sh flexq_amd/libflexq_hip.so tools/libflexq_hip_pb32.so tools/libflexq_hip_pb32s.so > gpurun_out/pb32_ab.txt 2>&1
