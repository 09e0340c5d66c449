# development: bit-plane activation paths (fused unpack, import kernel) -- parity, then timings
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_planes.py tests/test_gpu_wrapper.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pl_tests.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "bit_packing or import or bmma" --timeout 120 --timeout-method thread >> gpurun_out/pl_tests.log 2>&1 && \
PB_M=8,16 timeout -k 10 250 python tools/planes_bench.py > gpurun_out/pl_bench.txt 2>&1
