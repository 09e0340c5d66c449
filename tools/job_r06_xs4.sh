# round-6: the refined rows-in-slots rule -- decode parity tests, then M = 8 / 12 / 16 one-item launches
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_dispatch_sweep.py tests/test_gpu_kernels.py tests/test_gpu_wrapper.py tests/test_gpu_planes.py -x -q --timeout 200 --timeout-method thread > gpurun_out/xs4_tests.log 2>&1 || { tail -30 gpurun_out/xs4_tests.log; exit 1; }
tail -1 gpurun_out/xs4_tests.log
for M in 8 12 16; do FQ_SWEEP=gemm timeout -k 10 120 python3 -u tools/shape_sweep.py $M 4096 4096 4096 11008 2048 8192 12288 4096 2>&1 | grep us/launch || exit 1; done | tee gpurun_out/r06_xs_rule.txt
