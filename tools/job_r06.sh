# round-6 development job: chain + dispatch tests, the NaN-on-failure A/B, the mid-M rule's launches
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_dispatch_sweep.py tests/test_gpu_chain.py tests/test_gpu_planes.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r06_j4_tests.log 2>&1 || { tail -30 gpurun_out/r06_j4_tests.log; exit 1; }
tail -1 gpurun_out/r06_j4_tests.log
AB_OUT=gpurun_out/r06_chain_nan_ab.txt timeout -k 10 500 bash tools/ab.sh step 3 flexq_amd/libflexq_hip.so abtmp/libflexq_hip_nonan.so || exit 1
FQ_SWEEP=gemm timeout -k 10 200 python -u tools/shape_sweep.py 64 4096 4096 12288 4096 22016 4096 4096 11008 > gpurun_out/r06_m64.txt 2>&1 || exit 1
FQ_SWEEP=gemm timeout -k 10 200 python -u tools/shape_sweep.py 128 4096 4096 12288 4096 22016 4096 4096 11008 >> gpurun_out/r06_m64.txt 2>&1 || exit 1
FQ_SWEEP=gemm timeout -k 10 200 python -u tools/shape_sweep.py 48 4096 4096 12288 4096 22016 4096 4096 11008 >> gpurun_out/r06_m64.txt 2>&1 || exit 1
cat gpurun_out/r06_m64.txt | grep us/launch
