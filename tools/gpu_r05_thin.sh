# round-5: the plain chain's poll behind ring block 0 only (FQ_CHAIN_THIN) against HEAD
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_layers.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_thin_tests.log 2>&1 || { tail -30 gpurun_out/r05_thin_tests.log; exit 1; }
tail -1 gpurun_out/r05_thin_tests.log
timeout -k 10 700 bash tools/ab.sh step 3 flexq_amd/libflexq_hip.so tools/libflexq_hip_head.so > gpurun_out/r05_thin_ab.txt 2>&1
cat gpurun_out/r05_thin_ab.txt
