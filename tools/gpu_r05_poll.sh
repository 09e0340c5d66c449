# round-5: the chain polls with every load in flight at once, against round 4's library (A/B in one run)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_layers.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_chain_tests4.log 2>&1 || { tail -30 gpurun_out/r05_chain_tests4.log; exit 1; }
tail -1 gpurun_out/r05_chain_tests4.log
timeout -k 10 700 bash tools/ab.sh step 3 flexq_amd/libflexq_hip.so tools/libflexq_hip_r04.so > gpurun_out/r05_poll_ab.txt 2>&1
timeout -k 10 500 bash tools/ab.sh e2e 2 flexq_amd/libflexq_hip.so tools/libflexq_hip_r04.so >> gpurun_out/r05_poll_ab.txt 2>&1
cat gpurun_out/r05_poll_ab.txt
