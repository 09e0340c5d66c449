# round-5: (1) the 256 x 256 prefill kernel with buffer-addressed DMA, immediate-offset row reads and
# the op_sel scale product; (2) the decode chain's next ring issued by each linear's tail
# (chain_ring_ahead) -- both A/B against HEAD's library (tools/libflexq_hip_head.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05_pf_tests.log 2>&1 || { tail -30 gpurun_out/r05_pf_tests.log; exit 1; }
tail -1 gpurun_out/r05_pf_tests.log
timeout -k 10 400 bash tools/ab.sh prefill 2 flexq_amd/libflexq_hip.so tools/libflexq_hip_head.so > gpurun_out/r05_pf_ab.txt 2>&1
cat gpurun_out/r05_pf_ab.txt
timeout -k 10 500 bash tools/ab.sh step 3 flexq_amd/libflexq_hip.so tools/libflexq_hip_head.so > gpurun_out/r05_ahead_ab.txt 2>&1
cat gpurun_out/r05_ahead_ab.txt
