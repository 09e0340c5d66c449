# round-5: the chain's next linear's first ring blocks from the current linear's last refills
# (FQ_CHAIN_XREFILL) -- chain + layer tests, the headline step and the decoder layers against HEAD, stamps
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_layers.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_xref_tests.log 2>&1 || { tail -30 gpurun_out/r05_xref_tests.log; exit 1; }
tail -1 gpurun_out/r05_xref_tests.log
timeout -k 10 700 bash tools/ab.sh step 3 flexq_amd/libflexq_hip.so tools/libflexq_hip_head.so > gpurun_out/r05_xref_ab.txt 2>&1
cat gpurun_out/r05_xref_ab.txt
timeout -k 10 200 python3 tools/chain_stamps.py 2>&1 | tail -4 > gpurun_out/r05_xref_stamps.txt
cat gpurun_out/r05_xref_stamps.txt
