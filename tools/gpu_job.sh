# scratch GPU job (development; rewritten per gpurun call)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/j4_tests.log 2>&1 || { tail -30 gpurun_out/j4_tests.log; exit 1; }
tail -2 gpurun_out/j4_tests.log
timeout -k 10 600 tools/ab.sh step 3 flexq_amd/libflexq_hip.so tools/libflexq_hip_qf32.so > gpurun_out/j4_step.txt 2>&1 || exit 1
cat gpurun_out/j4_step.txt
timeout -k 10 600 tools/ab.sh m16 2 flexq_amd/libflexq_hip.so tools/libflexq_hip_qf32.so > gpurun_out/j4_m16.txt 2>&1 || exit 1
cat gpurun_out/j4_m16.txt
timeout -k 10 200 python -u tools/ablate.py 0,2048 linear > gpurun_out/j4_abl.txt 2>&1 || exit 1
cat gpurun_out/j4_abl.txt
