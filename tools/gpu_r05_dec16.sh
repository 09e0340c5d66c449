# round-5: unfused decode (M > 4) DMAs all buffer-addressed, division-free staging and reduction
# indices -- GPU tests, then the batch-16 step and per-shape GEMMs against HEAD's library
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05_dec16_tests.log 2>&1 || { tail -30 gpurun_out/r05_dec16_tests.log; exit 1; }
tail -1 gpurun_out/r05_dec16_tests.log
timeout -k 10 500 bash tools/ab.sh m16 3 flexq_amd/libflexq_hip.so tools/libflexq_hip_head.so > gpurun_out/r05_dec16_ab.txt 2>&1
for L in flexq_amd/libflexq_hip.so tools/libflexq_hip_head.so; do
  for m in 8 16 32; do
    echo "== $L M=$m gemm"
    FQ_LIB=$L FQ_SWEEP=gemm timeout -k 10 150 python3 -u tools/shape_sweep.py $m 4096 4096 12288 4096 22016 4096 4096 11008 2>&1 | grep "us/launch"
  done
done >> gpurun_out/r05_dec16_ab.txt 2>&1
cat gpurun_out/r05_dec16_ab.txt
