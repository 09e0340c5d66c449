# round-5: the XS = 1 decode variant (activation rows per ring slot) before / after the buffer-addressed DMAs
set -o pipefail
cd $GRAFT_REPO_ROOT
for rep in 1 2 3; do
  for L in flexq_amd/libflexq_hip.so tools/libflexq_hip_pre.so; do
    for m in 16 32; do
      FQ_LIB=$L FQ_SWEEP=gemm timeout -k 10 150 python3 -u tools/shape_sweep.py $m 4096 11008 8192 28672 12288 4096 2>&1 | grep "us/launch"
    done
  done
done > gpurun_out/r05_xs_ab.txt 2>&1
cat gpurun_out/r05_xs_ab.txt
