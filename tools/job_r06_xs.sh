# round-6 development: batch-16 decode GEMM with the activation rows in the ring slots (XS = 1) instead of
# staged up front (XS = 0), graph-timed per LLaMA-2-7B shape, alternated
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for x in 0 1 0 1; do
  echo "== FQ_DEV_XS=$x"
  FQ_DEV_XS=$x FQ_LIB=abtmp/libflexq_hip_abl.so FQ_SWEEP=gemm timeout -k 10 120 python3 -u tools/shape_sweep.py 16 4096 4096 12288 4096 22016 4096 4096 11008 2>&1 | grep us/launch || exit 1
done | tee gpurun_out/r06_m16_xs_ab.txt
