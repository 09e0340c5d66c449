# round-6 development: rows-in-slots (XS = 1) vs staged at M = 8 and 12, one-item shapes
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for M in 8 12; do for x in 0 1 0 1; do
  echo "== M=$M FQ_DEV_XS=$x"
  FQ_DEV_XS=$x FQ_LIB=abtmp/libflexq_hip_abl.so FQ_SWEEP=gemm timeout -k 10 120 python3 -u tools/shape_sweep.py $M 4096 4096 4096 11008 2048 8192 2>&1 | grep us/launch || exit 1
done; done | tee gpurun_out/r06_m8_xs_ab.txt
