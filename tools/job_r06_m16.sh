# round-6 development: the batch-16 GEMM's slower loop -- ring depth 3 (FQ_RING_BUDGET=9216) and the M = 1
# LDS access pattern for the activation rows (FQ_DEV_ABLATION=4096, timing only)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
AB_TESTS="tests/test_gpu_dispatch_sweep.py" AB_OUT=gpurun_out/r06_m16_ring_ab.txt timeout -k 10 700 bash tools/ab.sh m16 3 flexq_amd/libflexq_hip.so abtmp/libflexq_hip_ring3.so || exit 1
for a in 0 4096 0 4096; do
  echo "== FQ_DEV_ABLATION=$a"
  FQ_DEV_ABLATION=$a FQ_LIB=abtmp/libflexq_hip_abl.so FQ_SWEEP=gemm timeout -k 10 120 python3 -u tools/shape_sweep.py 16 4096 4096 12288 4096 22016 4096 2>&1 | grep us/launch || exit 1
done > gpurun_out/r06_m16_lds_abl.txt
cat gpurun_out/r06_m16_lds_abl.txt
# run-to-run spread of the 32-layer decoder step (r05 1.295 / 1.320 ms at M = 1, r06 final 1.346)
AB_OUT=gpurun_out/r06_e2e_spread.txt timeout -k 10 700 bash tools/ab.sh e2e 3 flexq_amd/libflexq_hip.so || exit 1
