# round-5: the 256 x 256 prefill dequant with biased accumulators and two v_pk_add_f32 per block instead of four v_cvt_f32_i32 (8 VALU per block instead of 10); bit-identity first
set -o pipefail
cd $GRAFT_REPO_ROOT
for L in flexq_amd/libflexq_hip.so tools/libflexq_hip_pksub.so; do
  FQ_LIB=$L timeout -k 10 100 python3 -u tools/prefill_hash.py 2>&1 | grep sha || exit 1
done > gpurun_out/r05_pksub_ab.txt
for rep in 1 2 3; do
  for L in flexq_amd/libflexq_hip.so tools/libflexq_hip_pksub.so; do
    echo "lib $L"
    FQ_LIB=$L FQ_REPS=6 timeout -k 10 150 python3 -u tools/prefill_bench.py 16384 2>&1 | grep -v amdgpu.ids || exit 1
  done
done >> gpurun_out/r05_pksub_ab.txt
cat gpurun_out/r05_pksub_ab.txt
