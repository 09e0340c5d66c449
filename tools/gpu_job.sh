# scratch GPU job (development; rewritten per gpurun call)
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do for L in flexq_amd/libflexq_hip.so tools/libflexq_hip_d6.so tools/libflexq_hip_d8.so; do
  echo "== $L"; FLEXQ_AMD_LIB=$L timeout -k 10 200 python -u tools/chain_bench.py 20 2>&1 | grep -v amdgpu.ids || exit 1
done; done > gpurun_out/j8_depth.txt 2>&1
cat gpurun_out/j8_depth.txt
