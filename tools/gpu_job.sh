# scratch GPU job (development; rewritten per gpurun call)
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2 3; do for L in flexq_amd/libflexq_hip.so tools/libflexq_hip_sl0.so; do
  echo "== $L"; FLEXQ_AMD_LIB=$L timeout -k 10 200 python -u tools/chain_bench.py 20 2>&1 | grep -v amdgpu.ids | grep -v "^launches" || exit 1
done; done
