# scratch GPU job (development; rewritten per gpurun call)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_chain.py tests/test_gpu_layers.py -k "chain" > gpurun_out/j19_tests.txt 2>&1 || { tail -30 gpurun_out/j19_tests.txt; exit 1; }
tail -3 gpurun_out/j19_tests.txt
for rep in 1 2; do for L in flexq_amd/libflexq_hip.so tools/libflexq_hip_c091.so; do
  echo "== $L"; OLD=; [ "$L" = tools/libflexq_hip_c091.so ] && OLD=1; FQ_CHAIN_OLDABI=$OLD FLEXQ_AMD_LIB=$L timeout -k 10 200 python -u tools/chain_bench.py 20 2>&1 | grep -v amdgpu.ids || exit 1
done; done > gpurun_out/j19_ab.txt 2>&1
cat gpurun_out/j19_ab.txt
