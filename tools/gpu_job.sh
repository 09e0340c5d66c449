# scratch GPU job (development; rewritten per gpurun call)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py -x -q --timeout 120 --timeout-method thread > gpurun_out/j13_chain.log 2>&1 || { tail -40 gpurun_out/j13_chain.log; exit 1; }
tail -2 gpurun_out/j13_chain.log
timeout -k 10 200 python -u tools/chain_stamps.py > gpurun_out/j13_cstamps.txt 2>&1 || { tail -20 gpurun_out/j13_cstamps.txt; exit 1; }
cat gpurun_out/j13_cstamps.txt
timeout -k 10 300 python -u tools/chain_bench.py 20 > gpurun_out/j13_chainbench.txt 2>&1 || { tail -20 gpurun_out/j13_chainbench.txt; exit 1; }
cat gpurun_out/j13_chainbench.txt
