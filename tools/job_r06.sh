# round-6 development job: chain stamps on the current chain, graph-timed prefill GEMMs per C5 shape
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 150 python3 -u tools/chain_stamps.py > gpurun_out/r06_chain_stamps.txt 2>&1 || { tail -20 gpurun_out/r06_chain_stamps.txt; exit 1; }
cat gpurun_out/r06_chain_stamps.txt
FQ_REPS=6 timeout -k 10 300 python3 -u tools/prefill_bench.py 16384 > gpurun_out/r06_prefill_bench.txt 2>&1 || { tail -20 gpurun_out/r06_prefill_bench.txt; exit 1; }
cat gpurun_out/r06_prefill_bench.txt
