# round-6 check after the decode epilogue quantizer: the full GPU suite, smoke, the default bench line, the 2-rank rehearsal
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/gpu_round_check.sh r06b || { tail -30 gpurun_out/r06b_tests.log; tail -20 gpurun_out/r06b_bench.err; exit 1; }
tail -1 gpurun_out/r06b_tests.log; tail -1 gpurun_out/r06b_smoke.log
