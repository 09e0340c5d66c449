# round-6 final check: the full GPU suite, smoke, the default bench line, the 2-rank rehearsal, then the
# committed profiles (kernel traces, FETCH_SIZE passes, prefill PMC) -- bash tools/job_r06.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/gpu_round_check.sh r06 || { tail -30 gpurun_out/r06_tests.log; tail -20 gpurun_out/r06_bench.err; exit 1; }
tail -1 gpurun_out/r06_tests.log; tail -1 gpurun_out/r06_smoke.log
timeout -k 10 1500 bash tools/profile_round.sh r06 > gpurun_out/r06_profile_round.log 2>&1 || { tail -30 gpurun_out/r06_profile_round.log; exit 1; }
echo profiled
