# round-6 final check (after the decode epilogue quantizer and the rows-in-slots rule): the full GPU suite,
# smoke, the default bench line, the 2-rank rehearsal, then the committed profiles -- bash tools/job_r06c.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/gpu_round_check.sh r06c || { tail -30 gpurun_out/r06c_tests.log; tail -20 gpurun_out/r06c_bench.err; exit 1; }
tail -1 gpurun_out/r06c_tests.log; tail -1 gpurun_out/r06c_smoke.log
timeout -k 10 1500 bash tools/profile_round.sh r06c > gpurun_out/r06c_profile_round.log 2>&1 || { tail -30 gpurun_out/r06c_profile_round.log; exit 1; }
echo profiled
