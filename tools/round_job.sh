# A round's GPU check in one gpurun call: the full -m gpu suite, smoke(), the default bench line (+ detail file),
# the 2-rank shared-GPU rehearsal (tools/gpu_round_check.sh), then -- unless NO_PROFILES=1 -- the committed
# profiles (tools/profile_round.sh: kernel traces, FETCH_SIZE passes, prefill PMC) into gpurun_out/profiles/.
#   gpurun -- 'bash tools/round_job.sh r06c'    (then copy gpurun_out/profiles/r06c_* and the bench files into profiles/)
set -o pipefail
R=${1:?usage: bash tools/round_job.sh rNN}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/gpu_round_check.sh $R || { tail -30 gpurun_out/${R}_tests.log; tail -20 gpurun_out/${R}_bench.err; exit 1; }
tail -1 gpurun_out/${R}_tests.log; tail -1 gpurun_out/${R}_smoke.log
[ "$NO_PROFILES" = 1 ] && exit 0
timeout -k 10 1500 bash tools/profile_round.sh $R > gpurun_out/${R}_profile_round.log 2>&1 || { tail -30 gpurun_out/${R}_profile_round.log; exit 1; }
echo profiled
