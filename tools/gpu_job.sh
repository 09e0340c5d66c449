# scratch GPU job (development; rewritten per gpurun call)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1100 bash tools/profile_round.sh r04 > gpurun_out/j10_prof.log 2>&1 || { tail -30 gpurun_out/j10_prof.log; exit 1; }
tail -5 gpurun_out/j10_prof.log
ls gpurun_out/profiles/
