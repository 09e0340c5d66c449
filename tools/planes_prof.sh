# rocprofv3 kernel-trace summary of the bit-plane activation paths at M = 1 (tools/planes_bench.py)
set -o pipefail
mkdir -p gpurun_out/planes_prof
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
PB_M=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/planes_prof -o run -- python3 tools/planes_bench.py > gpurun_out/planes_prof/bench.txt 2>&1
