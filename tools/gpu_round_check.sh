# Round-end style GPU check: the full -m gpu suite, smoke(), the default bench (line + detail file) and
# the 2-rank shared-GPU rehearsal of the multi-rank bench path.  usage: bash tools/gpu_round_check.sh rNN
set -o pipefail
R=${1:-r05}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${R}_tests.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${R}_smoke.log 2>&1 && \
timeout -k 10 700 python bench.py --detail-out gpurun_out/${R}_bench_detail.json > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err && \
timeout -k 10 600 python bench.py --gpus 2 --share-gpu --steps 3 --warmup 1 --cpu-budget 0 --no-fp16-compare \
    --detail-out gpurun_out/${R}_share2_detail.json > gpurun_out/${R}_share2.json 2> gpurun_out/${R}_share2.err
