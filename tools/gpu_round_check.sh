# Round-end style GPU check: new tests first, then the full -m gpu suite, smoke() and the default bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_planes.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t0_planes.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t1_tests.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/t1_smoke.log 2>&1 && \
timeout -k 10 400 python bench.py > gpurun_out/t1_bench.json 2> gpurun_out/t1_bench.err
