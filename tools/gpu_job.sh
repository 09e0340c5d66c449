# scratch GPU job (development; rewritten per gpurun call)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/f5_tests.txt 2>&1 || { tail -30 gpurun_out/f5_tests.txt; exit 1; }
tail -1 gpurun_out/f5_tests.txt
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/f5_smoke.txt 2>&1 || { tail -20 gpurun_out/f5_smoke.txt; exit 1; }
tail -1 gpurun_out/f5_smoke.txt
