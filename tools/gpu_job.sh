# scratch GPU job (development; rewritten per gpurun call)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/chain_bench.py 20 > gpurun_out/j7_chainbench.txt 2>&1 || { tail -20 gpurun_out/j7_chainbench.txt; exit 1; }
cat gpurun_out/j7_chainbench.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py -x -q --timeout 120 --timeout-method thread > gpurun_out/j7_chain.log 2>&1 || { tail -40 gpurun_out/j7_chain.log; exit 1; }
tail -2 gpurun_out/j7_chain.log
timeout -k 10 300 python -u bench.py --cpu-budget 0 --no-fp16-compare --no-calibrate --no-extra-configs --no-layers --no-reference-sweep > gpurun_out/j7_bench.json 2> gpurun_out/j7_bench.err || { tail -20 gpurun_out/j7_bench.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/j7_bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'ms', d['ms_per_step'], 'frac', d['roofline']['frac'], d['config']['decode_form']); print(d.get('decode_chain'))"
