# scratch GPU job (development; rewritten per gpurun call)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/j14_tests.log 2>&1 || { tail -30 gpurun_out/j14_tests.log; exit 1; }
tail -2 gpurun_out/j14_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/j14_smoke.log 2>&1 || { tail -20 gpurun_out/j14_smoke.log; exit 1; }
tail -1 gpurun_out/j14_smoke.log
timeout -k 10 800 python -u bench.py > gpurun_out/j14_bench.json 2> gpurun_out/j14_bench.err || { tail -20 gpurun_out/j14_bench.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/j14_bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'ms', d['ms_per_step'], 'frac', d['roofline']['frac'], d['config']['decode_form'])
print('chain', {k: d['decode_chain'][k] for k in ('ms_per_step','launches_ms_per_step','bit_identical_to_launches')})
for k in ('c3_llama2_7b_m16','c5_llama3_8b_prefill','c4_llama2_70b_1gpu'): print(k, d.get(k,{}).get('ms_per_step'))
e=d.get('decoder_layers_e2e',{}); print('e2e', {m: (e.get(m) or {}).get('w6_ms_per_step') for m in ('M1','M16')})
"
