# scratch GPU job (development; rewritten per gpurun call)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/f4_tests.txt 2>&1 || { tail -30 gpurun_out/f4_tests.txt; exit 1; }
tail -1 gpurun_out/f4_tests.txt
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/f4_smoke.txt 2>&1 || { tail -20 gpurun_out/f4_smoke.txt; exit 1; }
tail -1 gpurun_out/f4_smoke.txt
timeout -k 10 500 python -u bench.py > gpurun_out/f4_bench.json 2> gpurun_out/f4_bench.err || { tail -30 gpurun_out/f4_bench.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/f4_bench.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['decode_chain']['launches_ms_per_step']);x=d['c5_llama3_8b_prefill'];print('c3',d['c3_llama2_7b_m16']['ms_per_step'],'c5',x['ms_per_step'],x.get('epilogue_quantize'),'e2e',d['decoder_layers_e2e']['M1']['w6_ms_per_step'])"
