# scratch GPU job (development; rewritten per gpurun call)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "quantized_output" > gpurun_out/q3_tests.txt 2>&1 || { tail -40 gpurun_out/q3_tests.txt; exit 1; }
tail -1 gpurun_out/q3_tests.txt
for rep in 1 2; do
timeout -k 10 300 python -u bench.py --config llama2-7b-m1 --no-layers --no-reference-sweep --no-fp16-compare --cpu-budget 0 --no-calibrate --no-chain 2> gpurun_out/q3.err | tail -1 > gpurun_out/q3.json || { tail -30 gpurun_out/q3.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/q3.json').read());x=d['c5_llama3_8b_prefill'];e=x.get('epilogue_quantize');print(x['ms_per_step'], e['ms_per_step'], e['separate_quantize_ms_per_step'], e['last_output_identical'])"
done
