# scratch GPU job (development; rewritten per gpurun call)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py --gpus 2 --share-gpu --steps 3 --warmup 1 --cpu-budget 0 --no-fp16-compare --no-reference-sweep > gpurun_out/f2_share2.json 2> gpurun_out/f2_share2.err || { tail -30 gpurun_out/f2_share2.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/f2_share2.json').read().strip().splitlines()[-1]);print(d['value'],d['n_gpus'],d['ms_per_step'],d['config'].get('parallelism'),d.get('rehearsal'));print(list(d.keys()))"
