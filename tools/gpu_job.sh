# scratch GPU job (development; rewritten per gpurun call)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u bench.py --gpus 2 --share-gpu --steps 3 --warmup 1 --no-layers --no-reference-sweep > gpurun_out/j11_share2.json 2> gpurun_out/j11_share2.err || { tail -30 gpurun_out/j11_share2.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/j11_share2.json').read().strip().splitlines()[-1])
print('value', d['value'], 'ms', d['ms_per_step'], d['config']['workload'][:80], d.get('rehearsal'))
print({k: (v if not isinstance(v, dict) else {kk: v.get(kk) for kk in ('ms_per_step','value','error','skipped','gather','bit_identical_to_rccl')}) for k, v in d.items() if k in ('tp','tp_peer_gather','tp_llama2_7b','tp_llama2_7b_peer_gather','replicas')})
"
