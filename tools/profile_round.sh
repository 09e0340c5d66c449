# Regenerates the committed profiles/ for the current code (run on the GPU box via gpurun).
# usage: bash tools/profile_round.sh rNN   (then: cp gpurun_out/profiles/rNN_* profiles/)
set -e
R=${1:-r01}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof gpurun_out/profiles
P=gpurun_out/profiles  # merged back by gpurun; copy into profiles/ afterwards
B="python3 bench.py --cpu-budget 0 --no-fp16-compare --no-layers --no-extra-configs --no-reference-sweep"
# 1. kernel trace + stats of the default bench (LLaMA-2-7B, M=1)
echo "[profile_round] 1. kernel trace + stats of the default bench (LLaMA-2-7B, " ; date
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof/kt -o run -- $B --steps 5 > gpurun_out/prof/kt.log 2>&1
cp gpurun_out/prof/kt/run_kernel_stats.csv $P/${R}_kernel_stats.csv
python3 tools/trace_summary.py gpurun_out/prof/kt/run_kernel_trace.csv > $P/${R}_kernel_trace_summary.txt
grep '"metric"' gpurun_out/prof/kt.log | tail -1 > $P/${R}_bench_under_rocprof.json
# 2. HBM traffic: FETCH_SIZE pass alone (no other counters), decode kernel only
echo "[profile_round] 2. HBM traffic: FETCH_SIZE pass alone (no other counters)," ; date
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --kernel-include-regex fq_gemm_decode -f csv -d gpurun_out/prof/pmc -o run -- $B --no-chain --steps 2 --warmup 1 --roofline-reps 1 > gpurun_out/prof/pmc.log 2>&1
cp gpurun_out/prof/pmc/run_counter_collection.csv $P/${R}_pmc_fetch_size.csv
python3 tools/pmc_summary.py $P/${R}_pmc_fetch_size.csv fq_gemm_decode llama2-7b-m1 $P/${R}_pmc_summary.json > /dev/null
python3 - "$R" <<'PY'
import json, sys
p = f"gpurun_out/profiles/{sys.argv[1]}_pmc_summary.json"
d = json.load(open(p))
d.update(launch_pattern="qkv, o, gate_up (merged), down per layer", merged_gate_up=True,
         command="rocprofv3 --pmc FETCH_SIZE --kernel-trace --kernel-include-regex fq_gemm_decode -f csv -- "
                 "python3 bench.py --cpu-budget 0 --no-fp16-compare --no-layers --no-extra-configs "
                 "--no-reference-sweep --no-chain --steps 2 --warmup 1 --roofline-reps 1",
         note="one launch per linear (--no-chain): the chain form's linears stream the same image bytes "
              "per linear, plus 4 B per output element of hand-off granules")
d["source"] = f"profiles/{sys.argv[1]}_pmc_fetch_size.csv"  # where it is committed
json.dump(d, open(p, "w"), indent=1)
PY
# 3. batch-16 config and the prefill GEMM (kernel stats)
echo "[profile_round] 3. batch-16 config and the prefill GEMM (kernel stats)" ; date
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof/m16 -o run -- $B --config llama2-7b-m16 --steps 5 > gpurun_out/prof/m16.log 2>&1
python3 tools/trace_summary.py gpurun_out/prof/m16/run_kernel_trace.csv > $P/${R}_m16_kernel_trace_summary.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof/pf -o run -- python3 tools/prefill_bench.py 16384 > gpurun_out/prof/pf.log 2>&1
python3 tools/trace_summary.py gpurun_out/prof/pf/run_kernel_trace.csv > $P/${R}_prefill_kernel_trace_summary.txt
cp gpurun_out/prof/pf.log $P/${R}_prefill_bench_under_rocprof.txt
# 4. C5 (LLaMA-3-8B W6A8 prefill, M = 16384) bench under the kernel trace
echo "[profile_round] 4. C5 (LLaMA-3-8B W6A8 prefill, M = 16384) bench under the" ; date
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof/c5 -o run -- $B --config llama3-8b-prefill --steps 2 --warmup 1 --no-calibrate > gpurun_out/prof/c5.log 2>&1
python3 tools/trace_summary.py gpurun_out/prof/c5/run_kernel_trace.csv > $P/${R}_c5_kernel_trace_summary.txt
grep '"metric"' gpurun_out/prof/c5.log | tail -1 > $P/${R}_c5_bench_under_rocprof.json
# 4b. C5 HBM traffic: FETCH_SIZE pass over the prefill GEMM launches of the C5 bench (roofline.traffic)
echo "[profile_round] 4b. C5 HBM traffic: FETCH_SIZE pass over the prefill GEMM " ; date
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --kernel-include-regex fq_gemm_prefill -f csv -d gpurun_out/prof/c5pmc -o run -- $B --config llama3-8b-prefill --steps 1 --warmup 1 --roofline-reps 1 --no-calibrate > gpurun_out/prof/c5pmc.log 2>&1
cp gpurun_out/prof/c5pmc/run_counter_collection.csv $P/${R}_c5_pmc_fetch_size.csv
python3 tools/pmc_summary.py $P/${R}_c5_pmc_fetch_size.csv fq_gemm_prefill llama3-8b-prefill $P/${R}_c5_pmc_summary.json > /dev/null
python3 - "$R" <<'PY'
import json, sys
p = f"gpurun_out/profiles/{sys.argv[1]}_c5_pmc_summary.json"
d = json.load(open(p))
d.update(merged_gate_up=True, launch_pattern="qkv, o, gate_up (merged), down per layer; the prefill GEMM launches only",
         command="rocprofv3 --pmc FETCH_SIZE --kernel-trace --kernel-include-regex fq_gemm_prefill -f csv -- "
                 "python3 bench.py --cpu-budget 0 --no-fp16-compare --no-layers --config llama3-8b-prefill "
                 "--steps 1 --warmup 1 --roofline-reps 1 --no-calibrate")
d["source"] = f"profiles/{sys.argv[1]}_c5_pmc_fetch_size.csv"
json.dump(d, open(p, "w"), indent=1)
PY
# 5. prefill PMC passes (one GEMM shape, the U8 big-tile kernel) and their per-dispatch averages
echo "[profile_round] 5. prefill PMC passes (one GEMM shape, the U8 big-tile ker" ; date
rm -rf gpurun_out/pf0 gpurun_out/pf1 gpurun_out/pf2 gpurun_out/pf3 gpurun_out/pf4 gpurun_out/pf5
PF_SHAPE="${PF_SHAPE:-16384 28672 4096}" bash tools/pfprof.sh
for i in 0 5 1 2 3 4; do python3 tools/pmc_avg.py gpurun_out/pf$i fq_gemm_prefill; done > $P/${R}_prefill_pmc.txt
grep "TOPS" gpurun_out/pf1.log | tail -1 >> $P/${R}_prefill_pmc.txt
python3 tools/pmc_summary.py gpurun_out/pf0/p_counter_collection.csv fq_gemm_prefill prefill-16384x4096x4096 $P/${R}_prefill_fetch_summary.json > /dev/null
echo profiles done
