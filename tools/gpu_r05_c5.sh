# round-5: C5 after the prefill VALU cut (bench line + PMC passes on the gate_up shape) and the M = 16
# decode breakdown (GEMM alone / linear / quantizer against M = 1)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --config llama3-8b-prefill --steps 3 --warmup 1 --cpu-budget 0 --no-fp16-compare \
    --no-layers --no-reference-sweep --detail-out gpurun_out/r05_c5_detail.json > gpurun_out/r05_c5_bench.json 2> gpurun_out/r05_c5_bench.err
tail -c 1500 gpurun_out/r05_c5_bench.json
rm -rf gpurun_out/pf0 gpurun_out/pf1 gpurun_out/pf2 gpurun_out/pf3 gpurun_out/pf4 gpurun_out/pf5
PF_SHAPE="16384 28672 4096" bash tools/pfprof.sh
for i in 0 5 1 2 3 4; do python3 tools/pmc_avg.py gpurun_out/pf$i fq_gemm_prefill; done > gpurun_out/r05_prefill_pmc_after.txt
grep "TOPS" gpurun_out/pf1.log | tail -1 >> gpurun_out/r05_prefill_pmc_after.txt
cat gpurun_out/r05_prefill_pmc_after.txt
for spec in "1 gemm" "16 gemm" "16 linear" "16 quant" "1 linear"; do
  set -- $spec
  echo "== M=$1 $2"
  FQ_SWEEP=$2 timeout -k 10 150 python3 -u tools/shape_sweep.py $1 4096 4096 12288 4096 22016 4096 4096 11008 2>&1 | grep "us/launch"
done > gpurun_out/r05_m16_sweep.txt 2>&1
cat gpurun_out/r05_m16_sweep.txt
