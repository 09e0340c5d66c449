# round-5: decode GEMM counters at M = 16 against M = 1 (pre-quantized codes, 4096 x 4096 and 12288 x 4096)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
set -o pipefail
for m in 1 16; do
  FQ_SWEEP=gemm timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU --kernel-include-regex fq_gemm_decode -f csv -d gpurun_out/p16_$m -o p -- python3 tools/shape_sweep.py $m 4096 4096 12288 4096 > gpurun_out/p16_$m.log 2>&1 || exit 1
  python3 tools/pmc_avg.py gpurun_out/p16_$m fq_gemm_decode
done > gpurun_out/r05_pmc_m16.txt
cat gpurun_out/r05_pmc_m16.txt
