#!/bin/bash
# Forced split-K sweep of the 128 x 128 prefill kernel at 32 < M < 2048 (development; calibrates
# prefill_split's cost model in fq_gemm.hip): per M, the planner's choice (product library) and
# every forced S (ablation library, FQ_DEV_PS), graph-timed per launch by tools/shape_sweep.py.
SHAPES="4096 4096 12288 4096 22016 4096 4096 11008"
for M in ${PSPLIT_M:-33 64 128 256 512 1024}; do
  echo "== M=$M planner"; FQ_SWEEP=gemm timeout -k 10 60 python3 tools/shape_sweep.py $M $SHAPES 2>&1 | grep "us/launch" || exit 1
  for S in 1 2 4 8 16; do
    echo "== M=$M S=$S"; FQ_DEV_PS=$S FQ_LIB=abtmp/libflexq_hip_abl.so FQ_SWEEP=gemm timeout -k 10 60 python3 tools/shape_sweep.py $M $SHAPES 2>&1 | grep "us/launch" || exit 1
  done
done
