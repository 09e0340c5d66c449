#!/bin/bash
# Prefill GEMM at 2048 <= M < 16384: the 256 x 256 kernel (product) vs the 128 x 128 kernel over
# the same unpacked weights (development switch FQ_DEV_PF128), graph-free timing (development).
for m in ${PF_MS:-2048 3072 4096 8192}; do
  echo "== M=$m big"; FQ_REPS=20 timeout -k 10 120 python3 tools/prefill_bench.py $m 2>&1 | grep "^M=" | sed -E "s/\| fp16.*//" || exit 1
  echo "== M=$m 128"; FQ_DEV_PF128=1 FQ_LIB=tools/libflexq_hip_abl.so FQ_REPS=20 timeout -k 10 120 python3 tools/prefill_bench.py $m 2>&1 | grep "^M=" | sed -E "s/\| fp16.*//" || exit 1
done
