#!/bin/bash
# A/B of prefill GEMM builds in one run (development): tools/prefill_bench.py per library, twice.
for rep in 1 2; do
  for L in "$@"; do
    echo "== $L"; FQ_REPS=${FQ_REPS:-6} FQ_LIB=$L timeout -k 10 200 python3 tools/prefill_bench.py ${PF_M:-16384} 2>&1 | grep -E "^M=" | sed -E 's/\| linear.*//' || exit 1
  done
done
