#!/bin/bash
# A/B of decode builds (development): the fused M = 1 linear on the LLaMA-2-7B launch shapes,
# graph-timed per launch by tools/shape_sweep.py, libraries alternated three times.
for rep in 1 2 3; do
  for L in "$@"; do
    FQ_LIB=$L timeout -k 10 120 python3 tools/shape_sweep.py 1 12288 4096 4096 4096 22016 4096 4096 11008 2>&1 | grep "us/launch" || exit 1
  done
done
