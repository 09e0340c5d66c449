#!/bin/bash
# A/B of library builds in one run (development): every build timed REPS times, alternating, so
# clock and box drift hit every arm alike.  Replaces the per-experiment ab_*.sh stubs.
#
#   tools/ab.sh MODE REPS LIB [LIB ...]
#
# MODE
#   step     the headline bench step (LLaMA-2-7B, M = 1): ms/step and per-launch us
#   m16      the batch-16 step (--config llama2-7b-m16): ms/step
#   e2e      the 32-layer decoder step at M = 1 and 16 (bench decoder_layers_e2e)
#   shapes   graph-timed decode launches (tools/shape_sweep.py; SHAPES="N K ...", M=..., FQ_SWEEP=...)
#   prefill  prefill GEMMs (tools/prefill_bench.py at PF_M, default 16384)
# Libraries are selected with FLEXQ_AMD_LIB / FQ_LIB (flexq_amd/_lib.py); build variants with
#   make -C flexq_amd/csrc variant NAME=x DEFS="-DFOO=1"   ->  abtmp/libflexq_hip_x.so
# (abtmp/ is git-ignored; clear it after the experiment so later pushes do not carry the libraries)
# AB_TESTS="tests/test_gpu_chain.py ..."  runs those GPU tests against EVERY library first and stops on a
#   failure (an A/B of a variant that is not bit-identical is not an A/B); AB_TESTS_K="expr" selects with
#   pytest -k (leave out tests of the behaviour the variant changes); AB_OUT=file tees the table.
# AB_ENVS="FQ_DEV_XS=0 FQ_DEV_XS=1" makes each environment setting an arm of its own with every library
#   (development switches read at run time, e.g. the ablation library's FQ_DEV_*; "-" = no setting;
#   comma-separate several variables of one arm).
# One gpurun call per experiment:  AB_TESTS=... bash tools/ab.sh step 3 flexq_amd/libflexq_hip.so abtmp/x.so
set -o pipefail
MODE=$1; REPS=$2; shift 2
[ -n "$MODE" ] && [ -n "$REPS" ] && [ $# -ge 1 ] || { sed -n 2,20p "$0"; exit 2; }
mkdir -p gpurun_out
if [ -n "$AB_TESTS" ]; then
  for L in "$@"; do
    FLEXQ_AMD_LIB=$L timeout -k 10 600 python3 -u -m pytest $AB_TESTS ${AB_TESTS_K:+-k "$AB_TESTS_K"} -x -q --timeout 200 --timeout-method thread \
      > gpurun_out/ab_tests.log 2>&1 || { echo "tests failed with $L"; tail -30 gpurun_out/ab_tests.log; exit 1; }
    echo "$L: $(tail -1 gpurun_out/ab_tests.log)"
  done
fi
[ -n "$AB_OUT" ] && exec > >(tee "$AB_OUT")
B="python3 -u bench.py --cpu-budget 0 --no-fp16-compare --no-calibrate"
J='import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1])'
for rep in $(seq "$REPS"); do
  for L in "$@"; do for E in ${AB_ENVS:--}; do
    printf "%s " "$L"; [ "$E" != - ] && printf "%s " "$E"
    ( [ "$E" != - ] && export ${E//,/ }
    case $MODE in
      step)    FLEXQ_AMD_LIB=$L timeout -k 10 200 $B --no-layers --no-extra-configs 2>/dev/null |
                 python3 -c "$J; print(d['ms_per_step'], d['roofline']['per_launch_us'])" || exit 1 ;;
      m16)     FLEXQ_AMD_LIB=$L timeout -k 10 300 $B --no-layers --no-extra-configs --config llama2-7b-m16 2>/dev/null |
                 python3 -c "$J; print(d['ms_per_step'], d['roofline']['per_launch_us'])" || exit 1 ;;
      e2e)     FLEXQ_AMD_LIB=$L timeout -k 10 300 $B --no-extra-configs --steps 5 --warmup 2 2>/dev/null |
                 python3 -c "$J; e=d['decoder_layers_e2e']; print(e['M1']['w6_ms_per_step'], e['M16']['w6_ms_per_step'])" || exit 1 ;;
      shapes)  echo; FQ_LIB=$L timeout -k 10 150 python3 -u tools/shape_sweep.py ${M:-1} ${SHAPES:-4096 4096 12288 4096 22016 4096 4096 11008} 2>&1 |
                 grep "us/launch" || exit 1 ;;
      prefill) echo; FQ_REPS=${FQ_REPS:-6} FQ_LIB=$L timeout -k 10 200 python3 tools/prefill_bench.py ${PF_M:-16384} 2>&1 |
                 grep -E "^M=" | sed -E 's/\| linear.*//' || exit 1 ;;
      *) echo "unknown mode $MODE"; exit 2 ;;
    esac ) || exit 1
  done; done
done
