# round-6: XS = 1 for one-item 16-row decode plans -- parity of the decode paths, then the C3 step A/B
# (ablation library: FQ_DEV_XS=0 forces the staged plan, unset = the new rule)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_dispatch_sweep.py tests/test_gpu_kernels.py tests/test_gpu_wrapper.py -x -q --timeout 200 --timeout-method thread > gpurun_out/xs_tests.log 2>&1 || { tail -30 gpurun_out/xs_tests.log; exit 1; }
tail -1 gpurun_out/xs_tests.log
B="python3 -u bench.py --cpu-budget 0 --no-fp16-compare --no-calibrate --no-layers --no-extra-configs --config llama2-7b-m16"
J='import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["ms_per_step"], d["roofline"]["per_launch_us"] if "per_launch_us" in d["roofline"] else "")'
for rep in 1 2 3; do
  for x in 0 new; do
    printf "FQ_DEV_XS=%s " $x
    if [ $x = new ]; then FLEXQ_AMD_LIB=abtmp/libflexq_hip_abl.so timeout -k 10 300 $B 2>/dev/null | python3 -c "$J" || exit 1
    else FQ_DEV_XS=0 FLEXQ_AMD_LIB=abtmp/libflexq_hip_abl.so timeout -k 10 300 $B 2>/dev/null | python3 -c "$J" || exit 1; fi
  done
done | tee gpurun_out/r06_m16_xs_step_ab.txt
