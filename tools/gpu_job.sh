# scratch GPU job (development; rewritten per gpurun call)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/chain_stress.py 120 50 2>&1 | grep -v amdgpu.ids | tee gpurun_out/f3_soak.txt
