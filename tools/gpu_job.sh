# scratch GPU job (development; rewritten per gpurun call)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/chain_stamps.py > gpurun_out/j25_plain.txt 2>&1 || { tail -20 gpurun_out/j25_plain.txt; exit 1; }
FQ_STAMPS_PRO=1 timeout -k 10 120 python -u tools/chain_stamps.py > gpurun_out/j25_pro.txt 2>&1 || { tail -20 gpurun_out/j25_pro.txt; exit 1; }
cat gpurun_out/j25_plain.txt gpurun_out/j25_pro.txt | grep -v amdgpu.ids
