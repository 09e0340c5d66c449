# round-5: decode-kernel timelines (development build's per-WG stamps) at M = 16 against M = 1
set -o pipefail
cd $GRAFT_REPO_ROOT
for m in 1 16; do
  FQ_STAMP_M=$m FQ_STAMP_SHAPES="4096 4096 12288 4096 22016 4096 4096 11008" timeout -k 10 200 python3 -u tools/stamps.py 2>&1 | grep -E "^(gemm|linear)"
done > gpurun_out/r05_stamps_m16.txt
cat gpurun_out/r05_stamps_m16.txt
