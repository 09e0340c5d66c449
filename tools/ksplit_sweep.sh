# Development: decode launch time per forced k-split S (abtmp/libflexq_hip_abl.so, FQ_DEV_S) on the
# tensor-parallel shard shapes and the 70B qkv, M = 1 and M = 16.  usage: bash tools/ksplit_sweep.sh
export FQ_LIB=abtmp/libflexq_hip_abl.so
SH="10240 8192 5120 8192 1280 8192 1024 8192 2048 8192 1024 28672 2048 28672 14336 8192 2048 11008 1024 11008 512 11008 512 4096 1024 4096 1536 4096"
for M in 1 16; do
  for S in 1 2 3 4 6 8; do
    FQ_DEV_S=$S timeout -k 10 120 python3 tools/shape_sweep.py $M $SH > gpurun_out/ks_${M}_$S.log 2>&1 || exit 1
    sed "s/^/S=$S /" gpurun_out/ks_${M}_$S.log | grep us/launch
  done
done
