# Launch-overhead sensitivity to HIP runtime knobs (development): the empty-kernel graph floor and
# the decode shape sweep under each setting.
set -e
S="4096 4096 12288 4096"
for kv in "" "HIP_FORCE_DEV_KERNARG=1" "HIP_FORCE_DEV_KERNARG=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1"; do
  echo "== env: ${kv:-default}"
  env $kv timeout -k 10 60 ./tools/ubench_chain | grep -E "^empty   us|^touch|MB=  14.0 U=2"
  env $kv timeout -k 10 120 python3 -u tools/shape_sweep.py 1 $S | grep linear
done
