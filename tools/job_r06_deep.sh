# round-6 development: the plain chain's deep first pass (FQ_CHAIN_DEEP = 3 / 6 extra ring blocks per wave,
# issued behind the input poll) against the current chain -- chain tests on every library, then the step
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
AB_OUT=gpurun_out/r06_chain_deep_ab.txt timeout -k 10 900 bash tools/ab.sh step 3 flexq_amd/libflexq_hip.so abtmp/libflexq_hip_deep3.so
