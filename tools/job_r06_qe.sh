# round-6 development: the decode epilogue quantizer (fq_gemm_w6ax_q) -- the C3 A/B, graph and eager
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/c3_qe_ab.py 3 16 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r06_c3_qe_ab.txt
