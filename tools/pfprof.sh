# PMC passes over one prefill GEMM shape (development; tools/prefill_one.py), one rocprofv3 run per
# counter set: HBM traffic (FETCH_SIZE, WRITE_SIZE: the gfx950 x2 correction is applied when read),
# SQ issue / wait breakdown, instruction mix, L2 hit rate and TA busy.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P="python3 tools/prefill_one.py ${PF_SHAPE:-16384 4096 4096} 3"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d gpurun_out/pf0 -o p -- $P > gpurun_out/pf0.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -f csv -d gpurun_out/pf5 -o p -- $P > gpurun_out/pf5.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES -f csv -d gpurun_out/pf1 -o p -- $P > gpurun_out/pf1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -f csv -d gpurun_out/pf2 -o p -- $P > gpurun_out/pf2.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_VALU_MFMA_COEXEC_CYCLES -f csv -d gpurun_out/pf3 -o p -- $P > gpurun_out/pf3.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE TA_BUSY_avr TCC_HIT_sum TCC_MISS_sum -f csv -d gpurun_out/pf4 -o p -- $P > gpurun_out/pf4.log 2>&1
