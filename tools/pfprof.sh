# PMC passes over one prefill GEMM shape (development; tools/prefill_one.py)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P="python3 tools/prefill_one.py 16384 4096 4096 3"
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES -f csv -d gpurun_out/pf1 -o p -- $P > gpurun_out/pf1.log 2>&1 &&
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -f csv -d gpurun_out/pf2 -o p -- $P > gpurun_out/pf2.log 2>&1 &&
timeout -k 10 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_VALU_MFMA_COEXEC_CYCLES -f csv -d gpurun_out/pf3 -o p -- $P > gpurun_out/pf3.log 2>&1 &&
timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_LDS_UNALIGNED_STALL TA_BUSY_avr TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum -f csv -d gpurun_out/pf4 -o p -- $P > gpurun_out/pf4.log 2>&1
