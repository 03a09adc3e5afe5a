#!/bin/bash
# rocprofv3 kernel trace + one --pmc pass per counter group over the C4 bench (run through gpurun):
# tools/prof_session.sh TAG  ->  gpurun_out/prof_TAG/
export FM3D_LM_MAX_SECONDS=40
export FM3D_PMC="FETCH_SIZE WRITE_SIZE,TCC_HIT_sum,TCC_MISS_sum SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_INSTS_VALU,SQ_INSTS_SALU SQ_INSTS_LDS,SQ_ACTIVE_INST_LDS,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_LDS_ADDR_CONFLICT,SQ_LDS_UNALIGNED_STALL,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR"
tools/prof_lm.sh ${1:-c4} --steps 2 --warmup 1 --no-cpu
