#!/bin/bash
# Round-end measurement on one GPU box (run through gpurun): GPU parity suite, smoke(),
# the default bench line (with the CPU baseline), then the rocprofv3 kernel trace and one
# --pmc pass per counter group (tools/prof_lm.sh).  Outputs under gpurun_out/.
export FM3D_LM_MAX_SECONDS=${FM3D_LM_MAX_SECONDS:-40}
export FM3D_PMC="FETCH_SIZE \
WRITE_SIZE,TCC_HIT_sum,TCC_MISS_sum \
SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_INSTS_VALU,SQ_INSTS_SALU \
SQ_INSTS_LDS,SQ_ACTIVE_INST_LDS,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_LDS_ADDR_CONFLICT,SQ_LDS_UNALIGNED_STALL,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR"
tools/gpu_session.sh \
  "timeout -k 10 300 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread" \
  "timeout -k 10 200 python -u -c 'import __graft_entry__ as g; g.smoke()'" \
  "timeout -k 10 400 python -u bench.py --out gpurun_out/bench_final.json" \
  "tools/prof_lm.sh final --steps 2 --warmup 1 --no-cpu"
