#!/bin/bash
# Round-2 GPU session: parity suite, smoke, C4 bench line, rocprofv3 trace + PMC passes of the
# C4 bench, FETCH_SIZE calibration.  Outputs under gpurun_out/.
export FM3D_LM_MAX_SECONDS=${FM3D_LM_MAX_SECONDS:-60}
export FM3D_PMC="FETCH_SIZE \
WRITE_SIZE,TCC_HIT_sum,TCC_MISS_sum \
SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_INSTS_VALU,SQ_INSTS_SALU \
SQ_INSTS_LDS,SQ_ACTIVE_INST_LDS,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_LDS_ADDR_CONFLICT,SQ_LDS_UNALIGNED_STALL,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR"
STEPS=()
[ -z "$NO_TESTS" ] && STEPS+=("timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 900 --timeout-method thread -s")
[ -z "$NO_TESTS" ] && STEPS+=("timeout -k 10 200 python -u -c 'import __graft_entry__ as g; g.smoke()'")
STEPS+=("timeout -k 10 400 python -u bench.py --out gpurun_out/bench_c4.json")
[ -n "$PROF" ] && STEPS+=("tools/prof_lm.sh c4 --steps 2 --warmup 1 --no-cpu")
[ -n "$CALIB" ] && STEPS+=("tools/calib_session.sh")
tools/gpu_session.sh "${STEPS[@]}"
