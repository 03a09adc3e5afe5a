#!/bin/bash
# Round-5 C4 LM counters (one gpurun call): rocprofv3 kernel trace + one --pmc pass per counter group
# (tools/prof_lm.sh) of one resident C4 launch at a time, in the default (sequential) mode and in the
# tree mode (FM3D_LM_TREE=1), summarised to gpurun_out/r05_pmc_c4_{seq,tree}.json.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export FM3D_LM_MAX_SECONDS=40
ALL="FETCH_SIZE WRITE_SIZE,TCC_HIT_sum,TCC_MISS_sum SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_INSTS_VALU,SQ_INSTS_SALU SQ_INSTS_LDS,SQ_ACTIVE_INST_LDS,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_LDS_ADDR_CONFLICT,SQ_LDS_UNALIGNED_STALL,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR"
for mode in seq tree; do
  if [ $mode = tree ]; then export FM3D_LM_TREE=1; else unset FM3D_LM_TREE; fi
  FM3D_PMC="$ALL" tools/prof_lm.sh r05fres_$mode --mode resident --steps 2 --warmup 1 --no-cpu || exit 1
  python tools/pmc_summary.py gpurun_out/prof_r05fres_$mode lm2_kernel --workload 100000,64,3 --command "tools/r05_prof_c4.sh -> tools/prof_lm.sh r05fres_$mode (bench.py --mode resident --steps 2 --warmup 1 --no-cpu$( [ $mode = tree ] && echo ', FM3D_LM_TREE=1')), one rocprofv3 --pmc pass per counter group" --out gpurun_out/r05_pmc_c4_$mode.json > /dev/null || exit 1
done
