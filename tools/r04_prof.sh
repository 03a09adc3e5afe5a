#!/bin/bash
# Round-4 profiling on one GPU box (run through gpurun): rocprofv3 kernel trace + one --pmc pass per
# counter group over the C4 bench in resident mode (one frame pair per LM launch: the per-launch
# roofline and HBM traffic), kernel traces of the headline stream mode (two frame pairs per launch,
# launches overlapped) and of the C2 / C3 workloads.  Outputs under gpurun_out/prof_r04*.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export FM3D_LM_MAX_SECONDS=40
export FM3D_PMC="FETCH_SIZE WRITE_SIZE,TCC_HIT_sum,TCC_MISS_sum SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_INSTS_VALU,SQ_INSTS_SALU SQ_INSTS_LDS,SQ_ACTIVE_INST_LDS,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_LDS_ADDR_CONFLICT,SQ_LDS_UNALIGNED_STALL,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR"
cd "$R" && tools/prof_lm.sh r04res --mode resident --steps 2 --warmup 1 --no-cpu || exit 1
cd "$R" && python tools/pmc_summary.py gpurun_out/prof_r04res lm2_kernel --workload 100000,64,3 --command "tools/r04_prof.sh -> tools/prof_lm.sh r04res (bench.py --mode resident --steps 2 --warmup 1 --no-cpu), one rocprofv3 --pmc pass per counter group" --out gpurun_out/r04_pmc_c4.json > /dev/null || exit 1
export FM3D_PMC=""
cd "$R" && tools/prof_lm.sh r04stream --steps 6 --warmup 2 --no-cpu || exit 1
cd "$R" && tools/prof_lm.sh r04c2 --workload c2 --steps 100 --warmup 10 --no-cpu || exit 1
cd "$R" && tools/prof_lm.sh r04c3 --workload c3 --steps 20 --warmup 3 --no-cpu || exit 1
