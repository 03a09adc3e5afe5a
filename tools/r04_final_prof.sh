#!/bin/bash
# Round-4 closing measurement, part 2 (one gpurun call): rocprofv3 kernel traces + PMC passes (one
# counter group per run, tools/prof_lm.sh) of
#   * the C4 LM launch one at a time (--mode resident: the per-launch roofline and HBM bytes),
#   * the streamed headline (4 pairs in flight, 2 per launch: launches overlapped),
#   * C3 (ncc_kernel) and C2 (kernel trace),
#   * the MSER detector (kernel trace),
# with the PMC summaries written to gpurun_out/r04_pmc_*.json.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
export FM3D_LM_MAX_SECONDS=40
ALL="FETCH_SIZE WRITE_SIZE,TCC_HIT_sum,TCC_MISS_sum SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_INSTS_VALU,SQ_INSTS_SALU SQ_INSTS_LDS,SQ_ACTIVE_INST_LDS,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_LDS_ADDR_CONFLICT,SQ_LDS_UNALIGNED_STALL,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR"
BASIC="FETCH_SIZE WRITE_SIZE,TCC_HIT_sum,TCC_MISS_sum SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_INSTS_VALU,SQ_INSTS_SALU"
FM3D_PMC="$ALL" tools/prof_lm.sh r04fres --mode resident --steps 2 --warmup 1 --no-cpu || exit 1
python tools/pmc_summary.py gpurun_out/prof_r04fres lm2_kernel --workload 100000,64,3 --command "tools/r04_final_prof.sh -> tools/prof_lm.sh r04fres (bench.py --mode resident --steps 2 --warmup 1 --no-cpu), one rocprofv3 --pmc pass per counter group" --out gpurun_out/r04_pmc_c4.json > /dev/null || exit 1
FM3D_PMC="$BASIC" tools/prof_lm.sh r04fstream --steps 6 --warmup 2 --no-cpu || exit 1
python tools/pmc_summary.py gpurun_out/prof_r04fstream lm2_kernel --workload 100000,64,3 --command "tools/r04_final_prof.sh -> tools/prof_lm.sh r04fstream (bench.py --steps 6 --warmup 2 --no-cpu: 4 pairs in flight, 2 per LM launch), one rocprofv3 --pmc pass per counter group" --out gpurun_out/r04_pmc_c4_stream.json > /dev/null || exit 1
FM3D_PMC="$BASIC" tools/prof_lm.sh r04fc3 --workload c3 --steps 20 --warmup 3 --no-cpu || exit 1
python tools/pmc_summary.py gpurun_out/prof_r04fc3 ncc_kernel --workload 10000,32,3 --command "tools/r04_final_prof.sh -> tools/prof_lm.sh r04fc3 (bench.py --workload c3 --steps 20 --warmup 3 --no-cpu), one rocprofv3 --pmc pass per counter group" --out gpurun_out/r04_pmc_c3.json > /dev/null || exit 1
FM3D_PMC="" tools/prof_lm.sh r04fc2 --workload c2 --steps 100 --warmup 10 --no-cpu || exit 1
mkdir -p gpurun_out/prof_r04mser
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r04mser -o run --output-format csv -- python3 tools/mser_time.py > gpurun_out/prof_r04mser/log.txt 2>&1
