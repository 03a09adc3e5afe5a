#!/bin/bash
# Round-5 closing session (one gpurun call): the whole -m gpu suite, smoke(), the driver's C4 command
# and its rocprofv3 kernel trace, the C2 / C3 lines, and the counters bench.py reads for C3 and
# the 256-row-tile matcher.  Every step under its own limit; the first failure ends the session.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r05f_pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05f_smoke.log 2>&1 || exit 1
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r05f_c4.json 2> gpurun_out/r05f_c4.err || exit 1
timeout -k 10 300 python bench.py --workload c2 --steps 300 --warmup 30 > gpurun_out/r05f_c2.json 2> gpurun_out/r05f_c2.err || exit 1
timeout -k 10 300 python bench.py --workload c3 --steps 40 --warmup 4 > gpurun_out/r05f_c3.json 2> gpurun_out/r05f_c3.err || exit 1
BASIC="FETCH_SIZE WRITE_SIZE,TCC_HIT_sum,TCC_MISS_sum SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_INSTS_VALU,SQ_INSTS_SALU"
FM3D_PMC="$BASIC" tools/prof_lm.sh r05fc3 --workload c3 --inflight 1 --steps 6 --warmup 2 --no-cpu || exit 1
python tools/pmc_summary.py gpurun_out/prof_r05fc3 ncc_kernel --workload 10000,32,3 --command "tools/r05_final_session.sh -> tools/prof_lm.sh r05fc3 (bench.py --workload c3 --inflight 1 --steps 6 --warmup 2 --no-cpu), one rocprofv3 --pmc pass per counter group" --out gpurun_out/r05_pmc_c3.json > /dev/null || exit 1
FM3D_PMC="SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_INSTS_VALU,SQ_INSTS_SALU SQ_INSTS_LDS,SQ_ACTIVE_INST_LDS,SQ_LDS_BANK_CONFLICT,SQ_WAIT_INST_LDS,SQ_INSTS_VMEM_RD,SQ_VALU_MFMA_BUSY_CYCLES,SQ_INSTS_MFMA" \
  tools/prof_cmd.sh r05fknn tools/knn_parts_sweep.py --n 100000 --parts auto --reps 2 || exit 1
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r05fc4 -o run --output-format csv \
  -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu > $R/gpurun_out/r05f_c4_prof.log 2>&1 || exit 1
