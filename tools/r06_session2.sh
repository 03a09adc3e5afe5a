#!/bin/bash
# Round-6 GPU session 2 (one gpurun call): the -m gpu suite except the C3 / C5 fixture tests (their
# fixtures are being regenerated for the cvSVD DLT), smoke(), the C4 headline (u8 rows, then the float
# rows of the reference's cv::Mat), the C4 kernel traces (stream: copy / fill kernels; resident: the
# LM launch) and the LM counters of one resident launch.  Every step under its own limit; the first
# failure ends the session.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "not c5_1m and not c3_orb10k" > gpurun_out/r06_pytest_gpu2.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_smoke.log 2>&1 || exit 1
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r06_c4.json 2> gpurun_out/r06_c4.err || exit 1
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --desc-dtype f32 --no-cpu > gpurun_out/r06_c4_f32.json 2> gpurun_out/r06_c4_f32.err || exit 1
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r06c4 -o run --output-format csv \
  -- python3 $R/bench.py --steps 12 --warmup 3 --no-cpu > $R/gpurun_out/r06_c4_prof.log 2>&1 || exit 1
cd $R
export FM3D_LM_MAX_SECONDS=40
ALL="FETCH_SIZE WRITE_SIZE,TCC_HIT_sum,TCC_MISS_sum SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_INSTS_VALU,SQ_INSTS_SALU SQ_INSTS_LDS,SQ_ACTIVE_INST_LDS,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_LDS_ADDR_CONFLICT,SQ_LDS_UNALIGNED_STALL,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR"
FM3D_PMC="$ALL" tools/prof_lm.sh r06res --mode resident --steps 2 --warmup 1 --no-cpu || exit 1
python tools/pmc_summary.py gpurun_out/prof_r06res lm2_kernel --workload 100000,64,3 --command "tools/r06_session2.sh -> tools/prof_lm.sh r06res (bench.py --mode resident --steps 2 --warmup 1 --no-cpu), one rocprofv3 --pmc pass per counter group" --out gpurun_out/r06_pmc_c4.json > /dev/null || exit 1
