#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration passes over tools/micro/fetch_calib (run on the GPU box).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/calib
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $R/tools/micro/fetch_calib > $OUT/log.txt 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc1 -o run --output-format csv -- $R/tools/micro/fetch_calib >> $OUT/log.txt 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc2 -o run --output-format csv -- $R/tools/micro/fetch_calib >> $OUT/log.txt 2>&1 || exit 1
