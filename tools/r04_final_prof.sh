#!/bin/bash
# Round-4 closing measurement, part 2 (one gpurun call): rocprofv3 kernel traces + PMC passes of the
# C4 LM launch (resident: one launch at a time, the per-launch roofline and HBM bytes), the streamed
# headline, C2, C3, and the MSER detector; summaries under gpurun_out/prof_r04f*.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 1000 tools/r04_prof.sh || exit 1
mkdir -p gpurun_out/prof_r04mser
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r04mser -o run --output-format csv -- python3 tools/mser_time.py > gpurun_out/prof_r04mser/log.txt 2>&1
