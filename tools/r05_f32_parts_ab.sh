#!/bin/bash
# A/B of the part model on the bf16-prefilter float matcher at 100k x 100k SURF-128: FM3D_I8_PARTS=1
# (one part, round 4's choice for query sets that fill the CUs) against the model, alternating.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
for round in 1 2; do
  for v in one model; do
    if [ $v = one ]; then export FM3D_I8_PARTS=1; else unset FM3D_I8_PARTS; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_f32ab_${v}_$round -o run --output-format csv \
      -- python3 $R/tools/time_f32.py --n 100000 --reps 3 > $R/gpurun_out/f32ab_${v}_$round.log 2>&1 || exit 1
  done
done
