#!/bin/bash
# Same-box A/B of ncc_kernel with the camera constants re-read through the scalar cache at each
# use (3dfeaturematcher_amd/_ab/libfm3d_nccrr.so, -DFM3D_NCC_REREAD=1) against the in-tree build,
# both hypothesis counts, alternating: rocprofv3 kernel trace of tools/time_front.py.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
for round in 1 2; do
  for v in rr base; do
    if [ $v = rr ]; then export FM3D_LIB=$R/3dfeaturematcher_amd/_ab/libfm3d_nccrr.so; else unset FM3D_LIB; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_nccrr_${v}_$round -o run --output-format csv \
      -- python3 $R/tools/time_front.py --reps 5 > $R/gpurun_out/nccrr_${v}_$round.log 2>&1 || exit 1
  done
done
