#!/bin/bash
# Same-box A/B of ncc_kernel with wave-uniform plane constants in scalar registers
# (3dfeaturematcher_amd/_ab/libfm3d_nccuni.so, -DFM3D_NCC_UNI=1) against the in-tree build, for
# both hypothesis counts (16: ncc_kernel<4, true>, 32: ncc_kernel<8, true>), alternating:
# rocprofv3 kernel trace of tools/time_front.py.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
for round in 1 2; do
  for v in uni base; do
    if [ $v = uni ]; then export FM3D_LIB=$R/3dfeaturematcher_amd/_ab/libfm3d_nccuni.so; else unset FM3D_LIB; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_nccuni_${v}_$round -o run --output-format csv \
      -- python3 $R/tools/time_front.py --reps 5 > $R/gpurun_out/nccuni_${v}_$round.log 2>&1 || exit 1
  done
done
