#!/bin/bash
# Same-box A/B of knn2_i8_kernel: the previous commit's library (3dfeaturematcher_amd/_ab/libfm3d_knnold.so)
# against the in-tree one, alternating, rocprofv3 kernel trace of tools/knn_parts_sweep.py at 100k and 10k.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
for round in 1 2; do
  for v in old new; do
    if [ $v = old ]; then export FM3D_LIB=$R/3dfeaturematcher_amd/_ab/libfm3d_knnold.so; else unset FM3D_LIB; fi
    for n in 100000 10000; do
      timeout -k 10 200 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_knnab_${v}_${n}_$round -o run --output-format csv \
        -- python3 $R/tools/knn_parts_sweep.py --n $n --parts auto --reps 3 > $R/gpurun_out/knnab_${v}_${n}_$round.log 2>&1 || exit 1
    done
  done
done
