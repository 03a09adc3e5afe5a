cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
for round in 1 2; do
  for v in qg1tr cur; do
    if [ $v = cur ]; then unset FM3D_LIB; else export FM3D_LIB=$R/3dfeaturematcher_amd/_ab/libfm3d_$v.so; fi
    for n in 100000 10000; do
      timeout -k 10 200 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_qgab_${v}_${n}_$round -o run --output-format csv \
        -- python3 $R/tools/knn_parts_sweep.py --n $n --parts auto --reps 3 > $R/gpurun_out/qgab_${v}_${n}_$round.log 2>&1 || exit 1
    done
  done
done
