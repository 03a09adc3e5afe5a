cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in qg1 qg2; do
  for n in 100000 10000; do
    FM3D_LIB=$R/3dfeaturematcher_amd/_ab/libfm3d_$v.so timeout -k 10 200 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_ab_${v}_$n -o run --output-format csv -- python3 $R/tools/knn_parts_sweep.py --n $n --parts auto,4,8,16 --reps 3 > $R/gpurun_out/ab_${v}_$n.log 2>&1 || exit 1
  done
done
