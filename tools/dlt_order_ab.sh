#!/bin/bash
# Same-box A/B of the DLT Jacobi pair order in the C2 pipeline: the cyclic order with compile-time
# column indices (3dfeaturematcher_amd/_ab/libfm3d_cyc.so, -DFM3D_DLT_CYCLIC=1) against the in-tree
# round-robin build, alternating; rocprofv3 kernel trace of bench.py --workload c2 --inflight 1.
# The FM3D_DLT_CYCLIC switch was removed after the A/B (profiles/r05_dlt_order_ab.json); re-add the
# cyclic pair sequence under that macro in dlt_nullvec to repeat it.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
for round in 1 2; do
  for v in cyc rr; do
    if [ $v = cyc ]; then export FM3D_LIB=$R/3dfeaturematcher_amd/_ab/libfm3d_cyc.so; else unset FM3D_LIB; fi
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_dltab_${v}_$round -o run --output-format csv \
      -- python3 $R/bench.py --workload c2 --inflight 1 --steps 200 --warmup 20 --no-cpu > $R/gpurun_out/dltab_${v}_$round.log 2>&1 || exit 1
  done
done
