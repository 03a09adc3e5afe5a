#!/bin/bash
# Same-box A/B of ncc_kernel: a variant library ($NCC_A_LIB, default 3dfeaturematcher_amd/_ab/libfm3d_nccold.so:
# the round-4 projection form built from commit 2edf184's fm3d_ncc.hip) as "old" against the in-tree
# library as "new", alternating, rocprofv3 kernel trace of bench.py --workload c3 --inflight 1 each.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
for round in 1 2; do
  for v in old new; do
    if [ $v = old ]; then export FM3D_LIB=${NCC_A_LIB:-$R/3dfeaturematcher_amd/_ab/libfm3d_nccold.so}; else unset FM3D_LIB; fi
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_nccab_${v}_$round -o run --output-format csv \
      -- python3 $R/bench.py --workload c3 --inflight 1 --steps 6 --warmup 2 --no-cpu > $R/gpurun_out/nccab_${v}_$round.log 2>&1 || exit 1
  done
done
