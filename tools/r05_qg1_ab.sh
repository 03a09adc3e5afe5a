#!/bin/bash
# Same-box A/B of the u8 matcher's query groups for small query sets: FM3D_KNN_QG1_BELOW=20000
# (one query group per wave at 10k queries: twice the workgroups) against 0 (two groups, the
# 100k-tuned default).  GPU parity of the matcher with one group forced at every size, the
# 10k x 10k kernel under rocprofv3 at several part counts, then the C2 line alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
FM3D_KNN_QG1_BELOW=100000000 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "knn or match or c2 or pipeline" > gpurun_out/qg1_pytest.log 2>&1 || exit 1
for v in 0 20000; do
  FM3D_KNN_QG1_BELOW=$v tools/prof_cmd.sh qg1_$v tools/knn_parts_sweep.py --n 10000 --parts auto,10,16,20 --reps 20 || exit 1
done
for r in 1 2; do
  for v in 0 20000; do
    FM3D_KNN_QG1_BELOW=$v timeout -k 10 300 python bench.py --workload c2 --steps 300 --warmup 30 --no-cpu \
      > gpurun_out/qg1_c2_${v}_$r.json 2> gpurun_out/qg1_c2_${v}_$r.err || exit 1
  done
done
