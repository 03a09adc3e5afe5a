#!/bin/bash
# Same-box A/B of the LM kernel's deferred, lane-parallel sph2car (in-tree library) against the
# previous commit's lane-0 form (3dfeaturematcher_amd/_ab/libfm3d_trigold.so): resident C4 launches,
# alternating.  Then the LM parity tests of the in-tree library.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_lm_tree.py \
  -k "(normals or lm or c3_orb or c5 or pipeline or tree) and not c4_sift100k" > gpurun_out/r05_trig_pytest.log 2>&1 || exit 1
for round in 1 2; do
  for v in old new; do
    if [ $v = old ]; then export FM3D_LIB=$R/3dfeaturematcher_amd/_ab/libfm3d_trigold.so; else unset FM3D_LIB; fi
    timeout -k 10 300 python bench.py --mode resident --steps 3 --warmup 1 --no-cpu > gpurun_out/trigab_${v}_$round.json 2> gpurun_out/trigab_${v}_$round.err || exit 1
  done
done
