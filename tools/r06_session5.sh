#!/bin/bash
# Round-6 closing GPU session (one gpurun call) on the final tree, after the C3 / C5 fixtures were
# regenerated on OpenCV's SVD: the whole -m gpu suite, smoke(), the C4 headline as the driver runs it,
# and the C5 pair through fm3d_mgpu on one GPU (verified against full_c5sub.npz; stages_ms from one
# isolated pair).  Every step under its own limit; the first failure ends the session.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r06_pytest_gpu_final.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_smoke_final.log 2>&1 || exit 1
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r06_c4_final.json 2> gpurun_out/r06_c4_final.err || exit 1
timeout -k 10 900 python bench.py --gpus 1 --mgpu --steps 4 --warmup 1 > gpurun_out/r06_c5_mgpu_1gpu.json 2> gpurun_out/r06_c5_mgpu_1gpu.err || exit 1
