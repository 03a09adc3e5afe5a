#!/bin/bash
# Round-6 GPU session 6: the C4 full test against the regenerated full-set parity arrays (point for
# point), then C5 through fm3d_mgpu with device 0 listed 8 times (the 8-device host path on one GPU).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -s --timeout 400 --timeout-method thread \
  -k "c4_sift100k" > gpurun_out/r06_pytest_c4full.log 2>&1 || exit 1
timeout -k 10 900 python bench.py --gpus 8 --mgpu --alias-devices --steps 4 --warmup 1 --ref-steps 2 > gpurun_out/r06_c5_alias8.json 2> gpurun_out/r06_c5_alias8.err || exit 1
