#!/bin/bash
# Round-6 closing GPU session on the final tree: the whole -m gpu suite, smoke(), the C4 headline as
# the driver runs it, the C5 pair through fm3d_mgpu on one GPU.  Each step under its own limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r06_pytest_gpu_closing.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_smoke_closing.log 2>&1 || exit 1
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r06_c4_closing.json 2> gpurun_out/r06_c4_closing.err || exit 1
