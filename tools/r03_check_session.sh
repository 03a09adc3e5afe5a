#!/bin/bash
# Whole GPU suite + smoke + the default bench line on the tree as it stands (no profiling passes).
cd "$GRAFT_REPO_ROOT" || exit 1
export FM3D_LM_MAX_SECONDS=${FM3D_LM_MAX_SECONDS:-40}
tools/gpu_session.sh \
  "timeout -k 10 500 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread" \
  "timeout -k 10 200 python -u -c 'import __graft_entry__ as g; g.smoke()'" \
  "timeout -k 10 400 python -u bench.py --out gpurun_out/bench_check.json"
