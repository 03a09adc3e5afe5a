#!/bin/bash
# Full GPU suite + matcher kernel stats (all descriptor types) at 10k and 100k (via gpurun).
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp FM3D_LM_MAX_SECONDS=${FM3D_LM_MAX_SECONDS:-60}
tools/gpu_session.sh \
  "timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 900 --timeout-method thread -s" \
  "cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/match10k -o run --output-format csv -- python3 $R/tools/time_match.py --n 10000 --reps 5" \
  "cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/match100k -o run --output-format csv -- python3 $R/tools/time_match.py --n 100000 --reps 3"
