#!/bin/bash
# Round-5 GPU session: the whole -m gpu suite, the C2 bench line, C2 / C3 kernel traces (isolated
# launches).  Run through gpurun from the repo root; every step under its own time limit, the first
# failure ends the session.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} \
  > gpurun_out/r05_pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload c2 --steps 300 --warmup 30 > gpurun_out/r05_c2.json 2> gpurun_out/r05_c2.err || exit 1
FM3D_PMC= tools/prof_lm.sh r05c2b --workload c2 --inflight 1 --steps 200 --warmup 20 --no-cpu || exit 1
FM3D_PMC= tools/prof_lm.sh r05c3b --workload c3 --inflight 1 --steps 6 --warmup 2 --no-cpu || exit 1
