#!/bin/bash
# Round-4 closing measurement, part 1 (one gpurun call): the whole GPU parity suite, smoke(), the
# default bench line (the driver's command) and the C2 / C3 / C5-through-fm3d_mgpu lines.
export FM3D_LM_MAX_SECONDS=${FM3D_LM_MAX_SECONDS:-40}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tools/gpu_session.sh \
  "timeout -k 10 500 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread" \
  "timeout -k 10 200 python -u -c 'import __graft_entry__ as g; g.smoke()'" \
  "timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --out gpurun_out/bench_r04.json" \
  "timeout -k 10 120 python -u bench.py --workload c2 --steps 200 --warmup 10 --out gpurun_out/bench_r04_c2.json" \
  "timeout -k 10 120 python -u bench.py --workload c3 --steps 20 --warmup 3 --out gpurun_out/bench_r04_c3.json"
