#!/bin/bash
# Round-5 headline: smoke(), the driver's C4 command (bench.py --steps 20 --warmup 5), and the
# rocprofv3 kernel trace of the same command.  Every step under its own limit; the first failure ends it.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05_smoke.log 2>&1 || exit 1
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r05_c4.json 2> gpurun_out/r05_c4.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r05c4 -o run --output-format csv \
  -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu > $R/gpurun_out/r05_c4_prof.log 2>&1 || exit 1
