#!/bin/bash
# Round-3 measurement on one GPU box (run through gpurun): the whole GPU parity suite, smoke(), the
# rocprofv3 kernel trace and one --pmc pass per counter group over the C4 bench
# (tools/prof_session.sh), the PMC summary written where bench.py reads its traffic figure
# (profiles/r03_pmc_c4.json), then the default bench line (with the CPU baseline).  Outputs under
# gpurun_out/.
export FM3D_LM_MAX_SECONDS=${FM3D_LM_MAX_SECONDS:-40}
tools/gpu_session.sh \
  "timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread" \
  "timeout -k 10 200 python -u -c 'import __graft_entry__ as g; g.smoke()'" \
  "timeout -k 10 900 tools/prof_session.sh r03" \
  "python tools/pmc_summary.py gpurun_out/prof_r03 lm2_kernel --workload 100000,64,3 --command 'tools/r03_session.sh -> tools/prof_session.sh r03 (bench.py C4 --steps 2 --warmup 1 --no-cpu), one rocprofv3 --pmc pass per counter group' --out gpurun_out/r03_pmc_c4.json" \
  "timeout -k 10 400 python -u bench.py --out gpurun_out/bench_r03.json --pmc-json gpurun_out/r03_pmc_c4.json"
