#!/bin/bash
# Round-end measurement on one GPU box (run through gpurun): GPU parity suite, smoke(), the
# rocprofv3 kernel trace and one --pmc pass per counter group (tools/prof_session.sh), the PMC
# summary written where bench.py reads its traffic figure, then the default bench line (with the
# CPU baseline).  Outputs under gpurun_out/.
export FM3D_LM_MAX_SECONDS=${FM3D_LM_MAX_SECONDS:-40}
tools/gpu_session.sh \
  "timeout -k 10 300 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread" \
  "timeout -k 10 200 python -u -c 'import __graft_entry__ as g; g.smoke()'" \
  "timeout -k 10 900 tools/prof_session.sh final" \
  "python tools/pmc_summary.py gpurun_out/prof_final lm2_kernel --workload 100000,64,3 --command 'tools/final_session.sh -> tools/prof_session.sh final (bench.py C4 --steps 2 --warmup 1 --no-cpu), one rocprofv3 --pmc pass per counter group' --out profiles/r02_pmc_c4.json" \
  "timeout -k 10 400 python -u bench.py --out gpurun_out/bench_final.json"
