#!/bin/bash
# Round-3 closing measurement on one GPU box: tools/r03_session.sh's steps (the whole GPU parity suite,
# smoke(), the rocprofv3 kernel trace + one --pmc pass per counter group over the C4 bench, the PMC
# summary, the default bench line) and the rocprofv3 summary of the auxiliary kernels (tools/prof_aux.py).
export FM3D_LM_MAX_SECONDS=${FM3D_LM_MAX_SECONDS:-40}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tools/gpu_session.sh \
  "timeout -k 10 500 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread" \
  "timeout -k 10 200 python -u -c 'import __graft_entry__ as g; g.smoke()'" \
  "timeout -k 10 900 tools/prof_session.sh r03" \
  "python tools/pmc_summary.py gpurun_out/prof_r03 lm2_kernel --workload 100000,64,3 --command 'tools/r03_final_session.sh -> tools/prof_session.sh r03 (bench.py C4 --steps 2 --warmup 1 --no-cpu), one rocprofv3 --pmc pass per counter group' --out gpurun_out/r03_pmc_c4.json" \
  "timeout -k 10 400 python -u bench.py --out gpurun_out/bench_r03.json --pmc-json gpurun_out/r03_pmc_c4.json" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_aux_final -o aux --output-format csv -- python3 tools/prof_aux.py > gpurun_out/prof_aux_final.json"
