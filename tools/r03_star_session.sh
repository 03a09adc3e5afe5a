cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_star.py tests/test_gpu_features.py tests/test_gpu_surf.py tests/test_compat_main.py -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/r03_pytest_gpu_star.log 2>&1 && \
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_aux_star -o aux --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/prof_aux.py > $GRAFT_REPO_ROOT/gpurun_out/prof_aux_star.json 2> $GRAFT_REPO_ROOT/gpurun_out/prof_aux_star.err
