cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python -u -m pytest tests/test_compat_main.py tests/test_gpu_surf.py tests/test_gpu_sift.py -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/r03_pytest_gpu_compat.log 2>&1
