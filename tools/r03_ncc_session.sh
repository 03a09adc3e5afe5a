cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_c2_pipeline.py tests/test_gpu_parity.py -k "ncc" -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/r03_pytest_gpu_ncc2.log 2>&1 && \
timeout -k 10 300 python -u bench.py --workload c3 --steps 10 --warmup 2 --out gpurun_out/r03_bench_c3ncc.json > gpurun_out/r03_bench_c3ncc.log 2>&1 && \
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_c3ncc -o c3 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload c3 --steps 10 --warmup 2 --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/prof_c3ncc.log 2>&1
