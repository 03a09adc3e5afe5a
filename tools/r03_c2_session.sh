cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_c2_pipeline.py tests/test_gpu_parity.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/r03_pytest_gpu_c2.log 2>&1 && \
timeout -k 10 300 python -u bench.py --workload c2 --steps 20 --warmup 3 --out gpurun_out/r03_bench_c2.json > gpurun_out/r03_bench_c2.log 2>&1 && \
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_c2 -o c2 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload c2 --steps 20 --warmup 3 --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/prof_c2.log 2>&1
