#!/bin/bash
# Round-6 GPU session 3: the pipeline tests after the chunked staging copies, the C2 lines (resident;
# host to host with u8 and float rows), C3, and the C4 stream trace with the runtime's small copies
# forced onto the DMA engines (GPU_FORCE_BLIT_COPY_SIZE=0) to see which copy / fill kernels remain.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_c2_pipeline.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 \
  --timeout-method thread -k "not c5_1m and not c3_orb10k and not c4_sift100k" > gpurun_out/r06_pytest_gpu3.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload c2 --steps 300 --warmup 30 > gpurun_out/r06s3_c2.json 2> gpurun_out/r06s3_c2.err || exit 1
timeout -k 10 300 python bench.py --workload c2 --steps 300 --warmup 30 --io host --no-cpu > gpurun_out/r06s3_c2_host_u8.json 2> gpurun_out/r06s3_c2_host_u8.err || exit 1
timeout -k 10 300 python bench.py --workload c2 --steps 300 --warmup 30 --io host --desc-dtype f32 > gpurun_out/r06s3_c2_host_f32.json 2> gpurun_out/r06s3_c2_host_f32.err || exit 1
timeout -k 10 300 python bench.py --workload c3 --steps 40 --warmup 4 > gpurun_out/r06s3_c3.json 2> gpurun_out/r06s3_c3.err || exit 1
cd /tmp
export GPU_FORCE_BLIT_COPY_SIZE=0
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r06c4sdma -o run --output-format csv \
  -- python3 $R/bench.py --steps 12 --warmup 3 --no-cpu > $R/gpurun_out/r06_c4_sdma_prof.log 2>&1 || exit 1
