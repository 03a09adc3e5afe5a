#!/bin/bash
# Round-6 GPU session 7: fm3d_pipeline_submit_dlt_pair (C2 from host memory with no host wait): the
# C2 pipeline tests, then the C2 host-to-host lines (u8 and float rows).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_c2_pipeline.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r06_pytest_c2pair.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload c2 --steps 300 --warmup 30 --io host > gpurun_out/r06s7_c2_host_u8.json 2> gpurun_out/r06s7_c2_host_u8.err || exit 1
timeout -k 10 300 python bench.py --workload c2 --steps 300 --warmup 30 --io host --desc-dtype f32 > gpurun_out/r06s7_c2_host_f32.json 2> gpurun_out/r06s7_c2_host_f32.err || exit 1
timeout -k 10 300 python bench.py --workload c2 --steps 300 --warmup 30 > gpurun_out/r06s7_c2.json 2> gpurun_out/r06s7_c2.err || exit 1
