#!/bin/bash
# Round-6 GPU session 4: the staging copies on host threads (StagingCopier): pipeline + C4 tests, the
# C2 host-to-host lines (u8 and float rows) and the C4 headline.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_c2_pipeline.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 \
  --timeout-method thread -k "not c5_1m and not c3_orb10k" > gpurun_out/r06_pytest_gpu4.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload c2 --steps 300 --warmup 30 --io host --no-cpu > gpurun_out/r06s4_c2_host_u8.json 2> gpurun_out/r06s4_c2_host_u8.err || exit 1
timeout -k 10 300 python bench.py --workload c2 --steps 300 --warmup 30 --io host --desc-dtype f32 > gpurun_out/r06s4_c2_host_f32.json 2> gpurun_out/r06s4_c2_host_f32.err || exit 1
FM3D_STAGING_THREADS=1 timeout -k 10 300 python bench.py --workload c2 --steps 300 --warmup 30 --io host --desc-dtype f32 --no-cpu > gpurun_out/r06s4_c2_host_f32_1thr.json 2> gpurun_out/r06s4_c2_host_f32_1thr.err || exit 1
timeout -k 10 600 python bench.py --no-cpu > gpurun_out/r06s4_c4.json 2> gpurun_out/r06s4_c4.err || exit 1
