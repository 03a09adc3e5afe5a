#!/bin/bash
# Round-6 GPU session 1: the cvSVD DLT / polar factor and the device-side float-row pack on the GPU
# (the -m gpu tests that do not read the full-size fixtures, which are being regenerated), the C2
# bench lines (resident u8; host-to-host u8 and float rows), a C2 kernel trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "not c4_sift100k and not c5_1m and not c3_orb10k" > gpurun_out/r06_pytest_gpu1.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload c2 --steps 300 --warmup 30 > gpurun_out/r06_c2.json 2> gpurun_out/r06_c2.err || exit 1
timeout -k 10 300 python bench.py --workload c2 --steps 300 --warmup 30 --io host --no-cpu > gpurun_out/r06_c2_host_u8.json 2> gpurun_out/r06_c2_host_u8.err || exit 1
timeout -k 10 300 python bench.py --workload c2 --steps 300 --warmup 30 --io host --desc-dtype f32 > gpurun_out/r06_c2_host_f32.json 2> gpurun_out/r06_c2_host_f32.err || exit 1
FM3D_PMC= tools/prof_lm.sh r06c2 --workload c2 --inflight 1 --steps 200 --warmup 20 --no-cpu || exit 1
