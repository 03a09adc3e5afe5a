#!/bin/bash
# Matcher session on the GPU box: matcher parity tests, then rocprofv3 kernel stats of
# tools/time_match.py at 10k and 100k (u8 + bits), and part-count variants at 10k.
# Usage (via gpurun): tools/match_session.sh [TAG]
TAG=${1:-m}
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
STEPS=("timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k 'knn2 or c2_ or c3_ or hamming or nndr' -x -q --timeout 120 --timeout-method thread")
for n in 10000 100000; do
  STEPS+=("cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_$n -o run --output-format csv -- python3 $R/tools/time_match.py --n $n --reps 5 --kinds sift128_u8,orb256_bits")
done
for p in ${PARTS:-}; do
  STEPS+=("cd /tmp && FM3D_I8_PARTS=$p timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_p$p -o run --output-format csv -- python3 $R/tools/time_match.py --n 10000 --reps 5 --kinds sift128_u8,orb256_bits")
done
tools/gpu_session.sh "${STEPS[@]}"
