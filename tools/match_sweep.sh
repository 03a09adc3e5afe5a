#!/bin/bash
# Sweep of the int8 matcher's launch variants (FM3D_I8_WPE x FM3D_I8_PARTS) under rocprofv3 kernel
# stats.  Usage (via gpurun): tools/match_sweep.sh TAG "N:WPE:PARTS:SCHED ..."
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
STEPS=()
for cfg in $1; do
  IFS=: read n w p sc <<< "$cfg"
  STEPS+=("cd /tmp && FM3D_I8_WPE=$w FM3D_I8_PARTS=$p FM3D_I8_SCHED=${sc:-0} FM3D_I8_MAX_PARTS=64 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_${n}_w${w}_p${p}_s${sc:-0} -o run --output-format csv -- python3 $R/tools/time_match.py --n $n --reps 5 --kinds ${KINDS:-sift128_u8,orb256_bits}")
done
tools/gpu_session.sh "${STEPS[@]}"
