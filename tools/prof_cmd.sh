#!/bin/bash
# PMC / kernel-trace passes over one python command on the GPU box (run via gpurun): one
# --kernel-trace --stats pass, then one --pmc pass per counter group in $FM3D_PMC.
# Usage: FM3D_PMC="A,B C,D" tools/prof_cmd.sh <tag> <script.py> <args...>
#   writes gpurun_out/prof_<tag>/{trace,pmc1,pmc2,...}; summarise with tools/pmc_summary.py
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
SCRIPT=$1; shift
run() {  # name, rocprofv3 args...
  local name=$1; shift
  echo "=== $name" >> $OUT/log.txt
  timeout -k 10 300 rocprofv3 "$@" -d $OUT/$name -o run --output-format csv -- python3 $R/$SCRIPT "${ARGS[@]}" >> $OUT/log.txt 2>&1
  local rc=$?
  echo "=== $name rc=$rc" >> $OUT/log.txt
  return $rc
}
ARGS=("$@")
run trace --kernel-trace --stats || exit 1
[ -n "$FM3D_PMC" ] || exit 0
i=0
for set in $FM3D_PMC; do
  i=$((i+1))
  run pmc$i --pmc ${set//,/ } || exit 1
done
