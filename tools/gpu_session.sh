#!/bin/bash
# One GPU session: each step under its own time limit; stop at the first crash/timeout.
# Usage: tools/gpu_session.sh "<step1 cmd>" "<step2 cmd>" ...   (logs in gpurun_out/stepN.log)
mkdir -p gpurun_out
export FM3D_ORACLE_THREADS=${FM3D_ORACLE_THREADS:-16}
i=0
for cmd in "$@"; do
  i=$((i+1))
  echo "=== step $i: $cmd" | tee -a gpurun_out/session.log
  bash -c "$cmd" > gpurun_out/step$i.log 2>&1
  rc=$?
  echo "=== step $i rc=$rc" | tee -a gpurun_out/session.log
  tail -5 gpurun_out/step$i.log | tee -a gpurun_out/session.log
  # any failure may be a GPU fault surfacing as an exception: start nothing more on the GPU
  if [ $rc -ne 0 ]; then echo "stopping after rc=$rc" | tee -a gpurun_out/session.log; exit $rc; fi
done
