#!/bin/bash
# gpurun wrapper for this container: retries ONLY when the box could not be prepared
# (status "transient": nothing ran, nothing charged).  Usage: tools/gpu_call.sh TIMEOUT 'cmd'
T=$1; shift
for attempt in $(seq 1 ${GPU_CALL_ATTEMPTS:-8}); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@" > /tmp/gpu_call.log 2>&1
  rc=$?
  if grep -q "status=transient" /tmp/gpu_call.log || [ $rc -eq 3 ]; then
    echo "[gpu_call] transient (attempt $attempt), waiting" >&2
    sleep 75
    continue
  fi
  cat /tmp/gpu_call.log | tail -4
  exit $rc
done
cat /tmp/gpu_call.log | tail -4
exit 3
