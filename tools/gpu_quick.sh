#!/bin/bash
# Parity subset + C4 bench on the GPU box (run through gpurun).  Usage: tools/gpu_quick.sh TAG [bench args]
TAG=$1; shift
export FM3D_LM_MAX_SECONDS=${FM3D_LM_MAX_SECONDS:-40}
tools/gpu_session.sh \
  "timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-cpu --out gpurun_out/bench_$TAG.json $*"
