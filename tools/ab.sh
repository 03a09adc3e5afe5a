#!/bin/bash
# A/B timing of in-tree library builds on one GPU box: tools/ab.sh name1 name2[:VAR=value] ...
# (3dfeaturematcher_amd/_ab/libfm3d_<name>.so, optionally with one environment setting),
# alternating runs, bench JSON per run.
export FM3D_LM_MAX_SECONDS=40
for round in 1 2; do
  for spec in "$@"; do
    n=${spec%%:*}; envs=""; tag=$n
    if [[ "$spec" == *:* ]]; then envs=${spec#*:}; tag=${n}_${envs//=/}; fi
    env $envs FM3D_LIB=$PWD/3dfeaturematcher_amd/_ab/libfm3d_$n.so timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 \
      --no-cpu --out gpurun_out/ab_${tag}_$round.json > gpurun_out/ab_${tag}_$round.log 2>&1 || exit $?
  done
done
