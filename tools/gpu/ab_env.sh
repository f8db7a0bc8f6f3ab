#!/bin/bash
# interleaved A/B of engine switches (FIELDS: comma-separated EngineConfig fields, all set to 1 / 0 through
# DBX_ENGINE) on the bench presets:  ab_env.sh OUT FIELDS "presets" rounds
set -o pipefail
O=${1:-gpurun_out/ab}; VAR=${2:-fuse_dw}; PRESETS=${3:-"resnet18_cifar10 resnet50_tiny_imagenet headline"}; R=${4:-2}
mkdir -p $O
for r in $(seq 1 $R); do
  for p in $PRESETS; do
    for v in 1 0; do
      args="--steps 30 --warmup 10"; [ $p = headline ] && args="--steps 15 --warmup 5" || args="$args --preset $p"
      envs="DBX_ENGINE="; for vv in ${VAR//,/ }; do envs="$envs$vv=$v,"; done; envs=${envs%,}
      env $envs timeout -k 10 300 python bench.py $args > $O/${p}_${v}_r$r.log 2>&1 || { tail -20 $O/${p}_${v}_r$r.log; exit 1; }
      echo "$p $VAR=$v r$r: $(grep -o '"value": [0-9.]*' $O/${p}_${v}_r$r.log)"
    done
  done
done
