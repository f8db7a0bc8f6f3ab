#!/bin/bash
# interleaved A/B of environment switches (VAR: comma-separated, all set to 1 / 0) on the bench
# presets:  ab_env.sh OUT VAR "presets" rounds
set -o pipefail
O=${1:-gpurun_out/ab}; VAR=${2:-DBX_FUSE_WGRAD_REDUCE}; PRESETS=${3:-"resnet18_cifar10 resnet50_tiny_imagenet headline"}; R=${4:-2}
mkdir -p $O
for r in $(seq 1 $R); do
  for p in $PRESETS; do
    for v in 1 0; do
      args="--steps 30 --warmup 10"; [ $p = headline ] && args="--steps 15 --warmup 5" || args="$args --preset $p"
      envs=""; for vv in ${VAR//,/ }; do envs="$envs $vv=$v"; done
      env $envs timeout -k 10 300 python bench.py $args > $O/${p}_${v}_r$r.log 2>&1 || { tail -20 $O/${p}_${v}_r$r.log; exit 1; }
      echo "$p $VAR=$v r$r: $(grep -o '"value": [0-9.]*' $O/${p}_${v}_r$r.log)"
    done
  done
done
