#!/bin/bash
# Interleaved A/B of a kernel build variant (DBX_EXT_VARIANT=$VAR, built by build_ext --variant) against
# the tree's _C on the bench presets:  ab_variant_presets.sh OUT VAR "presets" rounds
set -o pipefail
O=${1:-gpurun_out/abv}; VAR=${2:-r4}; PRESETS=${3:-"headline resnet50_tiny_imagenet"}; R=${4:-3}
mkdir -p $O
for r in $(seq 1 $R); do
  for p in $PRESETS; do
    for v in new $VAR; do
      args="--steps 20 --warmup 5"; [ $p != headline ] && args="--steps 30 --warmup 10 --preset $p"
      if [ $v = new ]; then envs=""; else envs="DBX_EXT_VARIANT=$VAR"; fi
      env $envs timeout -k 10 300 python bench.py $args > $O/${p}_${v}_r$r.log 2>&1 || { tail -20 $O/${p}_${v}_r$r.log; exit 1; }
      echo "$p $v r$r: $(grep -o '"value": [0-9.]*' $O/${p}_${v}_r$r.log)"
    done
  done
done
