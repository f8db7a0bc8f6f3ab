#!/bin/bash
# Side-stream modes under the two-queue graph setting (DEBUG_HIP_FORCE_GRAPH_QUEUES=2): headline and
# TinyImageNet with DBX_OVERLAP_WGRAD 0 / 1 / 2 / 3 (unset = the default per size).
set -o pipefail
O=${1:-gpurun_out/r4_s16}
mkdir -p $O
for p in headline resnet50_tiny_imagenet; do
  args="--steps 20 --warmup 5"; [ $p != headline ] && args="$args --preset $p"
  for m in def 0 1 2 3; do
    if [ $m = def ]; then
      timeout -k 10 300 python bench.py $args > $O/${p}_$m.log 2>&1 || { tail -20 $O/${p}_$m.log; exit 1; }
    else
      DBX_OVERLAP_WGRAD=$m timeout -k 10 300 python bench.py $args > $O/${p}_$m.log 2>&1 || { tail -20 $O/${p}_$m.log; exit 1; }
    fi
    echo "$p overlap=$m: $(grep -o '"value": [0-9.]*' $O/${p}_$m.log)"
  done
done
