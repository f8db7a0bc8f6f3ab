#!/bin/bash
# HIP graph queue count: DEBUG_HIP_FORCE_GRAPH_QUEUES=1 (every graph on one queue) vs the runtime
# default (parallel branches on extra queues; crashes in hipGraphLaunch on some graph shapes,
# profiles/r4_final2/README.md) -- bench throughput of the headline and the small presets.
set -o pipefail
O=${1:-gpurun_out/r4_q1}
mkdir -p $O
for p in headline resnet18_cifar10 resnet50_tiny_imagenet; do
  args="--steps 20 --warmup 5"; [ $p != headline ] && args="$args --preset $p"
  for q in def 1 def 1; do
    if [ $q = def ]; then
      timeout -k 10 300 python bench.py $args > $O/${p}_$q.log 2>&1 || { tail -20 $O/${p}_$q.log; exit 1; }
    else
      DEBUG_HIP_FORCE_GRAPH_QUEUES=$q timeout -k 10 300 python bench.py $args > $O/${p}_$q.log 2>&1 || { tail -20 $O/${p}_$q.log; exit 1; }
    fi
    echo "$p q=$q: $(grep -o '"value": [0-9.]*' $O/${p}_$q.log)"
  done
done
