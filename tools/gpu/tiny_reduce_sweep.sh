#!/bin/bash
# TinyImageNet: weight-gradient split-K reduction schedule with the deferred launch
set -o pipefail
O=${1:-gpurun_out/tiny_reduce}
for r in 1 2; do
  bash tools/gpu/sweep_env.sh $O/r$r "resnet50_tiny_imagenet" base DBX_DEFER_REDUCE=1 DBX_FUSE_WGRAD_REDUCE=1 DBX_DEFER_REDUCE=1+DBX_LAZY_JOIN=1 || exit 1
done
