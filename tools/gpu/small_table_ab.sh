#!/bin/bash
# The small-map fwd / dgrad tune entries (tune_small.sh) re-A/B'd after the deferred side launch.
set -o pipefail
O=${1:-gpurun_out/small_table_ab}
T=${2:?path of the candidate table inside the tree}
for r in 1 2; do
  bash tools/gpu/sweep_env.sh $O/r$r "resnet50_tiny_imagenet resnet18_cifar10" base DBX_TUNE_TABLE=$T || exit 1
done
