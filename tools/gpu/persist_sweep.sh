#!/bin/bash
# persistence switches on the small presets
set -o pipefail
O=${1:-gpurun_out/persist_sweep}
for r in 1 2; do
  bash tools/gpu/sweep_env.sh $O/r$r "resnet50_tiny_imagenet resnet18_cifar10" base DBX_PERSIST=0 DBX_PERSIST_DMA1=1 || exit 1
done
