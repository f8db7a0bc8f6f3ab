#!/bin/bash
# Round 4: batched reduce of the small-slab gradients only (DBX_DEFER_MAX_MB) on TinyImageNet / CIFAR.
set -o pipefail
O=${1:-gpurun_out/r4_s13}
export TMPDIR=/tmp
bash tools/gpu/sweep_env.sh $O "resnet50_tiny_imagenet" base DBX_DEFER_REDUCE=1+DBX_DEFER_MAX_MB=1 \
  DBX_DEFER_REDUCE=1+DBX_DEFER_MAX_MB=4 DBX_DEFER_REDUCE=1+DBX_DEFER_MAX_MB=16 base DBX_DEFER_REDUCE=1+DBX_DEFER_MAX_MB=4
bash tools/gpu/sweep_env.sh $O "resnet18_cifar10" base DBX_DEFER_MAX_MB=4 DBX_DEFER_MAX_MB=16 base
