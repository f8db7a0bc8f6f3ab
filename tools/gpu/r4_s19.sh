#!/bin/bash
# In-launch split-K weight-gradient reduce (DBX_FUSE_WGRAD_REDUCE, DBX_WGRAD_FUSE_MAX bytes) on the small presets.
set -o pipefail
O=${1:-gpurun_out/r4_s19}
bash tools/gpu/sweep_env.sh $O "resnet50_tiny_imagenet" base DBX_FUSE_WGRAD_REDUCE=1 DBX_FUSE_WGRAD_REDUCE=1+DBX_WGRAD_FUSE_MAX=4194304 \
  DBX_FUSE_WGRAD_REDUCE=1+DBX_WGRAD_FUSE_MAX=16777216 base DBX_FUSE_WGRAD_REDUCE=1 \
  && bash tools/gpu/sweep_env.sh $O "resnet18_cifar10" base DBX_FUSE_WGRAD_REDUCE=1 DBX_FUSE_WGRAD_REDUCE=1+DBX_WGRAD_FUSE_MAX=4194304 base
