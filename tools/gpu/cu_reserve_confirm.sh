#!/bin/bash
set -o pipefail
O=${1:-gpurun_out/cu_reserve3}
for r in 1 2; do
  bash tools/gpu/sweep_env.sh $O/r$r "headline" base DBX_SIDE_CU_RESERVE=64 DBX_SIDE_CU_RESERVE=80 || exit 1
  bash tools/gpu/sweep_env.sh $O/r$r "resnet50_tiny_imagenet resnet18_cifar10" base DBX_SIDE_CU_RESERVE=64 || exit 1
done
