#!/bin/bash
# side-stream weight gradients sized to leave N CUs to the main chain (DBX_SIDE_CU_RESERVE)
set -o pipefail
O=${1:-gpurun_out/cu_reserve}
for r in 1 2; do
  bash tools/gpu/sweep_env.sh $O/r$r "headline" base DBX_SIDE_CU_RESERVE=8 DBX_SIDE_CU_RESERVE=16 DBX_SIDE_CU_RESERVE=32 DBX_SIDE_CU_RESERVE=64 || exit 1
done
bash tools/gpu/sweep_env.sh $O/r3 "resnet50_tiny_imagenet resnet18_cifar10" base DBX_SIDE_CU_RESERVE=16 DBX_SIDE_CU_RESERVE=32 || exit 1
