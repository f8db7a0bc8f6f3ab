#!/bin/bash
set -o pipefail
O=${1:-gpurun_out/cu_reserve2}
for r in 1 2; do
  bash tools/gpu/sweep_env.sh $O/r$r "headline" base DBX_SIDE_CU_RESERVE=64 DBX_SIDE_CU_RESERVE=96 DBX_SIDE_CU_RESERVE=128 || exit 1
  bash tools/gpu/sweep_env.sh $O/r$r "resnet50_tiny_imagenet" base DBX_SIDE_CU_RESERVE=32 DBX_SIDE_CU_RESERVE=64 DBX_SIDE_CU_RESERVE=96 || exit 1
done
