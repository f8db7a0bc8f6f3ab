#!/bin/bash
set -o pipefail
O=${1:-gpurun_out/ldspad}
for r in 1 2; do
  bash tools/gpu/sweep_env.sh $O/r$r "headline resnet50_tiny_imagenet" base DBX_WGRAD_LDS_PAD=32768 DBX_SIDE_CU_RESERVE=32+DBX_WGRAD_LDS_PAD=32768 || exit 1
done
