#!/bin/bash
# per-block forks + deferred launch + lazy joins: reservation / stem placement around it, all presets
set -o pipefail
O=${1:-gpurun_out/mode3_sweep}
M3="DBX_OVERLAP_WGRAD=3+DBX_SIDE_DEFER=1+DBX_LAZY_JOIN=1"
for r in 1 2; do
  bash tools/gpu/sweep_env.sh $O/r$r "headline" base $M3 $M3+DBX_SIDE_CU_RESERVE=32 $M3+DBX_SIDE_CU_RESERVE=96 $M3+DBX_STEM_WG_MAIN=1 || exit 1
  bash tools/gpu/sweep_env.sh $O/r$r "resnet50_tiny_imagenet resnet18_cifar10" base $M3 $M3+DBX_SIDE_CU_RESERVE=32 $M3+DBX_SIDE_CU_RESERVE=96 || exit 1
done
