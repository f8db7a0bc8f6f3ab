#!/bin/bash
# TinyImageNet: how many of the last batch's gradients go to the main stream with the deferred launch; headline:
# the deferred launch with the main-stream tail / stem switches.
set -o pipefail
O=${1:-gpurun_out/defer_sweep2}
for r in 1 2; do
  bash tools/gpu/sweep_env.sh $O/r$r "resnet50_tiny_imagenet" base DBX_TAIL_MAIN=3 DBX_TAIL_MAIN=4 DBX_TAIL_MAIN=5 || exit 1
  bash tools/gpu/sweep_env.sh $O/r$r "headline" base DBX_SIDE_DEFER=1 DBX_SIDE_DEFER=1+DBX_TAIL_MAIN=1 DBX_SIDE_DEFER=1+DBX_STEM_WG_MAIN=1 || exit 1
done
