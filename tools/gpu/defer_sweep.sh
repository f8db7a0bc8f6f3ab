#!/bin/bash
# Side-stream schedule knobs re-swept with the deferred launch (clean main / side queue split) on the small presets.
set -o pipefail
O=${1:-gpurun_out/defer_sweep}
for r in 1 2; do
  bash tools/gpu/sweep_env.sh $O/r$r "resnet50_tiny_imagenet resnet18_cifar10" base DBX_OVERLAP_WGRAD=3 DBX_LAST_SEG_BLOCKS=1 DBX_TAIL_MAIN=0 DBX_TAIL_MAIN=3 DBX_STEM_WG_MAIN=0 DBX_SEG_TAIL_MAIN=1 || exit 1
done
