#!/bin/bash
# BN-backward apply folding thresholds re-swept on the small presets with the deferred side launch
set -o pipefail
O=${1:-gpurun_out/fold_sweep}
for r in 1 2; do
  bash tools/gpu/sweep_env.sh $O/r$r "resnet50_tiny_imagenet resnet18_cifar10" base DBX_FOLD_MIN_ELEMS=0 DBX_FOLD_MIN_ELEMS=1048576 DBX_FOLD_MIN_ELEMS=4194304 DBX_FOLD_MIN_ELEMS=0+DBX_FOLD_MAX_RATIO=8 || exit 1
done
