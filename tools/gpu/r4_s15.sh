#!/bin/bash
# Round 4: engine-switch sweep on TinyImageNet after the small-step changes.
set -o pipefail
O=${1:-gpurun_out/r4_s15}
export TMPDIR=/tmp
bash tools/gpu/sweep_env.sh $O "resnet50_tiny_imagenet" base DBX_OVERLAP_WGRAD=3 DBX_FOLD_MIN_ELEMS=0 \
  DBX_FOLD_MIN_ELEMS=0+DBX_FOLD_MAX_RATIO=8 DBX_NSHARD=8 DBX_FAST=0 DBX_FAST_STAGE=32 DBX_FAST_MAT=0 DBX_TAP_PRUNE=0 base
