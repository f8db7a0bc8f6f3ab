#!/bin/bash
# per-block default: the stem weight gradient on the main stream or behind layer1's side batches
set -o pipefail
O=${1:-gpurun_out/m3_stem}
for r in 1 2; do
  bash tools/gpu/sweep_env.sh $O/r$r "headline resnet50_tiny_imagenet" base DBX_STEM_WG_MAIN=1 DBX_STEM_WG_MAIN=0 || exit 1
done
