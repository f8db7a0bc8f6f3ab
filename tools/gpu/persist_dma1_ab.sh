#!/bin/bash
# DBX_PERSIST_DMA1 threshold A/B: 8 (default: persistent only with >= 8 tiles per workgroup), 1 (always), 0 (never)
set -o pipefail
O=${1:-gpurun_out/persist_dma1b}
mkdir -p $O
for r in 1 2 3; do
  bash tools/gpu/sweep_env.sh $O/r$r "headline resnet50_tiny_imagenet" base DBX_PERSIST_DMA1=1 DBX_PERSIST_DMA1=0 || exit 1
done
