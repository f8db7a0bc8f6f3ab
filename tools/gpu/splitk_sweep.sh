#!/bin/bash
# split-K policy sweep (splitk_wgs / splitk_min_kb) on the small presets, interleaved rounds
set -o pipefail
O=${1:-gpurun_out/splitk_sweep}; R=${2:-2}
mkdir -p $O
for r in $(seq 1 $R); do
  bash tools/gpu/sweep_env.sh $O/r$r "resnet50_tiny_imagenet resnet18_cifar10" DBX_ENGINE=splitk_wgs=0 \
    DBX_ENGINE=splitk_wgs=256 DBX_ENGINE=splitk_wgs=384 DBX_ENGINE=splitk_wgs=512 DBX_ENGINE=splitk_wgs=768 \
    DBX_ENGINE=splitk_wgs=512,splitk_min_kb=2 DBX_ENGINE=splitk_wgs=512,splitk_min_kb=8 || exit 1
done
