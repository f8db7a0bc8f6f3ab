#!/bin/bash
# side-stream schedule switches on the ZeRO-1 AdamW b256 preset (1.05 TFLOP of forward conv work)
set -o pipefail
O=${1:-gpurun_out/zero1_sweep}
for r in 1 2; do
  bash tools/gpu/sweep_env.sh $O/r$r "resnet50_imagenet_zero1" base DBX_SIDE_DEFER=1 DBX_STEM_WG_MAIN=1 DBX_SIDE_DEFER=1+DBX_STEM_WG_MAIN=1 DBX_SIDE_DEFER=1+DBX_TAIL_MAIN=2 || exit 1
done
