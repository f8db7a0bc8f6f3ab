#!/bin/bash
# Round 4: the backward consumer-side finalize on TinyImageNet (3 interleaved rounds).
set -o pipefail
O=${1:-gpurun_out/r4_s11}
export TMPDIR=/tmp
bash tools/gpu/sweep_env.sh $O "resnet50_tiny_imagenet" base DBX_COEFF_IN=1 base DBX_COEFF_IN=1 base DBX_COEFF_IN=1
