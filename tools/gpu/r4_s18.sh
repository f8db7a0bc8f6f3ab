#!/bin/bash
# Consumer-side BN-backward coefficients limited to narrow BNs (DBX_COEFF_IN_MAXC) on TinyImageNet / CIFAR.
set -o pipefail
O=${1:-gpurun_out/r4_s18}
bash tools/gpu/sweep_env.sh $O "resnet50_tiny_imagenet" base DBX_COEFF_IN=1 DBX_COEFF_IN=1+DBX_COEFF_IN_MAXC=1024 \
  DBX_COEFF_IN=1+DBX_COEFF_IN_MAXC=512 DBX_COEFF_IN=1+DBX_COEFF_IN_MAXC=256 base DBX_COEFF_IN=1+DBX_COEFF_IN_MAXC=512 DBX_COEFF_IN=1+DBX_COEFF_IN_MAXC=256 \
  && bash tools/gpu/sweep_env.sh $O "resnet18_cifar10" base DBX_COEFF_IN_MAXC=256 DBX_COEFF_IN_MAXC=128 base DBX_COEFF_IN_MAXC=256
