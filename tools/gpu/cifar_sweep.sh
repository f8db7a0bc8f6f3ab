#!/bin/bash
# CIFAR schedule knobs with the deferred launch + lazy joins
set -o pipefail
O=${1:-gpurun_out/cifar_sweep}
for r in 1 2; do
  bash tools/gpu/sweep_env.sh $O/r$r "resnet18_cifar10" base DBX_TAIL_MAIN=1 DBX_TAIL_MAIN=2 DBX_STEM_WG_MAIN=0 DBX_DEFER_REDUCE=0 DBX_FIN_IN=0 || exit 1
done
