#!/bin/bash
# Round 4: launch-count levers on the small presets -- fewer BN-statistics shards (so the consumer
# side / in-launch finalize reads less), the consumer-side forward finalize and the in-launch finalize.
set -o pipefail
O=${1:-gpurun_out/r4_small}
export TMPDIR=/tmp
bash tools/gpu/sweep_env.sh $O "resnet18_cifar10 resnet50_tiny_imagenet" base DBX_NSHARD=4 \
  DBX_NSHARD=4+DBX_FIN_IN=1 DBX_NSHARD=4+DBX_FUSE_BN_FIN=1 DBX_NSHARD=8+DBX_FIN_IN=1 DBX_FIN_IN=1 base
