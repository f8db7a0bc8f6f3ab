#!/bin/bash
# the backward BN-coefficient launches on the headline (starved beside the side-stream weight gradients:
# 4.9 us alone, 26.5 us in the overlapped step): consumer-side / producer-side finalize
set -o pipefail
O=${1:-gpurun_out/coeff_sweep}
for r in 1 2; do
  bash tools/gpu/sweep_env.sh $O/r$r "headline" base DBX_COEFF_IN=1 DBX_FUSE_BN_FIN=1 DBX_COEFF_IN=1+DBX_FUSE_BN_FIN=1 || exit 1
done
