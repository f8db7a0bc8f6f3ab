#!/bin/bash
# layer1's weight gradients forked per block, with the deferred side launch (headline)
set -o pipefail
O=${1:-gpurun_out/l1blocks_defer}
for r in 1 2; do
  bash tools/gpu/sweep_env.sh $O/r$r "headline" base DBX_SIDE_DEFER=1 DBX_SIDE_DEFER=1+DBX_LAST_SEG_BLOCKS=1 DBX_SIDE_DEFER=1+DBX_LAST_SEG_BLOCKS=1+DBX_STEM_WG_MAIN=1 DBX_LAST_SEG_BLOCKS=1 || exit 1
done
