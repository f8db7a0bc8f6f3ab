#!/bin/bash
# the 3x3 patch weight gradient (64->64 @56, layer1) capped to all but the reserved CUs (default) vs all CUs
set -o pipefail
O=${1:-gpurun_out/patch3_reserve}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_patch3_gpu.py > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || exit 1
for r in 1 2 3; do
  bash tools/gpu/sweep_env.sh $O/r$r "headline" base DBX_PATCH3_RESERVE=0 || exit 1
done
