#!/bin/bash
# A/B of deeper LDS-DMA rings: the 256x256 weight gradient in a 5-slot ring of 32-pixel stages
# (DBX_WGRAD_RING5) and the eight-wave conv kernel in 4 / 5 slots of 32-channel stages
# (DBX_FAST_STAGE=32, DBX_FAST_SLOTS=5): numerics first, then two interleaved headline sweeps.
set -o pipefail
O=${1:-gpurun_out/ring_ab}
mkdir -p $O
DBX_WGRAD_RING5=1 DBX_FAST_STAGE=32 DBX_FAST_SLOTS=5 timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_conv_dma_gpu.py tests/test_conv_fast_gpu.py > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || exit 1
bash tools/gpu/sweep_env.sh $O/s1 "headline" base DBX_WGRAD_RING5=1 DBX_FAST_STAGE=32 DBX_FAST_STAGE=32+DBX_FAST_SLOTS=5 DBX_WGRAD_RING5=1+DBX_FAST_STAGE=32+DBX_FAST_SLOTS=5 && \
bash tools/gpu/sweep_env.sh $O/s2 "headline" base DBX_WGRAD_RING5=1 DBX_FAST_STAGE=32 DBX_FAST_STAGE=32+DBX_FAST_SLOTS=5 DBX_WGRAD_RING5=1+DBX_FAST_STAGE=32+DBX_FAST_SLOTS=5
