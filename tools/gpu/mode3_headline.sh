#!/bin/bash
# per-block side forks (DBX_OVERLAP_WGRAD=3) on the headline / TinyImageNet, with the deferred launch and lazy joins
set -o pipefail
O=${1:-gpurun_out/mode3}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_program_gpu.py -k "side_stream_bit_identical and 3" > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || exit 1
for r in 1 2; do
  bash tools/gpu/sweep_env.sh $O/r$r "headline" base DBX_OVERLAP_WGRAD=3+DBX_SIDE_DEFER=1 DBX_OVERLAP_WGRAD=3+DBX_SIDE_DEFER=1+DBX_LAZY_JOIN=1 || exit 1
  bash tools/gpu/sweep_env.sh $O/r$r "resnet50_tiny_imagenet" base DBX_OVERLAP_WGRAD=3+DBX_LAZY_JOIN=1 || exit 1
done
