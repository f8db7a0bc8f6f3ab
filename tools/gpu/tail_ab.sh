#!/bin/bash
# The exposed end of the step: the stem weight gradient on the main stream (DBX_STEM_WG_MAIN) and the
# last side-stream batch's tail moved to the main stream (DBX_TAIL_MAIN): bit-identity first, then
# interleaved sweeps of the three presets.
set -o pipefail
O=${1:-gpurun_out/tail_ab}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_program_gpu.py -k "side_stream_bit_identical" > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || exit 1
for r in 1 2; do
  bash tools/gpu/sweep_env.sh $O/r$r "headline" DBX_STEM_WG_MAIN=0 base DBX_TAIL_MAIN=1 DBX_TAIL_MAIN=2 DBX_TAIL_MAIN=3 DBX_TAIL_MAIN=4 || exit 1
  bash tools/gpu/sweep_env.sh $O/r$r "resnet50_tiny_imagenet resnet18_cifar10" DBX_STEM_WG_MAIN=0 base DBX_TAIL_MAIN=1 DBX_TAIL_MAIN=2 || exit 1
done
