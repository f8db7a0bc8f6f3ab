#!/bin/bash
# layer1's weight gradients forked per block (DBX_LAST_SEG_BLOCKS): bit-identity, then interleaved A/B
set -o pipefail
O=${1:-gpurun_out/l1blocks}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_program_gpu.py -k "side_stream_bit_identical" > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || exit 1
for r in 1 2; do
  bash tools/gpu/sweep_env.sh $O/r$r "headline resnet50_tiny_imagenet resnet18_cifar10" base DBX_LAST_SEG_BLOCKS=1 || exit 1
done
