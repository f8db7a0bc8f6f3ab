#!/bin/bash
# Middle side-stream batches' tails on the main stream (DBX_SEG_TAIL_MAIN): bit-identity, then
# interleaved sweeps on TinyImageNet (the preset whose main stream waits at the joins) and the others.
set -o pipefail
O=${1:-gpurun_out/segtail_ab}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_program_gpu.py -k "side_stream_bit_identical" > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || exit 1
for r in 1 2; do
  bash tools/gpu/sweep_env.sh $O/r$r "resnet50_tiny_imagenet" base DBX_SEG_TAIL_MAIN=1 DBX_SEG_TAIL_MAIN=2 DBX_SEG_TAIL_MAIN=3 DBX_SEG_TAIL_MAIN=4 DBX_SEG_TAIL_MAIN=6 || exit 1
  bash tools/gpu/sweep_env.sh $O/r$r "resnet18_cifar10 headline" base DBX_SEG_TAIL_MAIN=1 DBX_SEG_TAIL_MAIN=2 || exit 1
done
