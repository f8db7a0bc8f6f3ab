#!/bin/bash
# Persistent tiles on the weights-by-DMA (DMA 1) BN-prologue forward convs: kernel numerics, the
# program's bit-identity / training tests, then an interleaved A/B (DBX_PERSIST_DMA1) on the presets.
set -o pipefail
O=${1:-gpurun_out/persist_dma1}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
  -k "persistent or conv_fwd" > $O/pytest_kernels.log 2>&1; rc=$?; tail -2 $O/pytest_kernels.log; [ $rc = 0 ] || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_program_gpu.py \
  -k "matches_autograd or side_stream_bit_identical or loss_decreases or graph or composer" > $O/pytest_program.log 2>&1; rc=$?; tail -2 $O/pytest_program.log; [ $rc = 0 ] || exit 1
bash tools/gpu/ab_env.sh $O/ab DBX_PERSIST_DMA1 "headline resnet50_tiny_imagenet resnet18_cifar10" 2
