#!/bin/bash
# Split-K head GEMM (DBX_HEAD_SPLITK): kernel numerics, the engine tests that run the head, the
# Composer layout-contract check (warnings listed with -rw), then interleaved A/B on the presets.
set -o pipefail
O=${1:-gpurun_out/headsplit}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -rw --timeout 300 --timeout-method thread tests/test_head_gpu.py \
  tests/test_program_gpu.py -k "split_k or small_gemm or side_stream_bit_identical or composer or cutmix" > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; grep -i "layout" $O/pytest.log | head -5; [ $rc = 0 ] || exit 1
bash tools/gpu/ab_env.sh $O/ab DBX_HEAD_SPLITK "resnet50_tiny_imagenet resnet18_cifar10 headline" 2
