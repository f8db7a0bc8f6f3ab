#!/bin/bash
# Round 4: deferred split-K weight-gradient reductions (two launches per side-stream batch):
# bit-exactness, then the presets with / without it (and the headline with it forced on).
set -o pipefail
O=${1:-gpurun_out/r4_s10}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_wgrad_batch_gpu.py tests/test_bn_fin_gpu.py -x -q --timeout 200 \
  --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc = 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
bash tools/gpu/sweep_env.sh $O "resnet18_cifar10 resnet50_tiny_imagenet" base DBX_DEFER_REDUCE=0 base DBX_DEFER_REDUCE=0
bash tools/gpu/sweep_env.sh $O "headline" base DBX_DEFER_REDUCE=1 base
