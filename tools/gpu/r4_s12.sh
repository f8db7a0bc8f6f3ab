#!/bin/bash
# Round 4: batched split-K reduce v2 (block-uniform job lookup): replay determinism (the test runs
# three trainers, twice), then the presets with / without it.
set -o pipefail
O=${1:-gpurun_out/r4_s12}
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 400 python -u -m pytest tests/test_wgrad_batch_gpu.py -x -q --timeout 300 --timeout-method thread \
    > $O/pytest_$r.log 2>&1
  rc=$?; tail -2 $O/pytest_$r.log; [ $rc = 0 ] || { grep -E "FAILED|Error|assert" $O/pytest_$r.log | head -20; exit $rc; }
done
bash tools/gpu/sweep_env.sh $O "resnet18_cifar10 resnet50_tiny_imagenet" base DBX_DEFER_REDUCE=1 base DBX_DEFER_REDUCE=1
