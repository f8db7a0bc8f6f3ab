#!/bin/bash
# Round 4: bn_apply with the in-launch forward finalize (BasicBlock outputs on small steps):
# bit-exactness, then the small presets against the previous step.
set -o pipefail
O=${1:-gpurun_out/r4_s8}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_bn_fin_gpu.py -x -q --timeout 200 --timeout-method thread \
  > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc = 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
bash tools/gpu/sweep_env.sh $O "resnet18_cifar10 resnet50_tiny_imagenet" base DBX_FIN_IN=0 base
