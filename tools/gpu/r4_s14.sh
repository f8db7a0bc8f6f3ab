#!/bin/bash
# Round 4: adaptive grid cap of the finalizing apply passes: COEFF_IN on TinyImageNet, CIFAR check.
set -o pipefail
O=${1:-gpurun_out/r4_s14}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_bn_fin_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
bash tools/gpu/sweep_env.sh $O "resnet50_tiny_imagenet" base DBX_COEFF_IN=1 base DBX_COEFF_IN=1
bash tools/gpu/sweep_env.sh $O "resnet18_cifar10" base base
