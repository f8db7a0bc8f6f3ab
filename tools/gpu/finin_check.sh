#!/bin/bash
set -o pipefail
O=${1:-gpurun_out/finin}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_bn_fin_gpu.py tests/test_program_gpu.py tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc = 0 ] || { grep -E "FAILED|Error" $O/pytest.log | head -20; exit $rc; }
tools/gpu/sweep_env.sh $O/ab "resnet18_cifar10 resnet50_tiny_imagenet" base DBX_FIN_IN=0 DBX_FIN_IN=1 base DBX_FIN_IN=0
