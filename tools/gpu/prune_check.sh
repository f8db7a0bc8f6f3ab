#!/bin/bash
# tap pruning: conv kernel numerics incl. the small-map cases, end-to-end program tests, then the
# small-shape presets with and without pruning (DBX_TAP_PRUNE)
set -o pipefail
O=${1:-gpurun_out/prune}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_program_gpu.py -x -q --timeout 200 --timeout-method thread -k "conv or program or grads or trains" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc = 0 ] || { grep -E "FAILED|Error" $O/pytest.log | head -20; exit $rc; }
tools/gpu/sweep_env.sh $O/ab "resnet18_cifar10 resnet50_tiny_imagenet" base DBX_TAP_PRUNE=0 base DBX_TAP_PRUNE=0
