#!/bin/bash
# head kernels (small_gemm / colsum) numerics, then the frozen-backbone configs (head-heavy steps) and
# the CIFAR preset
set -o pipefail
O=${1:-gpurun_out/head}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_head_gpu.py tests/test_program_gpu.py -k "colsum or gemm or frozen or head or cutmix" -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc = 0 ] || { grep -E "FAILED|Error" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 400 python tools/bench_frozen.py --steps 30 --warmup 5 --configs r18_cifar,r50_tiny > $O/frozen.log 2>&1 || { tail -20 $O/frozen.log; exit 1; }
tail -8 $O/frozen.log
timeout -k 10 300 python bench.py --preset resnet18_cifar10 --steps 30 --warmup 10 > $O/bench_cifar.log 2>&1 || { tail -20 $O/bench_cifar.log; exit 1; }
echo "resnet18_cifar10: $(grep -o '"value": [0-9.]*' $O/bench_cifar.log)"
