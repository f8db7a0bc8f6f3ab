#!/bin/bash
# TinyImageNet consumer-side finalize default (now off for the class) vs on; CIFAR unchanged check.
set -o pipefail
O=${1:-gpurun_out/tiny_fin}; R=${2:-3}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_program_gpu.py tests/test_bn_fin_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc = 0 ] || { grep -E "FAILED|Error" $O/pytest.log | head -20; exit $rc; }
for r in $(seq 1 $R); do
  for v in "" "fin_in=1"; do
    n=${v//[,=]/_}; n=${n:-default}
    DBX_ENGINE=$v timeout -k 10 300 python bench.py --preset resnet50_tiny_imagenet --steps 20 --warmup 5 > $O/b_${n}_$r.log 2>&1 || { tail -20 $O/b_${n}_$r.log; exit 1; }
    echo "tiny ${v:-default} r$r: $(grep -o '"value": [0-9.]*' $O/b_${n}_$r.log)" | tee -a $O/ab.txt
  done
done
timeout -k 10 300 python bench.py --preset resnet18_cifar10 --steps 20 --warmup 5 > $O/cifar.log 2>&1 && echo "cifar default: $(grep -o '"value": [0-9.]*' $O/cifar.log)" | tee -a $O/ab.txt
