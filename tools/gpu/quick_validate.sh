#!/bin/bash
# Quick validation on one GPU: the GPU suite, smoke, the preset bench lines (no profile). quick_validate.sh [OUT]
set -o pipefail
O=${1:-gpurun_out/quick_validate}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc = 0 ] || { grep -E "FAILED|Error" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
for p in headline resnet50_tiny_imagenet resnet18_cifar10 resnet50_imagenet_zero1 headline; do
  args="--steps 20 --warmup 5"; [ $p != headline ] && args="$args --preset $p"
  timeout -k 10 300 python bench.py $args > $O/bench_$p.log 2>&1 || { tail -20 $O/bench_$p.log; exit 1; }
  grep '"metric"' $O/bench_$p.log >> $O/bench_lines.txt
  echo "$p: $(grep -o '"value": [0-9.]*' $O/bench_$p.log)"
done
