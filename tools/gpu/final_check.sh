#!/bin/bash
# Round validation: full GPU test suite, smoke, headline bench, every BASELINE preset, and the MDS-fed
# TinyImageNet step (zstd shards -> C++ reader -> pinned ring -> native step) against synthetic data.
set -o pipefail
O=${1:-gpurun_out/final}
mkdir -p $O
tools/gpu/check.sh $O || exit $?
for p in resnet18_cifar10 resnet50_tiny_imagenet; do
  timeout -k 10 300 python bench.py --preset $p --steps 30 --warmup 10 > $O/bench_$p.log 2>&1 || { tail -20 $O/bench_$p.log; exit 1; }
  echo "$p: $(grep -o '"value": [0-9.]*' $O/bench_$p.log)"
done
timeout -k 10 600 python bench.py --preset resnet50_tiny_imagenet --data mds --steps 30 --warmup 10 > $O/bench_tiny_mds.log 2>&1 || { tail -20 $O/bench_tiny_mds.log; exit 1; }
echo "resnet50_tiny_imagenet --data mds: $(grep -o '"value": [0-9.]*' $O/bench_tiny_mds.log)"
grep -o '"data": "[^"]*"' $O/bench_tiny_mds.log | cut -c1-300
