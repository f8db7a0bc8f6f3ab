#!/bin/bash
# Kernel stats of the small presets on the current tree (13 steps: 3 warm-up + 10 timed).
set -o pipefail
O=${1:-gpurun_out/r4_s17}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for p in resnet50_tiny_imagenet resnet18_cifar10; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/rp_$p -o run --output-format csv -- python3 bench.py --preset $p --steps 10 --warmup 3 \
    > $O/rp_$p.log 2>&1 || { tail -20 $O/rp_$p.log; exit 1; }
  f=$(find $O/rp_$p -name "*kernel_stats.csv" | head -1)
  python3 tools/prof_top.py $f 13 45 > $O/top_$p.txt
  head -3 $O/top_$p.txt
done
