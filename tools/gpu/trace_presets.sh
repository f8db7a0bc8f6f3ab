#!/bin/bash
# kernel traces (rocpd) of the small presets with the current defaults, for tools/step_timeline.py / queue_report.py
set -o pipefail
O=${1:-gpurun_out/trace_presets}
mkdir -p $O
export TMPDIR=/tmp
for p in resnet50_tiny_imagenet resnet18_cifar10; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/rp_$p -o run -- python3 bench.py --preset $p --steps 8 --warmup 4 > $O/$p.log 2>&1 || { tail -20 $O/$p.log; exit 1; }
done
