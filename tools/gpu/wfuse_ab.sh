#!/bin/bash
# in-launch weight-gradient split-K reduce size limit (wgrad_fuse_max) re-check on the three presets
set -o pipefail
O=${1:-gpurun_out/wfuse}; R=${2:-2}; mkdir -p $O; export TMPDIR=/tmp
for r in $(seq 1 $R); do
  for p in resnet50_tiny_imagenet resnet18_cifar10 headline; do
    for v in "" "wgrad_fuse_max=0" "wgrad_fuse_max=4194304"; do
      n=${v//[,=]/_}; n=${n:-default}
      args="--steps 20 --warmup 5"; [ $p != headline ] && args="$args --preset $p"
      DBX_ENGINE=$v timeout -k 10 300 python bench.py $args > $O/b_${p}_${n}_$r.log 2>&1 || { echo "FAIL $p $v"; continue; }
      echo "$p ${v:-default} r$r: $(grep -o '"value": [0-9.]*' $O/b_${p}_${n}_$r.log)" | tee -a $O/ab.txt
    done
  done
done
