#!/bin/bash
# confirmation of the TinyImageNet knob candidates, and their effect on CIFAR (interleaved rounds)
set -o pipefail
O=${1:-gpurun_out/tiny_conf}; R=${2:-3}; mkdir -p $O; export TMPDIR=/tmp
V=("" "splitk_min_kb=8" "splitk_min_kb=8,coeff_in_maxc=256" "splitk_min_kb=8,coeff_in_maxc=256,tail_main=4")
for r in $(seq 1 $R); do
  for p in resnet50_tiny_imagenet resnet18_cifar10; do
    for v in "${V[@]}"; do
      n=${v//[,=]/_}; n=${n:-default}
      DBX_ENGINE=$v timeout -k 10 300 python bench.py --preset $p --steps 20 --warmup 5 > $O/b_${p}_${n}_$r.log 2>&1 || { echo "FAIL $v"; continue; }
      echo "$p ${v:-default} r$r: $(grep -o '"value": [0-9.]*' $O/b_${p}_${n}_$r.log)" | tee -a $O/ab.txt
    done
  done
done
