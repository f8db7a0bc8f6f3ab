#!/bin/bash
# ZeRO-1 b256 preset: split-K slice depth and a few step knobs (interleaved rounds)
set -o pipefail
O=${1:-gpurun_out/zero_knobs}; R=${2:-3}; mkdir -p $O; export TMPDIR=/tmp
V=("" "splitk_min_kb=4" "splitk_wgs=0" "side_cu_reserve=96" "sweep_min_tiles_per_cu=2")
for r in $(seq 1 $R); do
  for v in "${V[@]}"; do
    n=${v//[,=.]/_}; n=${n:-default}
    DBX_ENGINE=$v timeout -k 10 300 python bench.py --preset resnet50_imagenet_zero1 --steps 20 --warmup 5 > $O/b_${n}_$r.log 2>&1 || { echo "FAIL $v"; continue; }
    echo "zero1 ${v:-default} r$r: $(grep -o '"value": [0-9.]*' $O/b_${n}_$r.log)" | tee -a $O/ab.txt
  done
done
