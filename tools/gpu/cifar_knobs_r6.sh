#!/bin/bash
# CIFAR ResNet-18 knob re-check after the round-6 changes (interleaved rounds; "default" repeated).
set -o pipefail
O=${1:-gpurun_out/cifar_knobs}; R=${2:-2}; mkdir -p $O; export TMPDIR=/tmp
V=("" "fin_in=0" "coeff_in=0" "nshard=8" "splitk_min_kb=16" "splitk_wgs=1024" "splitk_wgs=256" "defer_reduce=0" "tail_main=1" "stem_wg_main=0" "side_cu_reserve=64" "lazy_join=0" "fold_min_elems=0" "block_tail_main=1" "block_tail_main=3")
for r in $(seq 1 $R); do
  for v in "${V[@]}"; do
    n=${v//[,=.]/_}; n=${n:-default}
    DBX_ENGINE=$v timeout -k 10 300 python bench.py --preset resnet18_cifar10 --steps 30 --warmup 5 > $O/b_${n}_$r.log 2>&1 || { echo "FAIL $v"; continue; }
    echo "cifar ${v:-default} r$r: $(grep -o '"value": [0-9.]*' $O/b_${n}_$r.log)" | tee -a $O/ab.txt
  done
done
