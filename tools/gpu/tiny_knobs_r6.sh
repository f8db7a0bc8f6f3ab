#!/bin/bash
# TinyImageNet knob re-check after the round-6 changes (interleaved rounds; "default" repeated).
set -o pipefail
O=${1:-gpurun_out/tiny_knobs}; R=${2:-2}; mkdir -p $O; export TMPDIR=/tmp
V=("" "coeff_in=0" "nshard=8" "coeff_in_maxc=0" "coeff_in_maxc=256" "side_defer=0" "lazy_join=0" "stem_wg_main=0" "tail_main=1" "tail_main=4" "dwf_cus=0" "side_cu_reserve=96" "side_cu_reserve=160" "defer_reduce=1" "fold_min_elems=4194304" "splitk_min_kb=2" "splitk_min_kb=8")
for r in $(seq 1 $R); do
  for v in "${V[@]}"; do
    n=${v//[,=]/_}; n=${n:-default}
    DBX_ENGINE=$v timeout -k 10 300 python bench.py --preset resnet50_tiny_imagenet --steps 20 --warmup 5 > $O/b_${n}_$r.log 2>&1 || { echo "FAIL $v"; tail -5 $O/b_${n}_$r.log; continue; }
    echo "tiny ${v:-default} r$r: $(grep -o '"value": [0-9.]*' $O/b_${n}_$r.log)" | tee -a $O/ab.txt
  done
done
