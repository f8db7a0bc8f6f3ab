#!/bin/bash
# TinyImageNet: consumer-side BN finalize (fin_in) against deeper split-K (every split workgroup
# finalizes the input BN itself).  usage: tiny_fin_splitk_ab.sh OUT ROUNDS
set -o pipefail
O=${1:-gpurun_out/tiny_fs}; R=${2:-2}; mkdir -p $O; export TMPDIR=/tmp
for r in $(seq 1 $R); do
  for v in "splitk_wgs=512" "fin_in=0" "splitk_wgs=1024" "fin_in=0,splitk_wgs=1024" "fin_in=0,coeff_in=0,splitk_wgs=1024"; do
    n=${v//[,=]/_}
    DBX_ENGINE=$v timeout -k 10 300 python bench.py --preset resnet50_tiny_imagenet --steps 20 --warmup 5 > $O/b_${n}_$r.log 2>&1 || { tail -20 $O/b_${n}_$r.log; exit 1; }
    echo "tiny $v r$r: $(grep -o '"value": [0-9.]*' $O/b_${n}_$r.log)" | tee -a $O/ab.txt
  done
done
