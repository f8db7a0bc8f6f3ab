#!/bin/bash
# forward sweep admission threshold (128-row blocks per CU) on the presets with few-block maps.
# usage: sweep_thresh_ab.sh OUT ROUNDS
set -o pipefail
O=${1:-gpurun_out/sweep_th}; R=${2:-2}; mkdir -p $O; export TMPDIR=/tmp
for r in $(seq 1 $R); do
  for v in "sweep_min_tiles_per_cu=4" "sweep_min_tiles_per_cu=1" "sweep_min_tiles_per_cu=0.25"; do
    for p in resnet50_tiny_imagenet resnet50_imagenet_zero1; do
      n=${v//[,=.]/_}
      DBX_ENGINE=$v timeout -k 10 300 python bench.py --preset $p --steps 20 --warmup 5 > $O/bench_${p}_${n}_$r.log 2>&1 || { tail -20 $O/bench_${p}_${n}_$r.log; exit 1; }
      echo "$p $v r$r: $(grep -o '"value": [0-9.]*' $O/bench_${p}_${n}_$r.log)" | tee -a $O/ab.txt
    done
  done
done
