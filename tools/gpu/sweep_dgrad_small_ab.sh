#!/bin/bash
# dgrad sweep at the round-6 admission threshold on the small / ZeRO presets (interleaved rounds)
set -o pipefail
O=${1:-gpurun_out/sdg_small}; R=${2:-3}; mkdir -p $O; export TMPDIR=/tmp
for r in $(seq 1 $R); do
  for p in resnet50_tiny_imagenet resnet50_imagenet_zero1; do
    for v in "" "sweep_dgrad=1"; do
      n=${v//[,=]/_}; n=${n:-default}
      DBX_ENGINE=$v timeout -k 10 300 python bench.py --preset $p --steps 20 --warmup 5 > $O/b_${p}_${n}_$r.log 2>&1 || { echo "FAIL $p $v"; continue; }
      echo "$p ${v:-default} r$r: $(grep -o '"value": [0-9.]*' $O/b_${p}_${n}_$r.log)" | tee -a $O/ab.txt
    done
  done
done
