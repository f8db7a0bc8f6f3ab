#!/bin/bash
# The committed table + the ResNet-50 b256 entries: headline and ZeRO-1 preset vs the previous table
# (git's copy shipped as gpurun_out-free file tools/tune_table_prev.json), alternating, same box.
set -o pipefail
O=gpurun_out/r2s5_tablecheck
mkdir -p $O
for r in 1 2; do
  for t in prev cur; do
    if [ $t = prev ]; then export DBX_TUNE_TABLE=tools/tune_table_prev.json; else unset DBX_TUNE_TABLE; fi
    timeout -k 10 300 python bench.py --steps 30 --warmup 10 > $O/b_head_${t}_$r.log 2>&1 || { echo "bench FAILED"; tail -20 $O/b_head_${t}_$r.log; exit 1; }
    timeout -k 10 300 python bench.py --preset resnet50_imagenet_zero1 --steps 20 --warmup 5 > $O/b_zero1_${t}_$r.log 2>&1 || { echo "bench FAILED"; tail -20 $O/b_zero1_${t}_$r.log; exit 1; }
    echo "$t run $r: headline $(tail -1 $O/b_head_${t}_$r.log | cut -c90-110) zero1 $(tail -1 $O/b_zero1_${t}_$r.log | cut -c90-110)"
  done
done
