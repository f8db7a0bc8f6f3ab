#!/bin/bash
# Per-op times of the TinyImageNet step (eager, no side stream) under split-K settings (DBX_ENGINE),
# to see which shapes gain / lose from splitting.  usage: splitk_ops.sh OUT
set -o pipefail
O=${1:-gpurun_out/splitk_ops}; mkdir -p $O; export TMPDIR=/tmp
for cfg in splitk_wgs=512 splitk_wgs=0 splitk_wgs=1024 "splitk_wgs=1024,splitk_min_kb=8" "splitk_wgs=2048,splitk_min_kb=16"; do
  n=$(echo $cfg | tr ',=' '__')
  DBX_ENGINE="$cfg" SIZE=64 CLASSES=200 BATCH=512 timeout -k 10 300 python tools/op_breakdown.py --steps 5 --top 80 > $O/ops_$n.txt 2>&1 || { tail -20 $O/ops_$n.txt; exit 1; }
  echo "== $cfg: $(head -1 $O/ops_$n.txt)"
done
