#!/bin/bash
# dgrad sweep with a different side-stream CU reservation (side_cu_reserve) -- does the faster
# main-chain dgrad pay once the side stream carries less?  usage: sweep_rebalance_ab.sh OUT ROUNDS
set -o pipefail
O=${1:-gpurun_out/sweep_cu}; R=${2:-2}; mkdir -p $O; export TMPDIR=/tmp
for r in $(seq 1 $R); do
  for v in "sweep_dgrad=0" "sweep_dgrad=1" "sweep_dgrad=1,side_cu_reserve=64" "sweep_dgrad=1,side_cu_reserve=192" "sweep_dgrad=0,side_cu_reserve=64"; do
    n=${v//[,=]/_}
    DBX_ENGINE=$v timeout -k 10 300 python bench.py --steps 15 --warmup 5 > $O/bench_${n}_$r.log 2>&1 || { tail -20 $O/bench_${n}_$r.log; exit 1; }
    echo "headline $v r$r: $(grep -o '"value": [0-9.]*' $O/bench_${n}_$r.log)" | tee -a $O/ab.txt
  done
done
