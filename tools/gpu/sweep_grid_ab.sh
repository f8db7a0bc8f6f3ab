#!/bin/bash
# dgrad N-sweep grid A/B inside the step (the side stream's weight gradients run beside it).
# usage: sweep_grid_ab.sh OUT ROUNDS
set -o pipefail
O=${1:-gpurun_out/sweep_grid}; R=${2:-2}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_sweep_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc = 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
for r in $(seq 1 $R); do
  for v in "sweep_dgrad=0" "sweep_dgrad_wgs=0" "sweep_dgrad_wgs=-1" "sweep_dgrad_wgs=192" "sweep_dgrad_wgs=128"; do
    for p in headline; do
      args="--steps 15 --warmup 5"; [ $p != headline ] && args="$args --preset $p"
      n=${v//[,=-]/_}
      DBX_ENGINE=$v timeout -k 10 300 python bench.py $args > $O/bench_${p}_${n}_$r.log 2>&1 || { tail -20 $O/bench_${p}_${n}_$r.log; exit 1; }
      echo "$p $v r$r: $(grep -o '"value": [0-9.]*' $O/bench_${p}_${n}_$r.log)" | tee -a $O/ab.txt
    done
  done
done
