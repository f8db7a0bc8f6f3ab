#!/bin/bash
# 4-slot 32-channel weight ring of the sweep forward (DBX_SWEEP_RING4): tests, probe on both builds, presets.
# usage: defer_ab.sh OUT ROUNDS   (base = production _C, noring4 = -D DBX_SWEEP_RING4=0)
set -o pipefail
O=${1:-gpurun_out/ring4}; R=${2:-2}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_sweep_gpu.py tests/test_program_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc = 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
for v in base noring4; do
  ev=""; [ $v != base ] && ev="DBX_EXT_VARIANT=$v"
  env $ev timeout -k 10 300 python -u tools/probe_sweep.py --sweep > $O/probe_$v.txt 2>&1 || { tail -20 $O/probe_$v.txt; exit 1; }
  echo "== $v"; grep "^fwd" $O/probe_$v.txt
done
for r in $(seq 1 $R); do
  for v in base noring4; do
    ev=""; [ $v != base ] && ev="DBX_EXT_VARIANT=$v"
    for p in headline resnet50_imagenet_zero1 resnet50_tiny_imagenet; do
      args="--steps 15 --warmup 5"; [ $p != headline ] && args="$args --preset $p"
      env $ev timeout -k 10 300 python bench.py $args > $O/bench_${p}_${v}_$r.log 2>&1 || { tail -20 $O/bench_${p}_${v}_$r.log; exit 1; }
      echo "$p $v r$r: $(grep -o '"value": [0-9.]*' $O/bench_${p}_${v}_$r.log)" | tee -a $O/ab.txt
    done
  done
done
