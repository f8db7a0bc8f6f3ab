#!/bin/bash
# N-sweep forward: GPU tests, per-launch probe against the igemm tile, interleaved bench A/B.
# usage: sweep_ab.sh OUT ROUNDS
set -o pipefail
O=${1:-gpurun_out/sweep}; R=${2:-2}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_sweep_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
timeout -k 10 300 python -u tools/probe_sweep.py --sweep > $O/probe.txt 2>&1 || { tail -20 $O/probe.txt; exit 1; }
grep -v amdgpu $O/probe.txt
for r in $(seq 1 $R); do
  for v in "sweep_fwd=1,sweep_dgrad=1" "sweep_fwd=1,sweep_dgrad=0" "sweep_fwd=0,sweep_dgrad=0"; do
    for p in headline resnet50_imagenet_zero1 resnet50_tiny_imagenet; do
      args="--steps 15 --warmup 5"; [ $p != headline ] && args="$args --preset $p"
      DBX_ENGINE=$v timeout -k 10 300 python bench.py $args > $O/bench_${p}_${v//[,=]/_}_$r.log 2>&1 || { tail -20 $O/bench_${p}_${v//[,=]/_}_$r.log; exit 1; }
      echo "$p $v r$r: $(grep -o '"value": [0-9.]*' $O/bench_${p}_${v//[,=]/_}_$r.log)" | tee -a $O/ab.txt
    done
  done
done
