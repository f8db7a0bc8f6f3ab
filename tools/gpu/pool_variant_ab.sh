#!/bin/bash
# pool_bn_bwd with out-of-range buffer loads for the absent candidate windows (variant "pool") vs the production build
set -o pipefail
O=${1:-gpurun_out/pool_ab}
mkdir -p $O
DBX_EXT_VARIANT=pool timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "pool" > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || exit 1
for v in base pool base pool; do
  ev=""; [ $v != base ] && ev="DBX_EXT_VARIANT=$v"
  env $ev timeout -k 10 120 python tools/bench_pool_bwd.py 2>&1 | grep -v amdgpu.ids | sed "s/^/$v: /"
done
for r in 1 2 3; do
  for v in base pool; do
    ev=""; [ $v != base ] && ev="DBX_EXT_VARIANT=$v"
    env $ev timeout -k 10 300 python bench.py --steps 15 --warmup 5 > $O/bench_${v}_$r.log 2>&1 || { tail -20 $O/bench_${v}_$r.log; exit 1; }
    echo "headline $v r$r: $(grep -o '"value": [0-9.]*' $O/bench_${v}_$r.log)"
  done
done
