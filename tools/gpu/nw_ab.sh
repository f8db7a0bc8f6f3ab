#!/bin/bash
# A/B of a conv_fast wave-count variant build (build_ext --variant V -D DBX_FAST_NW=4): the eight-wave
# kernel microbenchmark under both builds, the fast-kernel GPU tests under the variant, then interleaved
# preset benches.  nw_ab.sh OUT VARIANT "presets" ROUNDS
set -o pipefail
O=${1:-gpurun_out/nw_ab}; V=${2:-nw4}; P=${3:-"headline resnet50_tiny_imagenet"}; R=${4:-2}
mkdir -p $O; export TMPDIR=/tmp
for v in base $V; do
  e="DBX_EXT_VARIANT="; [ $v != base ] && e="DBX_EXT_VARIANT=$v"
  env $e timeout -k 10 300 python -u tools/bench_fast.py --rounds 3 --iters 5 > $O/bench_fast_$v.txt 2>&1 || { tail -20 $O/bench_fast_$v.txt; exit 1; }
  echo "== bench_fast $v"; grep -v amdgpu.ids $O/bench_fast_$v.txt | tail -16
done
DBX_EXT_VARIANT=$V timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv_fast_gpu.py \
  > $O/pytest_$V.txt 2>&1; rc=$?; tail -2 $O/pytest_$V.txt; [ $rc = 0 ] || exit $rc
bash tools/gpu/ab_variant_presets.sh $O $V "$P" $R
