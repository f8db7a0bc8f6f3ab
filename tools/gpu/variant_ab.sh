#!/bin/bash
# kernel-variant A/B: the fused conv3 backward microbench, then interleaved headline benches per
# variant build (DBX_EXT_VARIANT; "base" = the production _C).  usage: variant_ab.sh OUT ROUNDS v1 v2 ...
set -o pipefail
O=$1; R=$2; shift 2
mkdir -p $O
for v in base "$@"; do
  ev=""; [ $v != base ] && ev="DBX_EXT_VARIANT=$v"
  env $ev timeout -k 10 200 python tools/bench_dwfused.py > $O/dwf_$v.log 2>&1 || { tail -20 $O/dwf_$v.log; exit 1; }
  echo "== $v"; grep -v amdgpu.ids $O/dwf_$v.log | tail -6
done
for r in $(seq 1 $R); do
  for v in base "$@"; do
    ev=""; [ $v != base ] && ev="DBX_EXT_VARIANT=$v"
    env $ev timeout -k 10 300 python bench.py --steps 15 --warmup 5 > $O/bench_${v}_$r.log 2>&1 || { tail -20 $O/bench_${v}_$r.log; exit 1; }
    echo "headline $v r$r: $(grep -o '"value": [0-9.]*' $O/bench_${v}_$r.log)"
  done
done
