#!/bin/bash
# Same-box A/B: default build vs _C_variant_pfold (-DDBX_PF_OLD: next tile's B issued after the
# epilogue, branchy epilogue stores, no count-matching stores). Stats probe + alternating benches.
set -o pipefail
O=gpurun_out/r2s5_pfab
mkdir -p $O
for r in 1 2; do
  for v in "" pfold; do
    DBX_EXT_VARIANT=$v timeout -k 10 300 python tools/probe_stats.py > $O/probe_${v}_$r.txt 2>&1 || { echo "probe FAILED"; tail -5 $O/probe_${v}_$r.txt; exit 1; }
    echo "variant='$v' run $r"; grep -v amdgpu.ids $O/probe_${v}_$r.txt | head -4
  done
done
for r in 1 2 3; do
  for v in "" pfold; do
    DBX_EXT_VARIANT=$v timeout -k 10 300 python bench.py --steps 30 --warmup 10 > $O/bench_${v}_$r.log 2>&1 || { echo "bench FAILED"; tail -20 $O/bench_${v}_$r.log; exit 1; }
    echo "variant='$v' run $r: $(tail -1 $O/bench_${v}_$r.log | cut -c90-125)"
  done
done
