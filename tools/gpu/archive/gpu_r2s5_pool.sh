#!/bin/bash
# Specialised 3x3/s2 max-pool forward: kernel tests, then same-box A/B (DBX_MAXPOOL_GENERIC=1 = old kernel)
# on the per-op breakdown and alternating benches.
set -o pipefail
O=gpurun_out/r2s5_pool
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_stem_bwd_gpu.py -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1 || { echo "tests FAILED"; tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
for v in 0 1; do
  if [ $v = 1 ]; then export DBX_MAXPOOL_GENERIC=1; else unset DBX_MAXPOOL_GENERIC; fi
  timeout -k 10 300 python tools/op_breakdown.py > $O/op_breakdown_generic$v.txt 2>&1 || { echo "op_breakdown FAILED"; tail -5 $O/op_breakdown_generic$v.txt; exit 1; }
  echo "generic=$v: $(grep -E '^  maxpool_fwd|^batch' $O/op_breakdown_generic$v.txt | tr '\n' ' ')"
done
for r in 1 2; do
  for v in 0 1; do
    if [ $v = 1 ]; then export DBX_MAXPOOL_GENERIC=1; else unset DBX_MAXPOOL_GENERIC; fi
    timeout -k 10 300 python bench.py --steps 30 --warmup 10 > $O/bench_g${v}_$r.log 2>&1 || { echo "bench FAILED"; tail -20 $O/bench_g${v}_$r.log; exit 1; }
    echo "generic=$v run $r: $(tail -1 $O/bench_g${v}_$r.log | cut -c90-125)"
  done
done
