#!/bin/bash
# Stem weight gradient as one 64 x 256 tile per workgroup: tests, end-to-end A/B (DBX_STEM_WGRAD), op breakdown.
set -o pipefail
O=gpurun_out/r2s4_stem2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_stem_bwd_gpu.py tests/test_kernels_gpu.py -x -q -k "stem" --timeout 120 --timeout-method thread > $O/test.log 2>&1 || { echo "stem tests FAILED"; tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
for r in 1 2; do
  for f in tile generic; do
    DBX_STEM_WGRAD=$f timeout -k 10 300 python bench.py --steps 30 --warmup 10 > $O/bench_${f}_r$r.log 2>&1 || { echo "bench FAILED"; tail -20 $O/bench_${f}_r$r.log; exit 1; }
    echo "stem wgrad=$f run $r: $(tail -1 $O/bench_${f}_r$r.log | cut -c80-130)"
  done
done
timeout -k 10 300 python tools/op_breakdown.py > $O/op_breakdown_b1024.txt 2>&1 || { echo "op_breakdown FAILED"; tail -20 $O/op_breakdown_b1024.txt; exit 1; }
grep -E "wall|stem|pool|wgrad 4->64" $O/op_breakdown_b1024.txt | head -12
