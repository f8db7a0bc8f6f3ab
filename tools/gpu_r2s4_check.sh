#!/bin/bash
# After the fused conv3 backward: tests, headline + preset A/B (DBX_FUSE_DW), op breakdown, kernel stats.
set -o pipefail
O=gpurun_out/r2s4_check
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_dwfused_gpu.py -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1 || { echo "dwfused tests FAILED"; tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
for r in 1 2; do
  for f in 1 0; do
    DBX_FUSE_DW=$f timeout -k 10 300 python bench.py --steps 30 --warmup 10 > $O/bench_f${f}_r$r.log 2>&1 || { echo "bench FAILED"; tail -20 $O/bench_f${f}_r$r.log; exit 1; }
    echo "headline fuse=$f run $r: $(tail -1 $O/bench_f${f}_r$r.log | cut -c80-130)"
  done
done
for p in resnet50_imagenet_zero1 resnet50_tiny_imagenet; do
  for f in 1 0; do
    DBX_FUSE_DW=$f timeout -k 10 300 python bench.py --preset $p --steps 20 --warmup 5 > $O/bench_${p}_f$f.log 2>&1 || { echo "bench $p FAILED"; tail -20 $O/bench_${p}_f$f.log; exit 1; }
    echo "$p fuse=$f: $(tail -1 $O/bench_${p}_f$f.log | cut -c80-130)"
  done
done
timeout -k 10 300 python tools/op_breakdown.py > $O/op_breakdown_b1024.txt 2>&1 || { echo "op_breakdown FAILED"; tail -20 $O/op_breakdown_b1024.txt; exit 1; }
head -22 $O/op_breakdown_b1024.txt
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 2 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1; echo "prof rc=$?"
