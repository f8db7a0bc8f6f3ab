#!/bin/bash
# Fused conv3 backward (conv_dwfused.hip): numerics tests, end-to-end A/B (DBX_FUSE_DW), kernel stats.
set -o pipefail
O=gpurun_out/r2s4_dwf
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_dwfused_gpu.py -x -v --timeout 120 --timeout-method thread > $O/test.log 2>&1 || { echo "dwfused tests FAILED"; tail -40 $O/test.log; exit 1; }
tail -3 $O/test.log
for r in 1 2; do
  for f in 1 0; do
    DBX_FUSE_DW=$f timeout -k 10 300 python bench.py --steps 30 --warmup 10 > $O/bench_f${f}_r$r.log 2>&1 || { echo "bench FAILED"; tail -20 $O/bench_f${f}_r$r.log; exit 1; }
    echo "fuse=$f run $r: $(tail -1 $O/bench_f${f}_r$r.log | cut -c60-150)"
  done
done
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 2 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1; echo "prof rc=$?"
