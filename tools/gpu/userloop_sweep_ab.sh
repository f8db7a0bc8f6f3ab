#!/bin/bash
# native_module (user-loop) throughput with and without the sweep forward.
set -o pipefail
O=${1:-gpurun_out/userloop_sweep}; mkdir -p $O; export TMPDIR=/tmp
for r in 1 2; do
  for v in 1 0; do
    DBX_ENGINE=sweep_fwd=$v timeout -k 10 500 python tools/bench_native_module.py --impls native > $O/nm_${v}_$r.log 2>&1 || { tail -20 $O/nm_${v}_$r.log; exit 1; }
    grep '^{' $O/nm_${v}_$r.log | sed "s/^/sweep_fwd=$v r$r /" | tee -a $O/ab.txt
  done
done
