#!/bin/bash
# user-loop (native_module) and frozen-backbone workloads, refreshed on the current tree
set -o pipefail
O=${1:-gpurun_out/userloop}
mkdir -p $O
timeout -k 10 600 python tools/bench_native_module.py > $O/native_module.log 2>&1 || { tail -20 $O/native_module.log; exit 1; }
grep '^{' $O/native_module.log
timeout -k 10 600 python tools/bench_frozen.py > $O/frozen.log 2>&1 || { tail -20 $O/frozen.log; exit 1; }
grep '^{' $O/frozen.log
