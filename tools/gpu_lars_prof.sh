#!/bin/bash
# rocprofv3 kernel stats of the native LARS step (csv).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_lars -o run -- python bench.py --steps 5 --warmup 3 --optim lars > gpurun_out/prof_lars.log 2>&1 || { echo "prof FAILED"; tail -20 gpurun_out/prof_lars.log; exit 1; }
f=$(find gpurun_out/prof_lars -name "*kernel_stats.csv" | head -1)
head -1 "$f"
grep -i "lars\|sgd" "$f" | cut -c1-200
