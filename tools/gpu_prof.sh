#!/bin/bash
# Kernel-level profile of the native bench step (eager launches so every kernel is traced).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
B=${1:-1024}
cd /tmp && DBX_GRAPHS=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_b$B -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 2 --batch $B > $GRAFT_REPO_ROOT/gpurun_out/prof_b$B.log 2>&1; echo "prof rc=$?"
find $GRAFT_REPO_ROOT/gpurun_out/prof_b$B -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $GRAFT_REPO_ROOT/gpurun_out/kstats_b$B.csv
