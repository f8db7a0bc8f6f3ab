#!/bin/bash
# Headline config with LARS (native) + its rocprofv3 kernel stats; ZeRO-3 autograd throughput vs DDP autograd.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --optim lars > gpurun_out/bench_lars.log 2>&1 || { echo "lars bench FAILED"; tail -20 gpurun_out/bench_lars.log; exit 1; }
tail -1 gpurun_out/bench_lars.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_lars -o run -- python bench.py --steps 5 --warmup 3 --optim lars > gpurun_out/prof_lars.log 2>&1 || { echo "prof FAILED"; tail -20 gpurun_out/prof_lars.log; exit 1; }
find gpurun_out/prof_lars -name "*kernel_stats.csv" | head -1 | xargs grep -i "lars\|sgd" | cut -c1-160
timeout -k 10 400 python tools/zero3_bench.py > gpurun_out/zero3_bench.log 2>&1 || { echo "zero3 bench FAILED"; tail -20 gpurun_out/zero3_bench.log; exit 1; }
cat gpurun_out/zero3_bench.log | grep -v amdgpu.ids
