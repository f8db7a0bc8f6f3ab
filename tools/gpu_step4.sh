#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/test_gpu.log 2>&1; echo "gpu tests rc=$?"; tail -4 gpurun_out/test_gpu.log
for b in 256 512 1024; do
timeout -k 10 300 python bench.py --steps 15 --warmup 4 --batch $b > gpurun_out/bench_native_b$b.log 2>&1; echo "bench b$b rc=$?"; tail -1 gpurun_out/bench_native_b$b.log | cut -c1-200
done
timeout -k 10 400 python bench.py --impl torch --steps 10 --warmup 4 --batch 1024 > gpurun_out/bench_torch_b1024.log 2>&1; echo "torch b1024 rc=$?"; tail -1 gpurun_out/bench_torch_b1024.log | cut -c1-200
cd /tmp && DBX_GRAPHS=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_native -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof_native.log 2>&1; echo "prof rc=$?"
