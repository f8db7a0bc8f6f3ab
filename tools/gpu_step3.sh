#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/test_gpu.log 2>&1; echo "gpu tests rc=$?"; tail -15 gpurun_out/test_gpu.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_native.log 2>&1; echo "bench rc=$?"; tail -1 gpurun_out/bench_native.log
cd /tmp && DBX_GRAPHS=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_native -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof_native.log 2>&1; echo "prof rc=$?"
