#!/bin/bash
# Quick iteration: kernel numerics (optionally a -k filter), per-op breakdown, headline bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
K=${1:-}
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_program_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread ${K:+-k "$K"} > gpurun_out/test_quick.log 2>&1 || { echo "tests FAILED"; tail -40 gpurun_out/test_quick.log; exit 1; }
tail -1 gpurun_out/test_quick.log
timeout -k 10 300 python tools/op_breakdown.py --top 70 > gpurun_out/op_breakdown.txt 2>&1 || { echo "breakdown FAILED"; tail -20 gpurun_out/op_breakdown.txt; exit 1; }
head -20 gpurun_out/op_breakdown.txt
timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/bench.log 2>&1 || { echo "bench FAILED"; tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-260
