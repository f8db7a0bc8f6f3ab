#!/bin/bash
# One iteration: kernel numerics, optional conv breakdown, bench at batch 1024 (and 256).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu > gpurun_out/test_kernels.log 2>&1 || { echo "kernel tests FAILED"; tail -30 gpurun_out/test_kernels.log; exit 1; }
tail -1 gpurun_out/test_kernels.log
if [ "$1" == "bd" ]; then
timeout -k 10 400 python tools/conv_breakdown.py > gpurun_out/breakdown.log 2>&1 || { echo "breakdown FAILED"; tail -20 gpurun_out/breakdown.log; exit 1; }
fi
for b in 1024 256; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --batch $b > gpurun_out/bench_b$b.log 2>&1 || { echo "bench FAILED"; tail -20 gpurun_out/bench_b$b.log; exit 1; }
echo "b$b: $(tail -1 gpurun_out/bench_b$b.log | cut -c90-200)"
done
