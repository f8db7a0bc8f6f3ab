#!/bin/bash
# kernel numerics + conv microbench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu > gpurun_out/test_kernels.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -30 gpurun_out/test_kernels.log
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 400 python tools/bench_conv.py --batch 256 --out gpurun_out/conv_bench.md > gpurun_out/conv_bench.log 2>&1
  echo "bench rc=$?"
  tail -5 gpurun_out/conv_bench.log
fi
