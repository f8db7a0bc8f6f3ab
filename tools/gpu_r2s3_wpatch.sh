#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r2s3
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_conv_patch3_gpu.py > gpurun_out/r2s3/t_wpatch.log 2>&1 || { echo "tests FAILED"; tail -30 gpurun_out/r2s3/t_wpatch.log; exit 1; }
tail -1 gpurun_out/r2s3/t_wpatch.log
for r in 1 2; do
  for v in "fwd,dgrad" all; do
    DBX_PATCH3=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2s3/wpatch.log 2>&1 || { echo "bench $v FAILED"; tail -20 gpurun_out/r2s3/wpatch.log; exit 1; }
    echo "patch3=$v: $(tail -1 gpurun_out/r2s3/wpatch.log | cut -c80-140)"
  done
done
timeout -k 10 300 python tools/op_breakdown.py --steps 3 --top 90 > gpurun_out/r2s3/op_breakdown3.txt 2>&1 && grep -E "wgrad 64->64 3x3|wall" gpurun_out/r2s3/op_breakdown3.txt
