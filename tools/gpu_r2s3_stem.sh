#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r2s3
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_conv_patch3_gpu.py tests/test_kernels_gpu.py -k "stem or patch" > gpurun_out/r2s3/t_stem.log 2>&1 || { echo "tests FAILED"; tail -30 gpurun_out/r2s3/t_stem.log; exit 1; }
tail -1 gpurun_out/r2s3/t_stem.log
for r in 1 2; do
  for v in 0 1; do
    DBX_STEM_PATCH=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2s3/stem_$v.log 2>&1 || { echo "bench $v FAILED"; tail -20 gpurun_out/r2s3/stem_$v.log; exit 1; }
    echo "stem_patch=$v: $(tail -1 gpurun_out/r2s3/stem_$v.log | cut -c80-140)"
  done
done
timeout -k 10 300 python tools/op_breakdown.py --steps 3 --top 90 > gpurun_out/r2s3/op_breakdown2.txt 2>&1 && grep -E "stem|wall" gpurun_out/r2s3/op_breakdown2.txt
