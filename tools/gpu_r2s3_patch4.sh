#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r2s3
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_conv_patch3_gpu.py > gpurun_out/r2s3/t_patch4.log 2>&1 || { echo "tests FAILED"; tail -30 gpurun_out/r2s3/t_patch4.log; exit 1; }
tail -1 gpurun_out/r2s3/t_patch4.log
for c in "fwd3x3_64 128,64,1" "fwd3x3_64 patch_r" "fwd3x3_64 patch_s" "dgrad3x3_64 256,64,2" "dgrad3x3_64 patch_r" "dgrad3x3_64 patch_s"; do
  set -- $c
  timeout -k 10 60 python tools/conv_probe.py --case $1 --tile $2 --iters 9
done
for r in 1 2; do
  for v in fwd all; do
    DBX_PATCH3=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2s3/patch4_$v.log 2>&1 || { echo "bench $v FAILED"; tail -20 gpurun_out/r2s3/patch4_$v.log; exit 1; }
    echo "patch3=$v: $(tail -1 gpurun_out/r2s3/patch4_$v.log | cut -c80-140)"
  done
done
