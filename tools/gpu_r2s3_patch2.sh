#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r2s3
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_conv_patch3_gpu.py tests/test_conv_dma_gpu.py > gpurun_out/r2s3/t_patch2.log 2>&1 || { echo "tests FAILED"; tail -30 gpurun_out/r2s3/t_patch2.log; exit 1; }
tail -1 gpurun_out/r2s3/t_patch2.log
for c in "fwd3x3_64 128,64,1" "fwd3x3_64 patch" "dgrad3x3_64 256,64,2" "dgrad3x3_64 patch"; do
  set -- $c
  timeout -k 10 60 python tools/conv_probe.py --case $1 --tile $2 --iters 9
done
