#!/bin/bash
# Fold the BN-backward apply into 1x1 dgrads only up to an N / K ratio (DBX_FOLD_MAX_RATIO):
# bottleneck conv1 dgrads (N = 4K) re-read and re-apply their operand once per N tile.
set -o pipefail
mkdir -p gpurun_out/r2s3
for r in 1 2; do
  for v in inf 2 1; do
    export DBX_FOLD_MAX_RATIO=$v
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2s3/fold_$v.log 2>&1 || { echo "bench $v FAILED"; tail -20 gpurun_out/r2s3/fold_$v.log; exit 1; }
    echo "fold_max_ratio=$v: $(tail -1 gpurun_out/r2s3/fold_$v.log | cut -c95-150)"
  done
done
for v in 2 1; do
  export DBX_FOLD_MAX_RATIO=$v
  timeout -k 10 300 python bench.py --preset resnet50_tiny_imagenet --steps 20 --warmup 5 > gpurun_out/r2s3/fold_t$v.log 2>&1 && echo "tiny fold_max_ratio=$v: $(tail -1 gpurun_out/r2s3/fold_t$v.log | cut -c95-150)"
done
unset DBX_FOLD_MAX_RATIO
timeout -k 10 300 python bench.py --preset resnet50_tiny_imagenet --steps 20 --warmup 5 > gpurun_out/r2s3/fold_tinf.log 2>&1 && echo "tiny fold_max_ratio=inf: $(tail -1 gpurun_out/r2s3/fold_tinf.log | cut -c95-150)"
