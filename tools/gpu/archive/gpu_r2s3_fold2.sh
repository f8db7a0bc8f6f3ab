#!/bin/bash
# fold the ratio-4 conv1 BN-backward applies only at the 56x56 stage (DBX_FOLD_RATIO_MIN_HW=56) vs never
set -o pipefail
mkdir -p gpurun_out/r2s3
for r in 1 2; do
  for v in 100000 56 28; do
    DBX_FOLD_RATIO_MIN_HW=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2s3/fold2.log 2>&1 || { echo "bench $v FAILED"; tail -20 gpurun_out/r2s3/fold2.log; exit 1; }
    echo "fold_ratio_min_hw=$v: $(tail -1 gpurun_out/r2s3/fold2.log | cut -c80-140)"
  done
done
