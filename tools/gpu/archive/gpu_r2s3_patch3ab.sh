#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r2s3
for r in 1 2; do
  for v in 0 fwd all; do
    DBX_PATCH3=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2s3/patchab_$v.log 2>&1 || { echo "bench $v FAILED"; tail -20 gpurun_out/r2s3/patchab_$v.log; exit 1; }
    echo "patch3=$v: $(tail -1 gpurun_out/r2s3/patchab_$v.log | cut -c80-140)"
  done
done
