#!/bin/bash
# A/B of conv tile choices inside one box: heuristic vs tuned table (fwd only / both).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for m in none fwd fwd,dgrad none fwd,dgrad; do
DBX_TUNE_MODES=$m timeout -k 10 300 python bench.py --steps 20 --warmup 5 --batch 1024 > gpurun_out/ab_$m.log 2>&1 || { echo "bench $m FAILED"; tail -20 gpurun_out/ab_$m.log; exit 1; }
echo "$m: $(tail -1 gpurun_out/ab_$m.log | cut -c90-160)"
done
