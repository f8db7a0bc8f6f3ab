#!/bin/bash
# A/B the headline bench over tune tables (tools/tune_tables/*.json), interleaved rounds.
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for t in tools/tune_tables/*.json; do
    n=$(basename $t .json)
    DBX_TUNE_TABLE=$t timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/ab_$n.log 2>&1 || { echo "bench $n FAILED"; tail -20 gpurun_out/ab_$n.log; exit 1; }
    echo "round $r $n: $(tail -1 gpurun_out/ab_$n.log | cut -c90-140)"
  done
done
